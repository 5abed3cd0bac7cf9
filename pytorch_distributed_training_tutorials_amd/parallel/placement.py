"""Layer-wise model placement across GPUs for big-model inference.

Reference: ``LlamaForCausalLM.from_pretrained(..., device_map="auto")`` NB03:52-56
(SURVEY R24, M14): accelerate splits a 32-layer Llama-7B over 4 GPUs in layer
order (embed + layers 0-5 -> cuda:0, 6-13 -> cuda:1, 14-21 -> cuda:2, 22-31 +
norm + lm_head -> cuda:3, NB03:114-404) and hooks each block to move its
inputs to its device.

Here:
  * :func:`infer_device_map` -- balanced, order-preserving assignment of
    "placement units" (top-level blocks; ``no_split`` classes such as decoder
    layers are never split) to devices by parameter+buffer bytes, optionally
    capped per device (``max_memory``); with 288 GB of HBM per MI355X a 7B
    model fits on ONE GPU, so ``devices`` is normally chosen for throughput
    rather than capacity;
  * :func:`dispatch_model` -- moves each unit and installs a forward pre-hook
    that moves tensor args/kwargs to the unit's device (peer copies over xGMI);
  * :func:`placement_report` -- the reference's ``(index, name, device, dtype)``
    listing of every parameter.
"""
from __future__ import annotations

from collections import OrderedDict

import torch
import torch.nn as nn

DEFAULT_NO_SPLIT = ("LlamaDecoderLayer", "MistralDecoderLayer", "Bottleneck", "BasicBlock")


def _bytes(m: nn.Module, linear_weight_bytes: int | None = None) -> int:
    """Parameter + buffer bytes; ``linear_weight_bytes`` prices nn.Linear weights as if
    quantised (1 = int8) so placement can be planned before quantising (e.g. on meta)."""
    tot = 0
    for mod in m.modules():
        for name, p in mod.named_parameters(recurse=False):
            esz = linear_weight_bytes if (linear_weight_bytes and isinstance(mod, nn.Linear) and name == "weight"
                                          and not getattr(mod, "_ptdt_keep_fp", False)) else p.element_size()
            tot += p.numel() * esz
        tot += sum(b.numel() * b.element_size() for b in mod.buffers(recurse=False))
    return tot


def placement_units(model: nn.Module, no_split=DEFAULT_NO_SPLIT):
    """Ordered (name, module) units: recurse into containers, stop at no-split
    classes and at modules that own parameters directly."""
    out = []

    def visit(name, mod):
        children = list(mod.named_children())
        own = list(mod.named_parameters(recurse=False)) + list(mod.named_buffers(recurse=False))
        if type(mod).__name__ in no_split or not children or own:
            out.append((name, mod))
            return
        for cn, ch in children:
            visit(f"{name}.{cn}" if name else cn, ch)

    visit("", model)
    return out


HBM_BYTES = 288 * 2 ** 30  # one MI355X: the default per-device capacity when planning off-GPU (meta / CPU)


def _device_bytes(dev: torch.device) -> int:
    if dev.type == "cuda" and torch.cuda.is_available() and (dev.index or 0) < torch.cuda.device_count():
        return int(torch.cuda.get_device_properties(dev.index or 0).total_memory)
    return HBM_BYTES


def _is_layer(mod: nn.Module, no_split) -> bool:
    """A placement 'layer': a module that is never split (no children, or a no-split class)."""
    return not list(mod.children()) or type(mod).__name__ in no_split


def balanced_budgets(model: nn.Module, devices, max_memory: dict | None = None, no_split=DEFAULT_NO_SPLIT,
                     linear_weight_bytes: int | None = None, reserve_frac: float | None = None) -> list[int]:
    """Per-device byte budgets of the ``device_map="auto"`` ("balanced") policy the reference's
    ``from_pretrained`` ran (NB03:52-56, accelerate's balanced-memory planning):

      * every device but the last gets ``total / n`` plus a slack of 1.25 x max(first no-split block,
        mean leaf-module size), so no device ends up a layer short; the last keeps its whole capacity;
      * a quantised load keeps ``reserve_frac`` of every budget free for the int8 kernels' scratch
        (10 % under LLM.int8 sizing, ``linear_weight_bytes=1``).
    """
    devices = [torch.device(d) for d in devices]
    cap = []
    for i, d in enumerate(devices):
        v = None if max_memory is None else max_memory.get(str(d), max_memory.get(i))
        cap.append(int(v) if v is not None else _device_bytes(d))
    units = placement_units(model, no_split)
    sizes = [_bytes(m, linear_weight_bytes if n != "lm_head" else None) for n, m in units]
    total = sum(sizes)
    first_block = {}  # first unit of each no-split class
    for (_, m), s in zip(units, sizes):
        first_block.setdefault(type(m).__name__, s) if type(m).__name__ in no_split else None
    block = max(first_block.values(), default=0)
    # leaf modules holding tensors, priced like their units (an lm_head stays unquantised)
    leaves = []
    for name, m in model.named_modules():
        if not list(m.children()) and (any(True for _ in m.parameters(recurse=False))
                                       or any(True for _ in m.buffers(recurse=False))):
            leaves.append(_bytes(m, linear_weight_bytes if name != "lm_head" else None))
    mean_leaf = int(sum(leaves) / max(len(leaves), 1))
    per = total // len(devices) + int(1.25 * max(block, mean_leaf))
    budgets = [min(per, c) for c in cap[:-1]] + [cap[-1]]
    if reserve_frac is None:
        reserve_frac = 0.1 if linear_weight_bytes == 1 else 0.0
    return [int(b * (1.0 - reserve_frac)) for b in budgets]


def infer_device_map(model: nn.Module, devices, max_memory: dict | None = None, no_split=DEFAULT_NO_SPLIT,
                     linear_weight_bytes: int | None = None, balanced: bool = True,
                     reserve_frac: float | None = None):
    """Order-preserving unit -> device map (reference ``device_map="auto"``, NB03:52-56).

    Units (``placement_units``) are filled into the devices in order against per-device budgets
    (``balanced_budgets``; ``balanced=False``: the raw capacities / ``max_memory``). The first device
    keeps room for the largest layer still to place (the slot an offloaded layer would be staged
    through), which is why it ends up with fewer decoder layers. For the reference's int8
    Llama-7B over 4 devices this reproduces the recorded split exactly: embed + layers 0-5 ->
    cuda:0 (parameter idx 0-54), 6-13 -> cuda:1 (55-126), 14-21 -> cuda:2 (127-198), 22-31 + norm +
    lm_head -> cuda:3 (199-290), NB03:114-404."""
    devices = [torch.device(d) for d in devices]
    if balanced:
        budgets = balanced_budgets(model, devices, max_memory, no_split, linear_weight_bytes, reserve_frac)
    else:
        budgets = [int(max_memory.get(str(d), max_memory.get(i))) if max_memory is not None else _device_bytes(d)
                   for i, d in enumerate(devices)]
    units = placement_units(model, no_split)
    sizes = [_bytes(m, linear_weight_bytes if n != "lm_head" else None) for n, m in units]
    layer_sizes = [s if _is_layer(m, no_split) else 0 for (_, m), s in zip(units, sizes)]
    dmap = OrderedDict()
    d, used = 0, [0] * len(devices)
    for k, ((name, _), sz) in enumerate(zip(units, sizes)):
        while True:
            room = budgets[d]
            if d == 0:  # main device: keep the largest remaining layer's worth free
                room -= max(layer_sizes[k:], default=0)
            if used[d] + sz <= room or d == len(devices) - 1:
                break
            d += 1
        if used[d] + sz > budgets[d]:
            raise RuntimeError(f"model does not fit: unit {name!r} ({sz} B) exceeds {devices[d]}'s budget")
        dmap[name] = str(devices[d])
        used[d] += sz
    return dmap


def _move(obj, dev):
    if isinstance(obj, torch.Tensor):
        return obj.to(dev, non_blocking=True) if obj.device != dev else obj
    if isinstance(obj, tuple):
        return tuple(_move(o, dev) for o in obj)
    if isinstance(obj, list):
        return [_move(o, dev) for o in obj]
    if isinstance(obj, dict):
        return {k: _move(v, dev) for k, v in obj.items()}
    return obj


def dispatch_model(model: nn.Module, device_map: dict) -> nn.Module:
    mods = dict(model.named_modules())
    model._ptdt_hooks = []
    for name, dev in device_map.items():
        m = mods[name] if name else model
        d = torch.device(dev)
        m.to(d)

        def pre_hook(mod, args, kwargs, _d=d):
            return _move(args, _d), _move(kwargs, _d)

        model._ptdt_hooks.append(m.register_forward_pre_hook(pre_hook, with_kwargs=True))
    model.hf_device_map = dict(device_map)
    return model


def placement_report(model: nn.Module):
    """[(index, name, device, dtype)] for every parameter (reference NB03:409-410)."""
    return [(i, n, str(p.device), str(p.dtype)) for i, (n, p) in enumerate(model.named_parameters())] + \
        [(None, n, str(b.device), str(b.dtype)) for n, b in model.named_buffers() if b.dtype == torch.int8]
