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


def infer_device_map(model: nn.Module, devices, max_memory: dict | None = None, no_split=DEFAULT_NO_SPLIT,
                     linear_weight_bytes: int | None = None):
    devices = [torch.device(d) for d in devices]
    units = placement_units(model, no_split)
    sizes = [_bytes(m, linear_weight_bytes if n != "lm_head" else None) for n, m in units]
    total = sum(sizes) or 1
    n = len(devices)
    dmap = OrderedDict()
    d, used, cum = 0, [0] * n, 0
    for (name, _), sz in zip(units, sizes):
        cap = None if max_memory is None else max_memory.get(str(devices[d]), max_memory.get(d))
        # next device once this one holds its balanced share (or its cap), never going backwards
        while d < n - 1 and (cum >= total * (d + 1) / n or (cap is not None and used[d] + sz > cap)):
            d += 1
            cap = None if max_memory is None else max_memory.get(str(devices[d]), max_memory.get(d))
        if cap is not None and used[d] + sz > cap:
            raise RuntimeError(f"model does not fit: unit {name!r} ({sz} B) exceeds {devices[d]}'s budget")
        dmap[name] = str(devices[d])
        used[d] += sz
        cum += sz
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
