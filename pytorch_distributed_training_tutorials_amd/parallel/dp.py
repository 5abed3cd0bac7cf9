"""Single-process multi-GPU replica data parallelism (``nn.DataParallel`` surface).

Reference: ``model = nn.DataParallel(model)`` NB01:275-277 and its step
NB01:478-487: every forward re-broadcasts the
parameters from device 0, scatters the batch along dim 0, runs one replica per
device in a Python thread, gathers the outputs on device 0; backward scatters
the output gradient, runs the replicas' backward, and reduces the replica
gradients onto device 0.

MI355X implementation:
  * the parameter broadcast is coalesced into ONE flat buffer per dtype and
    moved with a single grouped RCCL broadcast over xGMI (an ``RcclClique``
    built with ``ncclCommInitAll`` for the device set) instead of per-tensor
    copies; the backward reduction is the mirror grouped ``ncclReduce`` onto
    the source device (replaces ``torch.cuda.nccl.reduce`` /
    ``ReduceAddCoalesced``);
  * input scatter / output gather are peer copies (``hipMemcpyPeerAsync``)
    issued non-blocking;
  * each replica thread binds its device explicitly (no "no current CUDA
    context" warning, quirk Q12).
Devices may repeat or be ``cpu`` (plumbing tests); then copies replace RCCL.
"""
from __future__ import annotations

import threading

import torch
import torch.nn as nn

from .._ext import has_native, native


def _dev(d) -> torch.device:
    if isinstance(d, int):
        return torch.device("cuda", d)
    return torch.device(d)


def _flatten(ts):
    return torch.cat([t.reshape(-1) for t in ts]) if ts else None


def _unflatten(flat, like):
    out, off = [], 0
    for t in like:
        n = t.numel()
        out.append(flat[off:off + n].view_as(t))
        off += n
    return out


class _Clique:
    """Grouped RCCL broadcast/reduce over distinct GPUs (None when not applicable)."""

    _cache: dict = {}

    @classmethod
    def get(cls, devices):
        if len(devices) < 2 or any(d.type != "cuda" for d in devices) or not has_native():
            return None
        ids = tuple(d.index for d in devices)
        if len(set(ids)) != len(ids):
            return None
        if ids not in cls._cache:
            cls._cache[ids] = native().RcclClique(list(ids))
        return cls._cache[ids]


class _Broadcast(torch.autograd.Function):
    """Coalesced parameter broadcast src -> devices; backward = reduce onto src."""

    @staticmethod
    def forward(ctx, devices, *tensors):
        ctx.devices = devices
        ctx.src = tensors[0].device if tensors else devices[0]
        ctx.n = len(tensors)
        groups = {}
        for i, t in enumerate(tensors):
            groups.setdefault(t.dtype, []).append(i)
        outs = [[None] * len(tensors) for _ in devices]
        clique = _Clique.get(devices)
        for dt, idxs in groups.items():
            ts = [tensors[i] for i in idxs]
            flat = _flatten(ts)
            if clique is not None:
                flats = [flat if d == ctx.src else torch.empty_like(flat, device=d) for d in devices]
                clique.broadcast(flats, devices.index(ctx.src))
            else:
                flats = [flat if d == ctx.src else flat.to(d, non_blocking=True) for d in devices]
            for j, f in enumerate(flats):
                for i, v in zip(idxs, _unflatten(f, ts)):
                    outs[j][i] = v
        return tuple(t for per_dev in outs for t in per_dev)

    @staticmethod
    def backward(ctx, *grads):
        n, devices = ctx.n, ctx.devices
        per_dev = [list(grads[j * n:(j + 1) * n]) for j in range(len(devices))]
        result = [None] * n
        clique = _Clique.get(devices)
        for i in range(n):
            if all(per_dev[j][i] is None for j in range(len(devices))):
                continue
            for j, d in enumerate(devices):
                if per_dev[j][i] is None:
                    ref = next(per_dev[k][i] for k in range(len(devices)) if per_dev[k][i] is not None)
                    per_dev[j][i] = torch.zeros(ref.shape, dtype=ref.dtype, device=d)
        live = [i for i in range(n) if per_dev[0][i] is not None]
        groups = {}
        for i in live:
            groups.setdefault(per_dev[0][i].dtype, []).append(i)
        root = devices.index(ctx.src)
        for dt, idxs in groups.items():
            flats = [_flatten([per_dev[j][i].contiguous() for i in idxs]) for j in range(len(devices))]
            if clique is not None:
                clique.reduce(flats, root)
                total = flats[root]
            else:
                total = flats[root].clone()
                for j, f in enumerate(flats):
                    if j != root:
                        total.add_(f.to(ctx.src, non_blocking=True))
            for i, v in zip(idxs, _unflatten(total, [per_dev[0][i] for i in idxs])):
                result[i] = v
        return (None, *result)


class _Scatter(torch.autograd.Function):
    @staticmethod
    def forward(ctx, devices, dim, x):
        ctx.dim, ctx.src = dim, x.device
        chunks = x.chunk(len(devices), dim)
        ctx.sizes = [c.size(dim) for c in chunks]
        return tuple(c.to(d, non_blocking=True).contiguous() if c.device != d else c.contiguous()
                     for c, d in zip(chunks, devices[:len(chunks)]))

    @staticmethod
    def backward(ctx, *grads):
        return None, None, torch.cat([g.to(ctx.src, non_blocking=True) for g in grads], ctx.dim)


class _Gather(torch.autograd.Function):
    @staticmethod
    def forward(ctx, target, dim, *xs):
        ctx.dim = dim
        ctx.devices = [x.device for x in xs]
        ctx.sizes = [x.size(dim) for x in xs]
        return torch.cat([x.to(target, non_blocking=True) for x in xs], dim)

    @staticmethod
    def backward(ctx, g):
        parts = g.split(ctx.sizes, ctx.dim)
        return (None, None, *[p.to(d, non_blocking=True).contiguous() for p, d in zip(parts, ctx.devices)])


def replicate(module: nn.Module, devices) -> list:
    """Per-device shallow replicas whose parameters are broadcast (non-leaf) copies."""
    params = list(module.parameters())
    bufs = list(module.buffers())
    pcopies = _Broadcast.apply(devices, *params) if params else ()
    n = len(params)
    pidx = {id(p): i for i, p in enumerate(params)}
    with torch.no_grad():
        bcopies = [[b.to(d, non_blocking=True) if b.device != d else b for b in bufs] for d in devices]
    bidx = {id(b): i for i, b in enumerate(bufs)}
    modules = list(module.modules())
    midx = {id(m): i for i, m in enumerate(modules)}
    reps = [[m._replicate_for_data_parallel() for m in modules] for _ in devices]
    for i, m in enumerate(modules):
        for j in range(len(devices)):
            r = reps[j][i]
            for k, ch in m._modules.items():
                r._modules[k] = None if ch is None else reps[j][midx[id(ch)]]
            for k, p in m._parameters.items():
                if p is None:
                    r._parameters[k] = None
                else:
                    setattr(r, k, pcopies[j * n + pidx[id(p)]])
            for k, b in m._buffers.items():
                r._buffers[k] = None if b is None else bcopies[j][bidx[id(b)]]
    return [reps[j][0] for j in range(len(devices))]


def parallel_apply(replicas, inputs, kwargs_list, devices):
    results = [None] * len(replicas)
    grad_enabled = torch.is_grad_enabled()
    autocast = torch.is_autocast_enabled()

    def work(i):
        try:
            d = devices[i]
            with torch.set_grad_enabled(grad_enabled), torch.autocast("cuda", enabled=autocast) \
                    if d.type == "cuda" else torch.set_grad_enabled(grad_enabled):
                if d.type == "cuda":
                    with torch.cuda.device(d):
                        results[i] = replicas[i](*inputs[i], **kwargs_list[i])
                else:
                    results[i] = replicas[i](*inputs[i], **kwargs_list[i])
        except BaseException as e:  # noqa: BLE001
            results[i] = e

    if len(replicas) == 1:
        work(0)
    else:
        threads = [threading.Thread(target=work, args=(i,)) for i in range(len(replicas))]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
    for r in results:
        if isinstance(r, BaseException):
            raise r
    return results


def _scatter_obj(obj, devices, dim):
    if isinstance(obj, torch.Tensor):
        return list(_Scatter.apply(devices, dim, obj))
    if isinstance(obj, (list, tuple)) and obj:
        cols = [_scatter_obj(o, devices, dim) for o in obj]
        n = min(len(c) for c in cols)
        return [type(obj)(c[i] for c in cols) for i in range(n)]
    if isinstance(obj, dict) and obj:
        cols = {k: _scatter_obj(v, devices, dim) for k, v in obj.items()}
        n = min(len(c) for c in cols.values())
        return [{k: c[i] for k, c in cols.items()} for i in range(n)]
    return [obj for _ in devices]


def _gather_obj(outs, target, dim):
    o0 = outs[0]
    if isinstance(o0, torch.Tensor):
        return _Gather.apply(target, dim, *outs)
    if isinstance(o0, (list, tuple)):
        return type(o0)(_gather_obj([o[i] for o in outs], target, dim) for i in range(len(o0)))
    if isinstance(o0, dict):
        return {k: _gather_obj([o[k] for o in outs], target, dim) for k in o0}
    return o0


class DataParallel(nn.Module):
    def __init__(self, module: nn.Module, device_ids=None, output_device=None, dim: int = 0):
        super().__init__()
        if device_ids is None:
            device_ids = list(range(torch.cuda.device_count())) or ["cpu"]
        self.module = module
        self.devices = [_dev(d) for d in device_ids]
        self.output_device = _dev(output_device) if output_device is not None else self.devices[0]
        self.dim = dim
        src = self.devices[0]
        for p in module.parameters():
            if p.device != src:
                raise RuntimeError(f"module must have its parameters on device_ids[0] ({src}), found {p.device}")

    def forward(self, *inputs, **kwargs):
        if len(self.devices) == 1:
            return self.module(*inputs, **kwargs)
        sin = _scatter_obj(inputs, self.devices, self.dim) if inputs else [() for _ in self.devices]
        skw = _scatter_obj(kwargs, self.devices, self.dim) if kwargs else [{} for _ in sin]
        n = len(sin)
        devs = self.devices[:n]
        replicas = replicate(self.module, devs)
        outs = parallel_apply(replicas, sin, skw, devs)
        return _gather_obj(outs, self.output_device, self.dim)
