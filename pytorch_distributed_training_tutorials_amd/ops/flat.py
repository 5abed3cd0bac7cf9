"""Flat (contiguous) parameter storage.

MI355X-first memory layout: a model's parameters (and optionally its
gradients / optimizer state) live in ONE contiguous buffer per (device, dtype),
and each ``nn.Parameter`` is a view into it. Then an optimizer step, a
gradient all-reduce or a broadcast is a single launch / single collective over
one coalesced region (16-B vector accesses, no per-tensor launch overhead),
instead of the reference's per-tensor foreach lists.
"""
from __future__ import annotations

from collections import OrderedDict

import torch


def _key(p: torch.Tensor):
    return (p.device, p.dtype)


class FlatParameters:
    """Moves ``params`` (in order) into contiguous buffers; ``p.data`` becomes a
    view so every existing reference (optimizer, hooks, state_dict) keeps working."""

    def __init__(self, params, with_grads: bool = False):
        self.params = [p for p in params]
        groups: "OrderedDict[tuple, list]" = OrderedDict()
        for p in self.params:
            groups.setdefault(_key(p), []).append(p)
        self.buffers: dict = {}
        self.grad_buffers: dict = {}
        self.offsets: dict = {}
        for key, ps in groups.items():
            n = sum(p.numel() for p in ps)
            flat = torch.empty(n, device=key[0], dtype=key[1])
            gflat = torch.zeros(n, device=key[0], dtype=key[1]) if with_grads else None
            off = 0
            for p in ps:
                k = p.numel()
                flat[off:off + k].copy_(p.data.reshape(-1))
                p.data = flat[off:off + k].view_as(p)
                if gflat is not None:
                    p.grad = gflat[off:off + k].view_as(p)
                self.offsets[id(p)] = (key, off, k)
                off += k
            self.buffers[key] = flat
            if gflat is not None:
                self.grad_buffers[key] = gflat

    def flat(self, device=None, dtype=None) -> torch.Tensor:
        if len(self.buffers) == 1 and device is None:
            return next(iter(self.buffers.values()))
        for (d, t), b in self.buffers.items():
            if (device is None or torch.device(device) == d) and (dtype is None or dtype == t):
                return b
        raise KeyError((device, dtype))

    def flat_grad(self, device=None, dtype=None) -> torch.Tensor:
        if len(self.grad_buffers) == 1 and device is None:
            return next(iter(self.grad_buffers.values()))
        for (d, t), b in self.grad_buffers.items():
            if (device is None or torch.device(device) == d) and (dtype is None or dtype == t):
                return b
        raise KeyError((device, dtype))


def contiguous_span(tensors) -> torch.Tensor | None:
    """If ``tensors`` are back-to-back dense blocks of one storage (in order; any
    dense memory order, e.g. channels_last), return the 1-D view covering all
    of them, else None. Elementwise use of two spans is only valid when the
    tensors pair up with equal strides (:func:`same_layout`)."""
    if not tensors:
        return None
    t0 = tensors[0]
    if not all(is_dense(t) for t in tensors):
        return None
    st = t0.untyped_storage().data_ptr()
    esz = t0.element_size()
    ptr = t0.data_ptr()
    for t in tensors:
        if t.untyped_storage().data_ptr() != st or t.dtype != t0.dtype or t.data_ptr() != ptr:
            return None
        ptr += t.numel() * esz
    total = sum(t.numel() for t in tensors)
    base = torch.empty(0, dtype=t0.dtype, device=t0.device).set_(
        t0.untyped_storage(), t0.storage_offset(), (total,), (1,))
    return base


def is_dense(t: torch.Tensor) -> bool:
    """Non-overlapping and dense: the elements fill exactly numel() consecutive
    slots starting at data_ptr() (any dimension order, positive strides)."""
    if t.is_contiguous():
        return True
    expect = 1
    for stride, size in sorted((st, sz) for st, sz in zip(t.stride(), t.shape) if sz != 1):
        if stride != expect:
            return False
        expect *= size
    return True


def same_layout(xs, ys) -> bool:
    """Pairwise equal shapes and memory orders (strides)."""
    return len(xs) == len(ys) and all(a.shape == b.shape and a.stride() == b.stride() for a, b in zip(xs, ys))


def dense_like(buf: torch.Tensor, p: torch.Tensor) -> torch.Tensor:
    """View ``buf`` (1-D, p.numel() elements) with ``p``'s shape and memory order."""
    if p.is_contiguous() or not is_dense(p):
        return buf.view(p.shape)
    return buf.as_strided(p.shape, p.stride())
