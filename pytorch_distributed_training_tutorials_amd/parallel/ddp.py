"""DistributedDataParallel on the native bucketed reducer + RCCL.

Reference: ``DistributedDataParallel(model, device_ids=[gpu_id])``
ddp_gpus.py:32 / ddp_gpus_torchrun.py:28. Same
observable contract: constructor verifies parameter shapes across ranks and
broadcasts rank 0's parameters and buffers; ``forward`` broadcasts buffers
(``broadcast_buffers=True``) and arms the reducer; backward all-reduces
gradient buckets (averaged) overlapped with the rest of backward; after
backward every ``p.grad`` holds the global average; the wrapper's
``state_dict`` keys carry the ``module.`` prefix; ``no_sync()`` accumulates
locally.

MI355X specifics (see csrc/reducer/reducer.h): gradients are bucket views (no
pack/unpack), RCCL ncclAvg (no scale kernel), buckets on a high-priority comm
stream launched in index order, xGMI-sized caps (parallel/bucketing.py), and a
rebuild in rank 0's observed ready order after the first iteration.
"""
from __future__ import annotations

import contextlib
import os
import weakref

import torch
import torch.nn as nn

from .._ext import native
from . import bucketing, comm as comm_mod


def _flatten_broadcast(tensors, c: comm_mod.Communicator, src: int = 0):
    """Coalesced broadcast: one flat buffer per (device, dtype)."""
    groups = {}
    for t in tensors:
        groups.setdefault((t.device, t.dtype), []).append(t)
    for (_, _), ts in groups.items():
        flat = torch.cat([t.detach().reshape(-1) for t in ts])
        c.broadcast(flat, src)
        off = 0
        for t in ts:
            n = t.numel()
            with torch.no_grad():
                t.copy_(flat[off:off + n].view_as(t))
            off += n


def _has_grad_fn(out) -> bool:
    """Whether any tensor in a (nested) forward output carries an autograd graph."""
    if isinstance(out, torch.Tensor):
        return out.grad_fn is not None
    if isinstance(out, (list, tuple)):
        return any(_has_grad_fn(o) for o in out)
    if isinstance(out, dict):
        return any(_has_grad_fn(o) for o in out.values())
    return False


def _same_dense_layout(a: torch.Tensor, b: torch.Tensor) -> bool:
    """Same shape and element order in memory: dense, equal strides on every dimension of size > 1
    (a [Cout, Cin, 1, 1] weight gradient is (Cin, 1, 1, 1) contiguous and (Cin, 1, Cin, Cin) in
    channels_last -- one layout)."""
    from ..ops.flat import is_dense

    if a.shape != b.shape or not (is_dense(a) and is_dense(b)):
        return False
    return all(sa == sb for n, sa, sb in zip(a.shape, a.stride(), b.stride()) if n > 1)


def _state_buffers(module: nn.Module):
    """Buffers that are model state (persistent): running statistics, counters. Non-persistent
    scratch (e.g. ops.norm.BatchNorm2d's kernel tickets) is neither synced nor checkpointed."""
    out = []
    for m in module.modules():
        for name, b in m._buffers.items():
            if b is not None and name not in m._non_persistent_buffers_set:
                out.append(b)
    return out


class DistributedDataParallel(nn.Module):
    def __init__(self, module: nn.Module, device_ids=None, output_device=None, broadcast_buffers: bool = True,
                 bucket_cap_mb: float | None = None, first_bucket_mb: float | None = None,
                 find_unused_parameters: bool = False, comm: comm_mod.Communicator | None = None,
                 rebuild_buckets: bool = True, init_sync: bool = True):
        super().__init__()
        self.module = module
        params = []
        seen = set()
        for p in module.parameters():
            if p.requires_grad and id(p) not in seen:
                seen.add(id(p))
                params.append(p)
        if not params:
            raise RuntimeError("DistributedDataParallel: module has no parameters that require grad")
        self.device = params[0].device
        if device_ids is not None and self.device.type == "cuda":
            want = torch.device("cuda", device_ids[0] if not isinstance(device_ids[0], torch.device) else device_ids[0].index)
            if want != self.device:
                raise ValueError(f"module parameters are on {self.device}, device_ids says {want}")
        self.comm = comm if comm is not None else comm_mod.get_default(self.device if self.device.type == "cuda" else None)
        self.world_size = self.comm.world
        self.broadcast_buffers = broadcast_buffers
        self.find_unused_parameters = find_unused_parameters
        self.require_backward_grad_sync = True
        self._params = params
        self._rebuild = rebuild_buckets and self.world_size > 1
        self._rebuilt = False
        f, cap = bucketing.xgmi_bucket_caps(self.world_size)
        self._first_cap = int(first_bucket_mb * bucketing.MiB) if first_bucket_mb is not None else f
        self._cap = int(bucket_cap_mb * bucketing.MiB) if bucket_cap_mb is not None else cap

        if init_sync and self.world_size > 1:
            self._verify_shapes()
            _flatten_broadcast(list(module.parameters()) + _state_buffers(module), self.comm, 0)

        plan = bucketing.plan(params, None, self._first_cap, self._cap, self.world_size)
        py_ar = None
        if self.device.type != "cuda":
            def py_ar(t, _c=self.comm):
                _c.all_reduce(t, "avg")
        self.reducer = native().Reducer(params, plan, self.comm.handle if self.device.type == "cuda" else None,
                                        py_ar, find_unused_parameters)
        self._queued = False
        self._hooks = [p.register_post_accumulate_grad_hook(self._make_hook(i)) for i, p in enumerate(params)]
        # grad sinks (ops/conv.py): weights cast through SinkCast land their gradient directly in
        # the bucket slot when .grad is None, which zero_grad arranges for exactly these params
        self._sink_params, self._sink_idx = [], []
        self._params = params
        self._forwards = 0
        self._defer, self._pending, self._remaining = False, {}, {}
        self._fwd_stream = None
        self._multi_use = set()  # weights seen with a second, non-SinkCast use: never deferred again
        if self.device.type == "cuda":
            from ..ops.conv import Conv2d
            from ..ops.linear import Linear
            from ..ops.norm import BatchNorm2d

            sink_ids = {id(m.weight) for m in module.modules() if isinstance(m, (Conv2d, Linear))}
            sink_ids |= {id(t) for m in module.modules() if isinstance(m, BatchNorm2d)
                         for t in (m.weight, m.bias) if t is not None}
            # deferred weight-gradient casts (ops/conv.py): a bucket's bf16 gradients are converted
            # into its slots by one launch, issued when the bucket's LAST parameter is marked ready
            # (before its all-reduce). Needs every parameter to report (no find_unused_parameters).
            self._defer = (not find_unused_parameters and os.environ.get("PTDT_DEFER_GRAD_CAST", "1") != "0")
            self._index_buckets()
            for i, p in enumerate(params):
                if id(p) in sink_ids:
                    p._ptdt_grad_sink = self._make_sink(i, p)
                    if self._defer:
                        p._ptdt_grad_defer = self._make_defer(i)
                        self._hooks.append(p.register_hook(self._make_tied_check(i)))
                    self._sink_params.append(p)
                    self._sink_idx.append(i)
        self._sink_ids = set(self._sink_idx)

    # --------------------------------------------------------------- internals
    def _verify_shapes(self):
        """Reference M2/M3: every rank must hold the same parameter list."""
        desc = [(tuple(p.shape), str(p.dtype)) for p in self.module.parameters()]
        allv = self.comm.all_gather_object(desc)
        for r, d in enumerate(allv):
            if d != desc:
                raise RuntimeError(f"DDP: rank {r} has a different parameter list than rank {self.comm.rank}")

    def _make_sink(self, i: int, p):
        """The bucket-slot view of parameter ``i`` for the FIRST gradient producer of
        this forward only. A weight used twice in one forward (tied weights, a
        module called twice) has several producers; the later ones get None and
        return an ordinary gradient, which autograd sums into the first one's
        slot before AccumulateGrad adopts it (writing each into the slot would
        overwrite the earlier contribution).

        The closure holds the wrapper weakly: the parameters outlive a dropped
        wrapper, which must stay collectable (``__del__`` detaches the sinks)."""
        ref = weakref.ref(self)

        def sink():
            ddp = ref()
            if ddp is None or getattr(p, "_ptdt_sink_forward", -1) == ddp._forwards:
                return None
            p._ptdt_sink_forward = ddp._forwards
            return ddp.reducer.grad_view(i)
        return sink

    def _make_defer(self, i: int):
        """Record parameter ``i``'s bf16 gradient for its bucket's batched cast into the slot.

        Only the index is kept, never the slot view the sink handed to autograd: an extra
        reference to that view would make AccumulateGrad copy it instead of adopting it.
        ``defer(None, None)`` (a second contribution to a tied weight arrived) casts the
        pending gradient now, before autograd adds the other contribution into the slot."""
        ref = weakref.ref(self)

        def defer(dst, src):
            ddp = ref()
            if ddp is None:
                return False
            b = ddp._bucket_of[i]
            if dst is None:  # tied weight: flush this parameter's entry now
                pend = ddp._pending.get(b, [])
                for k, (j, g) in enumerate(pend):
                    if j == i:
                        del pend[k]
                        ddp.reducer.grad_view(j).copy_(g)
                        break
                return True
            if (i in ddp._multi_use or src.dtype != torch.bfloat16 or dst.dtype != torch.float32
                    or not _same_dense_layout(src, dst)):
                return False
            ddp._pending.setdefault(b, []).append((i, src))
            return True
        return defer

    def _make_tied_check(self, i: int):
        """Leaf gradient pre-hook (runs on the SUM of every contribution, before AccumulateGrad) for a
        deferred-cast weight. With one contribution the incoming gradient IS the slot view the sink
        handed out, whose cast is still pending: nothing to do. A different tensor means autograd summed
        another, non-SinkCast use of the weight (e.g. a Linear weight tied to an fp32 F.embedding) onto
        the slot's STALE contents (zero_grad skips sink slots): the pending cast would then overwrite
        that sum. Return ``g - stale + cast`` instead (the other use's gradient plus this one's), drop
        the pending entry, and never defer this weight again."""
        ref = weakref.ref(self)

        def check(g):
            ddp = ref()
            if ddp is None or not ddp._defer:
                return None
            pend = ddp._pending.get(ddp._bucket_of.get(i))
            if not pend:
                return None
            k = next((k for k, (j, _) in enumerate(pend) if j == i), None)
            if k is None or g.data_ptr() == ddp._slot_ptr[i]:
                return None
            _, src = pend.pop(k)
            ddp._multi_use.add(i)
            return g - ddp.reducer.grad_view(i) + src.to(g.dtype)
        return check

    def _index_buckets(self):
        self._buckets = [list(b) for b in self.reducer.buckets()]
        self._bucket_of = {int(i): b for b, ps in enumerate(self._buckets) for i in ps}
        self._slot_ptr = {i: self.reducer.grad_view(i).data_ptr() for i in range(len(self._params))}

    def _flush_casts(self, b=None):
        keys = [b] if b is not None else list(self._pending)
        for k in keys:
            pend = self._pending.pop(k, None)
            if pend:
                cur = torch.cuda.current_stream(self.device)
                if cur != self._fwd_stream:  # hooks on another stream than the producers (an AccumulateGrad
                    for _, g in pend:        # node kept from another stream): keep the sources alive for it
                        g.record_stream(cur)
                native().cast_multi_([self.reducer.grad_view(j) for j, _ in pend], [g for _, g in pend])

    def _make_hook(self, i: int):
        ref = weakref.ref(self)  # as in _make_sink: parameters must not keep the wrapper alive

        def hook(_p):
            ddp = ref()
            if ddp is None:
                return
            if not ddp._queued and ddp.reducer.in_backward:
                ddp._queued = True
                torch.autograd.Variable._execution_engine.queue_callback(ddp._finalize)
            if ddp._defer:
                b = ddp._bucket_of.get(i)
                left = ddp._remaining.get(b, 0) - 1
                ddp._remaining[b] = left
                if left <= 0 and b in ddp._pending:  # the bucket completes with this mark: fill its slots
                    ddp._flush_casts(b)
            ddp.reducer.mark_ready(i)
        return hook

    def _finalize(self):
        self._queued = False
        self._flush_casts()  # anything a bucket never completed (e.g. no_sync accumulation)
        self.reducer.finalize()
        self._close_scope()

    def _close_scope(self):
        """Disarm the SPMD scope this wrapper's grad-enabled forward armed (utils/tuning.py)."""
        if getattr(self, "_scope_open", False):
            from ..utils import tuning

            tuning.spmd_end(self.comm)
            self._scope_open = False

    def _maybe_rebuild(self):
        if not self._rebuild or self._rebuilt or self.reducer.iteration < 1:
            return
        order = self.comm.broadcast_object(list(self.reducer.ready_order()), 0)
        if len(order) == len(self._params):
            self.reducer.rebuild(bucketing.plan(self._params, order, self._first_cap, self._cap, self.world_size))
            if hasattr(self, "_bucket_of"):
                self._index_buckets()
        self._rebuilt = True

    # --------------------------------------------------------------- API
    def forward(self, *args, **kwargs):
        self._maybe_rebuild()
        if self.broadcast_buffers and self.world_size > 1:
            bufs = _state_buffers(self.module)
            if bufs:
                _flatten_broadcast(bufs, self.comm, 0)
        if torch.is_grad_enabled():
            self.reducer.prepare_for_backward(self.require_backward_grad_sync)
            self._forwards += 1  # a new forward: every grad sink may be claimed once again
            if self._defer:
                self._flush_casts()
                self._fwd_stream = torch.cuda.current_stream(self.device)
                self._remaining = {b: len(ps) for b, ps in enumerate(self._buckets)}
        if self.world_size > 1:  # ranks run the same shapes in lock step until this step's backward ends
            from ..utils import tuning  # (utils imports this module: no top-level import)

            self._close_scope()  # the previous grad-enabled forward never ran backward: its scope is stale
            tuning.spmd_begin(self.comm)
            self._scope_open = True
            try:
                with tuning.ddp_forward():
                    out = self.module(*args, **kwargs)
            except BaseException:
                self._close_scope()
                raise
            # no backward will finalise (no grad mode, or nothing in the output needs a gradient)
            if not torch.is_grad_enabled() or not _has_grad_fn(out):
                self._close_scope()
            return out
        return self.module(*args, **kwargs)

    @contextlib.contextmanager
    def no_sync(self):
        old = self.require_backward_grad_sync
        self.require_backward_grad_sync = False
        try:
            yield
        finally:
            self.require_backward_grad_sync = old

    def bucket_sizes_bytes(self):
        return [int(t.numel() * t.element_size()) for t in self.reducer.bucket_tensors()]

    def bucket_params(self):
        return self.reducer.buckets()

    def remove_grad_sinks(self):
        """Detach the parameters from this wrapper's buckets (also done when it is collected):
        later backwards produce ordinary gradient tensors again."""
        for p in getattr(self, "_sink_params", ()):
            if getattr(p, "_ptdt_grad_sink", None) is not None:
                del p._ptdt_grad_sink
            if getattr(p, "_ptdt_grad_defer", None) is not None:
                del p._ptdt_grad_defer
        self._sink_params, self._sink_idx, self._sink_ids = [], [], set()

    def __del__(self):
        try:
            self._close_scope()
            self.remove_grad_sinks()
            for h in getattr(self, "_hooks", ()):
                h.remove()
        except Exception:  # noqa: BLE001 -- interpreter shutdown
            pass

    def zero_grad(self, set_to_none: bool = False):
        """Zero the gradient buckets in place (keeps .grad as bucket views; grad-sink
        parameters get ``None``, refilled in place by their cast's backward). When the sinks
        cover most parameters (ResNet-50: all but fc.bias) only the other slots are zeroed:
        every sink's producer overwrites its whole slot (a producer that does not -- a second
        use, an unused parameter -- goes through the reducer's copy / zero-on-demand path), so
        zeroing the full 102 MB of buckets each step was a wasted pass."""
        if self._sink_params and len(self._sink_ids) * 2 >= len(self._params):
            self.reducer.zero_grads_except(self._sink_idx)
        else:
            self.reducer.zero_grads()
        for p in self._sink_params:
            p.grad = None
