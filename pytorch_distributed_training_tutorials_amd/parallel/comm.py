"""Communicator: the framework's collective API.

GPU tensors go through the native RCCL communicator (``csrc/comm``; one
process per GPU, xGMI), host tensors through ``torch.distributed`` (gloo).
Reference collectives: DDP init ALLGATHER/BROADCAST (M2-M4),
bucket ALLREDUCE (M5/M15), DP REDUCE/BROADCAST (M7/M10), model-parallel P2P
(M11/M12).

The native communicator's unique id is exchanged through the default c10d
store (``torch.distributed`` must be initialised, except for a 1-rank group).
Every GPU collective is enqueued on the caller's current stream (or an
explicit one), so it can be captured into a hipGraph and overlapped on a side
stream; a watchdog thread in C++ aborts the communicator instead of hanging
when a collective exceeds ``PTDT_COMM_TIMEOUT`` seconds (default 600).
"""
from __future__ import annotations

import os
import threading

import torch
import torch.distributed as dist

from .._ext import has_native, native
from . import env

_OPS = {"sum": 0, "prod": 1, "max": 2, "min": 3, "avg": 4}
_TORCH_OPS = {"sum": dist.ReduceOp.SUM, "prod": dist.ReduceOp.PRODUCT, "max": dist.ReduceOp.MAX,
              "min": dist.ReduceOp.MIN}

_registry_lock = threading.Lock()
_default = None
_all: list = []
_uid_counter = [0]


def _stream_handle(stream) -> int:
    if stream is None:
        return 0
    return int(stream.cuda_stream)


class Communicator:
    """Collectives over ``world`` ranks. ``native`` is True when GPU tensors use
    the framework's RCCL communicator."""

    def __init__(self, device: torch.device | None = None, group=None, timeout_s: float | None = None,
                 fingerprint: bool | None = None, name: str = "default"):
        self.group = group
        self.rank = env.rank() if group is None else dist.get_rank(group)
        self.world = env.world_size() if group is None else dist.get_world_size(group)
        self.device = device if device is not None else env.device()
        self.timeout_s = float(os.environ.get("PTDT_COMM_TIMEOUT", 600)) if timeout_s is None else timeout_s
        if fingerprint is None:
            fingerprint = os.environ.get("PTDT_DEBUG_FINGERPRINT", "0") == "1"
        self.fingerprint = fingerprint
        self.debug_sync = os.environ.get("PTDT_DEBUG_SYNC", "0") == "1"
        self._native = None
        self.name = name
        self._fp: list = []  # collective fingerprints (op, numel, dtype) when enabled
        if self.device.type == "cuda":
            if not has_native():
                native()  # raises: the GPU path must not silently fall back
            self._native = self._make_native()

    # ------------------------------------------------------------ setup
    def _make_native(self):
        C = native()
        _uid_counter[0] += 1
        # the key names the group by its global ranks: disjoint subgroups with the same
        # communicator name never read each other's unique id
        members = "all" if self.group is None else "-".join(map(str, dist.get_process_group_ranks(self.group)))
        key = f"ptdt/rccl_uid/{self.name}/{members}/{_uid_counter[0]}"
        if self.world == 1:
            uid = C.RcclComm.new_unique_id()
        else:
            if not env.is_initialized():
                raise RuntimeError("a multi-rank native communicator needs torch.distributed initialised")
            store = dist.distributed_c10d._get_default_store()
            if self.rank == 0:
                uid = C.RcclComm.new_unique_id()
                store.set(key, uid)
            else:
                uid = store.get(key)
        return C.RcclComm(self.rank, self.world, uid, self.device.index or 0, self.timeout_s, self.fingerprint)

    @property
    def native(self) -> bool:
        return self._native is not None

    @property
    def handle(self):
        """The underlying native ``RcclComm`` (GPU) or None."""
        return self._native

    def _check(self):
        if self._native is not None and self._native.aborted:
            raise RuntimeError(f"communicator aborted: {self._native.error()}")

    def _record(self, op: str, t: torch.Tensor):
        if self.fingerprint:
            self._fp.append(f"{len(self._fp)}:{op}:{t.numel()}:{str(t.dtype).replace('torch.', '')}")

    def _after(self, stream=None):
        if self.debug_sync and self._native is not None:
            (stream or torch.cuda.current_stream(self.device)).synchronize()
            self._check()

    # ------------------------------------------------------------ collectives
    def all_reduce(self, t: torch.Tensor, op: str = "sum", stream=None) -> torch.Tensor:
        self._record(f"all_reduce.{op}", t)
        if t.is_cuda and self._native is not None:
            self._native.all_reduce(t, _OPS[op], _stream_handle(stream))
            self._after(stream)
            return t
        if self.world == 1:
            return t
        if op == "avg":
            dist.all_reduce(t, dist.ReduceOp.SUM, group=self.group)
            t.div_(self.world)
        else:
            dist.all_reduce(t, _TORCH_OPS[op], group=self.group)
        return t

    def broadcast(self, t: torch.Tensor, src: int = 0, stream=None) -> torch.Tensor:
        self._record("broadcast", t)
        if t.is_cuda and self._native is not None:
            self._native.broadcast(t, src, _stream_handle(stream))
            self._after(stream)
            return t
        if self.world > 1:
            dist.broadcast(t, src, group=self.group)
        return t

    def reduce(self, t: torch.Tensor, dst: int = 0, op: str = "sum", stream=None) -> torch.Tensor:
        self._record(f"reduce.{op}", t)
        if t.is_cuda and self._native is not None:
            self._native.reduce(t, dst, _OPS[op], _stream_handle(stream))
            self._after(stream)
            return t
        if self.world > 1:
            dist.reduce(t, dst, _TORCH_OPS[op], group=self.group)
        return t

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor, stream=None) -> torch.Tensor:
        """``out`` is ``[world * inp.numel()]`` (rank-major)."""
        self._record("all_gather", inp)
        if inp.is_cuda and self._native is not None:
            self._native.all_gather(out, inp, _stream_handle(stream))
            self._after(stream)
            return out
        if self.world == 1:
            out.view(-1).copy_(inp.view(-1))
            return out
        dist.all_gather_into_tensor(out, inp, group=self.group)
        return out

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, op: str = "sum", stream=None):
        self._record(f"reduce_scatter.{op}", inp)
        if inp.is_cuda and self._native is not None:
            self._native.reduce_scatter(out, inp, _OPS[op], _stream_handle(stream))
            self._after(stream)
            return out
        if self.world == 1:
            out.copy_(inp.view_as(out))
            return out
        chunks = list(inp.view(self.world, -1).clone().unbind(0))
        tmp = torch.empty_like(chunks[0])
        dist.reduce_scatter(tmp, chunks, op=_TORCH_OPS["sum" if op == "avg" else op], group=self.group)
        if op == "avg":
            tmp.div_(self.world)
        out.view(-1).copy_(tmp)
        return out

    def all_to_all(self, out: torch.Tensor, inp: torch.Tensor, stream=None):
        self._record("all_to_all", inp)
        if inp.is_cuda and self._native is not None:
            self._native.all_to_all(out, inp, _stream_handle(stream))
            self._after(stream)
            return out
        if self.world == 1:
            out.copy_(inp)
            return out
        dist.all_to_all_single(out, inp, group=self.group)
        return out

    def send(self, t: torch.Tensor, dst: int, stream=None):
        self._record("send", t)
        if t.is_cuda and self._native is not None:
            self._native.send(t, dst, _stream_handle(stream))
            self._after(stream)
            return
        dist.send(t, dst, group=self.group)

    def recv(self, t: torch.Tensor, src: int, stream=None):
        self._record("recv", t)
        if t.is_cuda and self._native is not None:
            self._native.recv(t, src, _stream_handle(stream))
            self._after(stream)
            return t
        dist.recv(t, src, group=self.group)
        return t

    def group_start(self):
        if self._native is not None:
            self._native.group_start()

    def group_end(self):
        if self._native is not None:
            self._native.group_end()

    def barrier(self) -> None:
        """Device-ordered barrier: a 1-element all-reduce on the current stream
        followed by a stream sync (GPU), or a gloo barrier (CPU)."""
        if self._native is not None:
            t = torch.zeros(1, device=self.device, dtype=torch.int32)
            self._native.all_reduce(t, 0, 0)
            torch.cuda.current_stream(self.device).synchronize()
            self._check()
            return
        if self.world > 1:
            dist.barrier(group=self.group)

    def broadcast_object(self, obj, src: int = 0):
        if self.world == 1:
            return obj
        lst = [obj]
        dist.broadcast_object_list(lst, src=src, group=self.group, device=torch.device("cpu"))
        return lst[0]

    def all_gather_object(self, obj):
        if self.world == 1:
            return [obj]
        out = [None] * self.world
        dist.all_gather_object(out, obj, group=self.group)
        return out

    def fingerprints(self):
        """Python-level collective log (op, numel, dtype in issue order), plus the
        native communicator's own log when PTDT_DEBUG_FINGERPRINT=1."""
        return list(self._fp)

    def destroy(self):
        self._native = None


def get_default(device: torch.device | None = None) -> Communicator:
    global _default
    with _registry_lock:
        if _default is None:
            _default = Communicator(device=device)
            _all.append(_default)
        return _default


def new_communicator(device=None, group=None, name: str = "sub") -> Communicator:
    c = Communicator(device=device, group=group, name=name)
    with _registry_lock:
        _all.append(c)
    return c


def destroy_all():
    global _default
    with _registry_lock:
        for c in _all:
            c.destroy()
        _all.clear()
        _default = None


class HostStagedComm:
    """Control plane for ranks that share one GPU (single-GPU rehearsals of the
    multi-rank paths and their tests): gloo collectives on host copies, since
    RCCL refuses two ranks on one device. Same surface as :class:`Communicator`
    for what the engines use; nothing here is graph-capturable."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.rank, self.world = dist.get_rank(), dist.get_world_size()

    def barrier(self):
        torch.cuda.synchronize(self.device)
        dist.barrier()

    def broadcast(self, t, src=0):
        h = t.detach().cpu()
        dist.broadcast(h, src)
        t.copy_(h)
        return t

    def all_reduce(self, t, op="sum", stream=None):
        h = t.detach().cpu()
        if op == "avg":
            dist.all_reduce(h, dist.ReduceOp.SUM)
            h /= self.world
        else:
            dist.all_reduce(h, _TORCH_OPS[op])
        t.copy_(h)
        return t

    def all_gather_object(self, obj):
        out = [None] * self.world
        dist.all_gather_object(out, obj)
        return out
