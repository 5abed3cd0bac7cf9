"""Rank-consistent, reproducible kernel-engine choices.

Two selectors time competing kernels on first use of a shape: plain big bf16 GEMMs
(ops/linear.py: gemm_big.hip vs hipBLASLt) and 1x1 conv + BN statistics
(ops/convbn.py: fused native kernel vs MIOpen + BN pass). Timing is noisy, so on
their own two DDP ranks could pick different kernels for one shape -- different
bf16 rounding, different BN statistics merges, replicas that are no longer
bit-identical. Here:

  * ``PTDT_TUNING_TABLE=<json>`` pins choices from a committed table
    (``{"linear": {"nt,128,1000,2048": "library"}, "convbn": {...}}``), so a run
    is reproducible across processes and days;
  * otherwise every rank times, and inside an SPMD scope rank 0's decision is broadcast to
    all ranks with a hash of the shape key; a rank that reached a different key raises
    instead of pairing its decision with an unrelated shape (two small collectives per new
    shape, outside graph capture). A multi-rank ``DistributedDataParallel`` forward arms a
    scope on its communicator (counted per communicator: two wrappers, or nested ones, each
    hold their own count) and its backward's finalisation disarms it; an armed scope is IN
    effect only while a DDP forward is running on this thread or a backward pass is running
    (autograd's graph task), so a grad-enabled forward that never ran backward cannot make a
    later rank-0-only inference broadcast alone. Outside any scope (rank-0-only eval,
    pipeline / tensor-parallel ranks with different layer shapes) each rank keeps its own
    timing and issues no collective;
  * decisions taken outside a scope are kept apart (:func:`lookup`): inside a scope such a
    key is agreed again (from this rank's earlier timing, not re-timed), so a shape first
    seen by rank 0 alone cannot be skipped by rank 0 while the other ranks broadcast;
  * :func:`choices` reports what was decided (benchmarks print it).

Reference context: the DDP replicas of ddp_gpus.py:32 must stay identical; the
per-shape find mirrors cudnn.benchmark, which the reference's ResNet (NB03:969-992)
triggers through MIOpen on ROCm.
"""
from __future__ import annotations

import contextlib
import json
import os
import threading
import zlib

import torch

_TABLE: dict | None = None
_DECIDED: dict[str, dict[str, str]] = {"linear": {}, "convbn": {}}  # everything decided (choices())
_AGREED: dict[str, dict[str, str]] = {"linear": {}, "convbn": {}}   # pinned or agreed in a scope: valid everywhere
_LOCAL: dict[str, dict[str, str]] = {"linear": {}, "convbn": {}}    # this rank's own timing, outside any scope


def _table() -> dict:
    global _TABLE
    if _TABLE is None:
        path = os.environ.get("PTDT_TUNING_TABLE")
        _TABLE = {}
        if path:
            with open(path) as f:
                _TABLE = json.load(f)
    return _TABLE


def key_str(key) -> str:
    return ",".join(str(k) for k in key)


def pinned(family: str, key) -> str | None:
    """The committed table's choice for ``key`` (None: not pinned)."""
    v = _table().get(family, {}).get(key_str(key))
    if v is not None:
        _DECIDED[family][key_str(key)] = v
        _AGREED[family][key_str(key)] = v
    return v


def lookup(family: str, key) -> str | None:
    """The cached decision for ``key`` valid here: an agreed (or pinned) one anywhere, this rank's
    own one only outside an SPMD scope (inside, the caller agrees it first: :func:`agree`)."""
    k = key_str(key)
    v = _AGREED[family].get(k)
    if v is None and not in_spmd_scope():
        v = _LOCAL[family].get(k)
    return v


def local_choice(family: str, key) -> str | None:
    """This rank's earlier out-of-scope decision for ``key`` (the input of a later agreement)."""
    return _LOCAL[family].get(key_str(key))


# armed scopes: id(comm) -> [comm, depth]; the most recently armed communicator is the current one
_SCOPES: dict[int, list] = {}
_ORDER: list[int] = []
_TLS = threading.local()  # per-thread depth of running DDP forwards


def spmd_begin(comm) -> None:
    """Arm an SPMD scope on ``comm`` (counted): every rank of ``comm`` reaches the same new shapes in
    the same order until the matching :func:`spmd_end` (DistributedDataParallel.forward arms it when
    world > 1, its backward's finalisation disarms it)."""
    e = _SCOPES.setdefault(id(comm), [comm, 0])
    e[1] += 1
    if id(comm) in _ORDER:
        _ORDER.remove(id(comm))
    _ORDER.append(id(comm))


def spmd_end(comm=None) -> None:
    """Disarm one count of ``comm``'s scope (None: the current one)."""
    k = id(comm) if comm is not None else (_ORDER[-1] if _ORDER else None)
    e = _SCOPES.get(k)
    if e is None:
        return
    e[1] -= 1
    if e[1] <= 0:
        del _SCOPES[k]
        _ORDER.remove(k)


@contextlib.contextmanager
def ddp_forward():
    """Marks a DDP forward running on this thread (an armed scope is in effect inside it)."""
    _TLS.depth = getattr(_TLS, "depth", 0) + 1
    try:
        yield
    finally:
        _TLS.depth -= 1


def _in_backward() -> bool:
    f = getattr(torch._C, "_current_graph_task_id", None)
    return f is not None and f() != -1


def _current_comm():
    for k in reversed(_ORDER):
        c = _SCOPES[k][0]
        if c.world > 1:
            return c
    return None


def in_spmd_scope() -> bool:
    if _current_comm() is None:
        return False
    return getattr(_TLS, "depth", 0) > 0 or _in_backward()


def scope_depth(comm) -> int:
    e = _SCOPES.get(id(comm))
    return e[1] if e is not None else 0


def _key_hash(family: str, key) -> int:
    return zlib.crc32(f"{family}:{key_str(key)}".encode())


def agree(family: str, key, local: str, options: tuple[str, str], device=None) -> str:
    """Rank 0's choice among ``options`` for ``key`` on every rank of the open SPMD scope
    (``local`` is this rank's own timing result); ``local`` outside a scope / at world 1.
    Raises on every rank if the ranks reached different keys."""
    choice = local
    agreed = False
    if in_spmd_scope() and not (torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()):
        c = _current_comm()
        h = _key_hash(family, key)
        dev = getattr(c, "device", None) or torch.device("cpu")
        msg = torch.tensor([float(options.index(local)), float(h & 0xFFFF), float(h >> 16)], device=dev)
        c.broadcast(msg, 0)
        got = [int(v) for v in msg.tolist()]
        bad = torch.tensor([0.0 if (got[1] | (got[2] << 16)) == h else 1.0], device=dev)
        c.all_reduce(bad, "max")
        if bad.item() != 0:
            raise RuntimeError(f"tuning.agree: ranks reached different {family} shape keys at the same point "
                               f"(this rank: {key_str(key)!r}); kernel choices would be paired with unrelated "
                               "shapes -- every rank of a DDP job must run the same shapes in the same order")
        choice = options[got[0]]
        agreed = True
    _DECIDED[family][key_str(key)] = choice
    (_AGREED if agreed else _LOCAL)[family][key_str(key)] = choice
    return choice


def choices() -> dict:
    """Every decision of this process so far: {family: {shape key: engine}}."""
    return {k: dict(v) for k, v in _DECIDED.items() if v}


def dump(path: str) -> None:
    """Write the decisions as a table loadable with ``PTDT_TUNING_TABLE``."""
    with open(path, "w") as f:
        json.dump(choices(), f, indent=1, sort_keys=True)
