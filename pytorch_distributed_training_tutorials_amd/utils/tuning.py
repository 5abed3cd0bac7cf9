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
  * otherwise every rank times, and inside an SPMD scope -- opened by a multi-rank
    ``DistributedDataParallel`` forward and closed when its backward finalises (or at
    the end of a no-grad forward) -- rank 0's decision is broadcast to all ranks with a
    hash of the shape key; a rank that reached a different key raises instead of
    pairing its decision with an unrelated shape (two small collectives per new shape,
    outside graph capture). Outside any scope (rank-0-only eval, pipeline / tensor
    parallel ranks with different layer shapes) each rank keeps its own timing: no
    collective is issued there, so asymmetric first uses cannot hang a run;
  * :func:`choices` reports what was decided (benchmarks print it).

Reference context: the DDP replicas of ddp_gpus.py:32 must stay identical; the
per-shape find mirrors cudnn.benchmark, which the reference's ResNet (NB03:969-992)
triggers through MIOpen on ROCm.
"""
from __future__ import annotations

import json
import os
import zlib

import torch

_TABLE: dict | None = None
_DECIDED: dict[str, dict[str, str]] = {"linear": {}, "convbn": {}}


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
    return v


_SCOPE: dict = {"comm": None, "depth": 0}


def spmd_begin(comm) -> None:
    """Open the SPMD scope: every rank of ``comm`` reaches the same new shapes in the same
    order until :func:`spmd_end` (DistributedDataParallel.forward opens it when world > 1)."""
    _SCOPE["comm"] = comm
    _SCOPE["depth"] = 1


def spmd_end() -> None:
    _SCOPE["depth"] = 0


def in_spmd_scope() -> bool:
    c = _SCOPE["comm"]
    return _SCOPE["depth"] > 0 and c is not None and c.world > 1


def _key_hash(family: str, key) -> int:
    return zlib.crc32(f"{family}:{key_str(key)}".encode())


def agree(family: str, key, local: str, options: tuple[str, str], device=None) -> str:
    """Rank 0's choice among ``options`` for ``key`` on every rank of the open SPMD scope
    (``local`` is this rank's own timing result); ``local`` outside a scope / at world 1.
    Raises on every rank if the ranks reached different keys."""
    choice = local
    if in_spmd_scope() and not (torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()):
        c = _SCOPE["comm"]
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
    _DECIDED[family][key_str(key)] = choice
    return choice


def choices() -> dict:
    """Every decision of this process so far: {family: {shape key: engine}}."""
    return {k: dict(v) for k, v in _DECIDED.items() if v}


def dump(path: str) -> None:
    """Write the decisions as a table loadable with ``PTDT_TUNING_TABLE``."""
    with open(path, "w") as f:
        json.dump(choices(), f, indent=1, sort_keys=True)
