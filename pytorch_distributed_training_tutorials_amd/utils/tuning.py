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
  * otherwise every rank times, and rank 0's decision is broadcast to all ranks
    (one 4-byte collective per new shape, outside graph capture);
  * :func:`choices` reports what was decided (benchmarks print it).

Reference context: the DDP replicas of ddp_gpus.py:32 must stay identical; the
per-shape find mirrors cudnn.benchmark, which the reference's ResNet (NB03:969-992)
triggers through MIOpen on ROCm.
"""
from __future__ import annotations

import json
import os

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


def agree(family: str, key, local: str, options: tuple[str, str], device=None) -> str:
    """Rank 0's choice among ``options`` for ``key``, on every rank (``local`` is this rank's own
    timing result). World 1 / no process group: ``local``."""
    choice = local
    if torch.distributed.is_available() and torch.distributed.is_initialized() and \
            torch.distributed.get_world_size() > 1 and not (torch.cuda.is_available()
                                                            and torch.cuda.is_current_stream_capturing()):
        from ..parallel import comm as comm_mod

        dev = device if (device is not None and torch.device(device).type == "cuda") else None
        c = comm_mod.get_default(dev)
        flag = torch.tensor([float(options.index(local))], device=dev if dev is not None else "cpu")
        c.broadcast(flag, 0)
        choice = options[int(flag.item())]
    _DECIDED[family][key_str(key)] = choice
    return choice


def choices() -> dict:
    """Every decision of this process so far: {family: {shape key: engine}}."""
    return {k: dict(v) for k, v in _DECIDED.items() if v}


def dump(path: str) -> None:
    """Write the decisions as a table loadable with ``PTDT_TUNING_TABLE``."""
    with open(path, "w") as f:
        json.dump(choices(), f, indent=1, sort_keys=True)
