"""Structured metrics: a JSONL sink plus step timers.

The reference only prints status lines (kept verbatim by the Trainer); this
adds machine-readable records -- samples/s, step time, all-reduce time,
scaling efficiency -- for the benchmark harness. Rank 0 writes by default.
"""
from __future__ import annotations

import json
import os
import time


class JsonlSink:
    def __init__(self, path: str | None, rank: int = 0, all_ranks: bool = False):
        self.path = path
        self.enabled = path is not None and (all_ranks or rank == 0)
        self.rank = rank
        if self.enabled:
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)

    def write(self, **rec) -> None:
        if not self.enabled:
            return
        rec.setdefault("ts", time.time())
        rec.setdefault("rank", self.rank)
        with open(self.path, "a") as f:
            f.write(json.dumps(rec) + "\n")


class Timer:
    """Wall timer; ``sync`` is called at start/stop (e.g. torch.cuda.synchronize)."""

    def __init__(self, sync=None):
        self.sync = sync
        self.t0 = None
        self.elapsed = 0.0

    def __enter__(self):
        if self.sync:
            self.sync()
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *a):
        if self.sync:
            self.sync()
        self.elapsed = time.perf_counter() - self.t0


def scaling_efficiency(throughputs: dict[int, float]) -> dict[int, float]:
    """E(N) = S(N) / (N * S(1)) for a weak-scaling sweep {N: samples/s}."""
    s1 = throughputs.get(1)
    if not s1:
        return {}
    return {n: v / (n * s1) for n, v in sorted(throughputs.items())}
