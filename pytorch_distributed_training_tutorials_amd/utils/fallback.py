"""Agreed fallback decisions for multi-rank runs (``bench.py``'s engine chain).

A first run on a multi-GPU node can fail in ways a one-GPU lease never shows: no
peer memory for the in-kernel xGMI exchange, a poll that times out, an RCCL
collective that refuses hipGraph capture, a replayed graph that computes
something else than its eager run. Each rank sees such a failure on its own, but
the next step is collective, so every rank must take the SAME next path.

* :meth:`Decider.check` is a decision point: each rank contributes its local
  verdict (plus any injected failure) and the verdicts are all-gathered over a
  host control plane (a gloo group, independent of RCCL's health). If any rank
  failed, every rank raises :class:`StageFailed` with all ranks' reasons.
* :func:`run_chain` tries engines in order; after each attempt the ranks agree
  on its outcome the same way (so a local exception also moves every rank on),
  and the failures travel into the JSON record's ``fallback`` field.

Fault injection: ``PTDT_BENCH_INJECT="point[@rank][,point[@rank]...]"`` fails the
named decision point (or a whole stage at its entry, ``stage:<name>``) on one rank (all
ranks without ``@``) -- the CPU tests drive every branch of the chain with it. Decision
points carry their names, so ranks that lost step (a local exception between two points
on one rank only) raise :class:`DesyncError` together instead of pairing wrong collectives.

Reference: the reference has no fallback at all (torchrun with
``max_restarts=0``, NCCL hard-coded); this belongs to the framework's
failure-detection layer next to ``utils/deadline.py`` and the RCCL watchdog.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


class DesyncError(RuntimeError):
    """The ranks reached different decision points: no agreed path exists any more."""


class StageFailed(RuntimeError):
    """A decision point failed on at least one rank (raised on every rank)."""

    def __init__(self, point: str, reasons: dict):
        self.point, self.reasons = point, reasons
        super().__init__(f"{point}: " + "; ".join(f"rank {r}: {w}" for r, w in sorted(reasons.items())))


def _parse_inject(spec: str | None):
    out = []
    for tok in (spec or "").split(","):
        tok = tok.strip()
        if tok:
            name, _, r = tok.partition("@")
            out.append((name, int(r) if r else None))
    return out


class Decider:
    """Decision points agreed across ranks over ``group`` (a gloo group; None: the default group)."""

    def __init__(self, rank: int = 0, world: int = 1, group=None, inject: str | None = None):
        self.rank, self.world, self.group = rank, world, group
        self.inject = _parse_inject(os.environ.get("PTDT_BENCH_INJECT") if inject is None else inject)
        self.points: list[str] = []  # decision points passed, in order (identical on every rank)

    def injected(self, point: str) -> bool:
        return any(n == point and (r is None or r == self.rank) for n, r in self.inject)

    def gather(self, why: str | None, point: str = "") -> dict:
        """{rank: reason} of the ranks whose ``why`` is not None (collective when world > 1). The
        point's name travels along: ranks at different decision points (a rank that left a stage
        by an exception the others did not see) is detected by every rank alike and ends the chain."""
        if self.world <= 1:
            return {} if why is None else {self.rank: why}
        got = [None] * self.world
        dist.all_gather_object(got, (point, why), group=self.group)
        names = {p for p, _ in got}
        if len(names) > 1:
            raise DesyncError(f"ranks at different decision points: {[p for p, _ in got]}")
        return {r: w for r, (_, w) in enumerate(got) if w is not None}

    def check(self, point: str, ok: bool = True, why: str = "") -> None:
        """Agree on decision point ``point``; raise StageFailed on every rank if any rank failed."""
        local = None if ok else (why or "failed")
        if local is None and self.injected(point):
            local = "injected failure (PTDT_BENCH_INJECT)"
        bad = self.gather(local, point)
        self.points.append(point)
        if bad:
            raise StageFailed(point, bad)

    def allclose(self, point: str, got: torch.Tensor, want: torch.Tensor, rtol=1e-5, atol=1e-6) -> None:
        ok = bool(torch.allclose(got.float().cpu(), want.float().cpu(), rtol=rtol, atol=atol))
        why = "" if ok else f"max |diff| {float((got.float() - want.float()).abs().max()):.3g}"
        self.check(point, ok, why)


def control_group(world: int):
    """A gloo group over all ranks for the decisions (None at world 1)."""
    if world <= 1 or not (dist.is_available() and dist.is_initialized()):
        return None
    return dist.new_group(backend="gloo")


def run_chain(decider: Decider, stages, log=print):
    """Try ``stages`` = [(name, fn(decider) -> result)] in order; return (name, result, failures)
    of the first stage that succeeds on EVERY rank. ``failures``: [{"stage", "point", "reasons"}]
    of the stages given up, identical on every rank. Raises StageFailed if every stage failed."""
    failures = []
    for name, fn in stages:
        point, local, res, reasons = None, None, None, None
        try:
            decider.check(f"stage:{name}")  # agreed entry (and the stage-level injection point)
            res = fn(decider)
        except StageFailed as e:  # agreed inside the stage: every rank is here, with the same reasons
            point, local, reasons = e.point, str(e), e.reasons
        except DesyncError:
            raise
        except Exception as e:  # noqa: BLE001 -- a local failure: agreed below
            local = f"{type(e).__name__}: {e}"
        bad = decider.gather(local, f"end:{name}")
        if not bad:
            return name, res, failures
        point = point or f"stage:{name}"
        reasons = reasons or bad  # the failing ranks' own reasons at the decision point
        failures.append({"stage": name, "point": point, "reasons": {str(r): w[:400] for r, w in reasons.items()}})
        if decider.rank == 0 and log is not None:
            log(f"[bench] {name} failed at {point!r} ({'; '.join(f'rank {r}: {w[:200]}' for r, w in reasons.items())}); "
                f"falling back", flush=True)
    raise StageFailed("every stage", {r: f["point"] for r, f in enumerate(failures)})
