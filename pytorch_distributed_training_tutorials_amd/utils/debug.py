"""Distributed debugging aids: collective fingerprint checks and
sync-after-every-collective mode.

* ``PTDT_DEBUG_FINGERPRINT=1`` makes every Communicator log each collective as
  ``seq:op:numel:dtype`` (the native RCCL communicator keeps its own log too);
  :func:`check_fingerprints` all-gathers the logs over the host control plane
  and raises on the first rank whose sequence diverges -- the classic cause of
  a silent DDP hang (ranks issuing different collectives), found without a
  hang, like c10d's ``TORCH_DISTRIBUTED_DEBUG=DETAIL`` ProcessGroupWrapper.
* ``PTDT_DEBUG_SYNC=1`` synchronises the stream after every collective and
  surfaces communicator errors at the call that caused them.
* :func:`debug_mode` enables both for a block (new communicators only).
"""
from __future__ import annotations

import contextlib
import hashlib
import os


class CollectiveMismatch(RuntimeError):
    pass


def check_fingerprints(comm) -> int:
    """Compare collective sequences across ranks; returns the number compared."""
    log = comm.fingerprints()
    digest = hashlib.sha1("\n".join(log).encode()).hexdigest()
    allv = comm.all_gather_object((len(log), digest, log[-64:]))
    ref_len, ref_dig, ref_tail = allv[0]
    for r, (n, dig, tail) in enumerate(allv):
        if (n, dig) != (ref_len, ref_dig):
            # locate the first differing entry within the shared tail window
            first = next((f"rank0={a!r} rank{r}={b!r}" for a, b in zip(ref_tail, tail) if a != b),
                         f"rank0 issued {ref_len} collectives, rank{r} issued {n}")
            raise CollectiveMismatch(f"collective sequence diverges between rank 0 and rank {r}: {first}")
    return ref_len


@contextlib.contextmanager
def debug_mode(sync: bool = True, fingerprint: bool = True):
    old = {k: os.environ.get(k) for k in ("PTDT_DEBUG_SYNC", "PTDT_DEBUG_FINGERPRINT")}
    if sync:
        os.environ["PTDT_DEBUG_SYNC"] = "1"
    if fingerprint:
        os.environ["PTDT_DEBUG_FINGERPRINT"] = "1"
    try:
        yield
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
