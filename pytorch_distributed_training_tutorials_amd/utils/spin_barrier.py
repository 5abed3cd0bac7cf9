"""Node-local shared-memory spin barrier: releases every rank of one node within a
microsecond or two, for timing windows that start on all ranks at once.

Why: ``bench.py`` times K steps between barriers and reports the MAX over ranks. A
collective barrier (RCCL all-reduce + stream sync, or gloo) releases the ranks tens
of microseconds apart, and with the persistent engines' in-kernel all-reduce an
early rank's clock runs while it waits for the late ones -- at the driver's 20 steps
of ~2 us that skew WAS the measurement (12.45 us/step at 20 steps vs
1.85 us/step at 2,000 in the 8-rank rehearsal). After the collective barrier, every
rank writes its arrival epoch into its own 64-byte slot of a ``/dev/shm`` page and
spins until all slots hold it: one cache line per rank, no atomics (each slot has
one writer), release within one poll of the last arrival.

Reference: the timing protocol of ddp_gpus_torchrun.py:16-88 as benchmarked by
bench.py (SURVEY §6, E(N) = S(N) / (N S(1))). Ranks of other nodes (WORLD_SIZE !=
LOCAL_WORLD_SIZE) are not covered: :func:`create` returns None there.
"""
from __future__ import annotations

import mmap
import os
import struct
import time
import uuid

_SLOT = 64  # bytes per rank: one cache line, one writer


class SetupFailed(RuntimeError):
    """Raised on EVERY rank when any rank could not create or map the shared page."""


class NodeSpinBarrier:
    def __init__(self, comm, timeout_s: float = 60.0):
        self.rank, self.world = comm.rank, comm.world
        self.timeout_s = timeout_s
        name = comm.all_gather_object(f"ptdt_spin_{os.getpid()}_{uuid.uuid4().hex[:12]}")[0]  # rank 0's
        self.path = os.path.join("/dev/shm", name)
        size = max(mmap.PAGESIZE, _SLOT * self.world)
        self.mm = None
        err = ""
        if self.rank == 0:
            try:
                fd = os.open(self.path, os.O_CREAT | os.O_EXCL | os.O_RDWR, 0o600)
                os.ftruncate(fd, size)
                os.close(fd)
            except OSError as e:
                err = f"rank 0: {e}"
        # every step agrees across ranks (a rank that raised alone would leave the others in a barrier)
        errs = [e for e in comm.all_gather_object(err) if e]
        if not errs:
            try:
                fd = os.open(self.path, os.O_RDWR)
                try:
                    self.mm = mmap.mmap(fd, size)
                finally:
                    os.close(fd)
            except OSError as e:
                err = f"rank {self.rank}: {e}"
            errs = [e for e in comm.all_gather_object(err) if e]
        if self.rank == 0:  # every rank has it mapped (or gave up): the name can go
            try:
                os.unlink(self.path)
            except OSError:
                pass
        if errs:
            self.close()
            raise SetupFailed("; ".join(errs))
        self.epoch = 0
        self._offs = [r * _SLOT for r in range(self.world)]

    def wait(self) -> float:
        """Arrive and spin until every local rank has arrived; returns seconds spent spinning."""
        self.epoch += 1
        e = self.epoch
        mm, offs = self.mm, self._offs
        struct.pack_into("<q", mm, offs[self.rank], e)
        t0 = time.monotonic()
        unpack = struct.unpack_from
        while True:
            for o in offs:
                if unpack("<q", mm, o)[0] < e:
                    break
            else:
                return time.monotonic() - t0
            if time.monotonic() - t0 > self.timeout_s:
                raise TimeoutError(f"spin barrier: rank {self.rank} waited {self.timeout_s:.0f} s for the other ranks")

    def close(self):
        try:
            if self.mm is not None:
                self.mm.close()
        except Exception:  # noqa: BLE001
            pass


def create(comm, timeout_s: float = 60.0):
    """A barrier over ``comm``'s ranks when they all share this node (else None)."""
    world = comm.world
    local = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if world <= 1 or local != world:
        return None
    try:
        return NodeSpinBarrier(comm, timeout_s)
    except SetupFailed:  # collective: every rank falls back to the collective barrier together
        return None
