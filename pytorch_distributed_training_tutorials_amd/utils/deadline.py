"""Whole-run deadline for benchmark / job processes.

A first multi-GPU run that hangs (a peer that never arrives, a collective that
never completes) must still leave a record before an outer time limit kills
the job. :class:`Deadline` is a watchdog thread with a named current *phase*:
when the deadline expires it

1. calls ``on_expire(phase, elapsed)`` (bench.py prints its error JSON line there),
2. aborts the registered communicators (``abort(reason)`` on each; bounded by a
   10 s grace so a stuck abort cannot hold the exit), and
3. ends the process with ``os._exit(code)``.

No new process is started and nothing is re-executed (an exec from a process
that touched the GPU is forbidden on this platform); every rank runs its own
deadline, so all ranks of a hung job leave at about the same time, and the
launcher (torchrun) tears the rest down on the first non-zero exit.

Reference: the reference has no timeouts at all (torchrun
``max_restarts=0`` and no heartbeats); this is part of the MI355X framework's
failure-detection layer, next to the RCCL watchdog (``csrc/comm/rccl_comm.cpp``)
and the launcher's teardown (``parallel/launcher.py``).
"""
from __future__ import annotations

import contextlib
import os
import sys
import threading
import time


class Deadline:
    def __init__(self, seconds: float, on_expire=None, exit_code: int = 3, grace_s: float = 10.0,
                 exit_delay_s: float = 0.0):
        self.seconds = float(seconds)
        self.on_expire = on_expire
        self.exit_code = exit_code
        self.grace_s = grace_s
        # a non-reporting rank waits this long before exiting: the launcher tears the job down
        # on the first exit, which must not cut off the reporting rank's record
        self.exit_delay_s = exit_delay_s
        self.phase = "start"
        self.t0 = time.monotonic()
        self._abortables: list = []
        self._done = threading.Event()
        self._thread = None
        if self.seconds > 0:
            self._thread = threading.Thread(target=self._watch, name="ptdt-deadline", daemon=True)
            self._thread.start()

    def set_phase(self, name: str) -> None:
        self.phase = name

    @contextlib.contextmanager
    def phase_of(self, name: str):
        old = self.phase
        self.phase = name
        try:
            yield
        finally:
            self.phase = old

    def register(self, obj) -> None:
        """``obj.abort(reason)`` is called on expiry (a native communicator handle)."""
        if obj is not None and hasattr(obj, "abort"):
            self._abortables.append(obj)

    def remaining(self) -> float:
        return self.seconds - (time.monotonic() - self.t0) if self.seconds > 0 else float("inf")

    def cancel(self) -> None:
        self._done.set()

    def _watch(self):
        if self._done.wait(self.seconds):
            return
        elapsed = time.monotonic() - self.t0
        try:
            if self.on_expire is not None:
                self.on_expire(self.phase, elapsed)
        except Exception as e:  # noqa: BLE001 -- the exit below must happen regardless
            print(f"[deadline] on_expire failed: {e!r}", file=sys.stderr, flush=True)

        def abort_all():
            for a in self._abortables:
                with contextlib.suppress(Exception):
                    a.abort(f"deadline of {self.seconds:.0f} s expired in phase {self.phase!r}")

        t = threading.Thread(target=abort_all, daemon=True)
        t.start()
        t.join(self.grace_s)
        if self.exit_delay_s > 0:
            time.sleep(self.exit_delay_s)
        with contextlib.suppress(Exception):
            sys.stdout.flush()
            sys.stderr.flush()
        os._exit(self.exit_code)
