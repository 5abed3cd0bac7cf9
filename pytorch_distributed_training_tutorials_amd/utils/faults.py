"""Fault injection for failure-detection tests.

``PTDT_FAULT_RANK=k PTDT_FAULT_STEP=s [PTDT_FAULT_MODE=exit|hang|raise]``
makes rank ``k`` fail when it reaches global step ``s``: ``exit`` kills the
process (``os._exit(17)``, as a crashed worker would), ``hang`` stops making
progress (exercises the communicator watchdog / launcher timeouts), ``raise``
throws. The launcher must then tear the job down instead of hanging.
"""
from __future__ import annotations

import os
import time


class FaultInjector:
    def __init__(self, rank: int):
        self.rank = rank
        fr = os.environ.get("PTDT_FAULT_RANK")
        self.armed = fr is not None and int(fr) == rank
        self.step_at = int(os.environ.get("PTDT_FAULT_STEP", "0"))
        self.mode = os.environ.get("PTDT_FAULT_MODE", "exit")

    def check(self, step: int) -> None:
        if not self.armed or step != self.step_at:
            return
        print(f"[ptdt] fault injection: rank {self.rank} fails at step {step} (mode={self.mode})", flush=True)
        if self.mode == "exit":
            os._exit(17)
        if self.mode == "hang":
            while True:
                time.sleep(3600)
        raise RuntimeError(f"injected fault on rank {self.rank} at step {step}")
