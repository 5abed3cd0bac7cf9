"""One-shot xGMI all-reduce for latency-bound gradient buckets.

The DDP toy's whole gradient is one 84-byte bucket per step; RCCL
spends a kernel launch plus protocol round trips on it. On a fully connected
8x MI355X xGMI mesh each rank can instead write its contribution straight into
every peer's memory and poll its own (csrc/comm/xgmi.h: LL words
``{seq, value}`` in an uncached IPC-shared buffer, two parities, rank-ordered
sums so every replica gets bit-identical averages, bounded polls). The fused
DDP step kernel embeds this all-reduce and the SGD update, so one DDP step is
ONE kernel launch at any world size.

Safety: buffers are exchanged through the host control plane (gloo), and a
self-test all-reduce must produce the exact expected average with no poll
timeout on EVERY rank (agreed by a min-reduction) before the path is enabled;
otherwise callers fall back to RCCL. ``PTDT_XGMI=0`` disables it.
"""
from __future__ import annotations

import os

import torch

from .._ext import native


class XgmiAllReduce:
    def __init__(self, comm, device, max_elems: int = 1 << 16, self_test: bool = True):
        self.comm = comm
        self.device = torch.device(device)
        self.world = comm.world
        self.rank = comm.rank
        self.max_elems = max_elems
        self.x = None
        self.why = None  # why the one-shot path is off (None: it is on); reported by benchmarks
        handle = b""
        try:  # every rank reaches every collective below, whatever fails locally
            self.x = native().XgmiComm(self.rank, self.world, max_elems, self.device.index or 0)
            handle = self.x.handle()
        except RuntimeError as e:
            self.why = f"buffer setup failed on rank {self.rank}: {e}"
            print(f"[ptdt] xGMI buffer setup failed on rank {self.rank}: {e}", flush=True)
        # device ordinals travel with the handles: open() refuses a peer device with no
        # direct access path (then every rank falls back to RCCL)
        pairs = comm.all_gather_object((handle, self.device.index or 0))
        handles = [h for h, _ in pairs]
        ok_open = int(all(len(h) > 0 for h in handles))
        if ok_open:
            try:
                self.x.open(handles, [d for _, d in pairs])
            except RuntimeError as e:  # e.g. peer access unavailable
                self.why = f"IPC open failed on rank {self.rank}: {e}"
                print(f"[ptdt] xGMI all-reduce unavailable on rank {self.rank}: {e}", flush=True)
                ok_open = 0
        self.ok = self._agree(ok_open)
        if not self.ok and self.why is None:
            self.why = "another rank could not set up or open the IPC buffers"
        if self.ok and self_test:
            self.ok = self._agree(int(self._self_test()))
            if not self.ok:
                self.why = "self-test failed (a rank saw wrong sums or a poll timeout)"

    def _agree(self, v: int) -> bool:
        return min(self.comm.all_gather_object(int(v))) == 1

    def _self_test(self) -> bool:
        # full poll budget (ranks may reach the test far apart, e.g. sharing one GPU),
        # whatever shorter bound PTDT_XGMI_MAX_POLLS sets for the training launches
        budget = self.x.max_polls
        self.x.max_polls = 1 << 22  # kXgmiMaxPolls
        try:
            return self._self_test_body()
        finally:
            self.x.max_polls = budget

    def _self_test_body(self) -> bool:
        for n in (1, 21, 1000, min(self.max_elems, 5000)):
            t = torch.full((n,), float(self.rank + 1), device=self.device)
            t += torch.arange(n, device=self.device, dtype=torch.float32) * 1e-3
            for _ in range(3):  # both parities + a wrap
                v = t.clone()
                self.x.all_reduce_avg(v)
                torch.cuda.synchronize(self.device)
                want = (self.world + 1) / 2.0 + torch.arange(n, device=self.device, dtype=torch.float32) * 1e-3
                if self.x.error() != 0 or not torch.allclose(v, want, rtol=1e-6, atol=1e-6):
                    print(f"[ptdt] xGMI all-reduce self-test failed on rank {self.rank} (n={n})", flush=True)
                    self.x.reset_error()
                    return False
        return True

    @property
    def handle(self):
        return self.x

    def all_reduce_avg(self, t: torch.Tensor) -> torch.Tensor:
        self.x.all_reduce_avg(t)
        return t

    def check(self) -> None:
        """Raise if any poll timed out (a peer died / never arrived)."""
        if self.x.error() != 0:
            raise RuntimeError(f"xGMI all-reduce: poll timeout on rank {self.rank} (a peer did not arrive)")


def maybe_create(comm, device, max_elems: int = 1 << 16, mode: str | None = None):
    """XgmiAllReduce if enabled and healthy on every rank, else None (use RCCL)."""
    mode = (mode or os.environ.get("PTDT_XGMI", "auto")).lower()
    if mode in ("0", "off", "rccl", "false") or torch.device(device).type != "cuda":
        return None
    if comm.world > 8:
        return None
    try:
        x = XgmiAllReduce(comm, device, max_elems)
    except RuntimeError as e:
        print(f"[ptdt] xGMI all-reduce disabled: {e}", flush=True)
        return None
    return x if x.ok else None
