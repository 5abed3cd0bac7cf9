#!/usr/bin/env python3
"""Fixed (per-launch) cost of the single-wave persistent engine, split by
in-kernel timers: wave 0's time from after the prologue barrier to the end
(stamps[8], 100 MHz realtime) vs the HIP-event time of the whole launch, for
the Feistel sampler and an explicit index list. One JSON line per case."""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def med(xs):
    xs = sorted(xs)
    return xs[len(xs) // 2]


def main():
    from pytorch_distributed_training_tutorials_amd.data import DeviceTensorDataset
    from pytorch_distributed_training_tutorials_amd.data.device_sampler import DeviceDistributedSampler
    from pytorch_distributed_training_tutorials_amd.models.toy import ddp_toy_model
    from pytorch_distributed_training_tutorials_amd.ops.fused_step import FusedMLPStep

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = ddp_toy_model(20, 1).to(dev)
    ds = DeviceTensorDataset.synthetic_regression(2048, 20, 1, device=dev, seed=0)
    X, Y = ds.tensors
    eng = FusedMLPStep(model, loss="ce_soft", lr=1e-2)
    sampler = DeviceDistributedSampler(len(ds), 1, 0, seed=0, device=dev)
    cursor = torch.zeros(2, dtype=torch.int32, device=dev)
    losses = torch.zeros(4096, device=dev)
    idx = torch.randperm(2048, device=dev).to(torch.int32)
    for given in (False, True):
        for n in (1, 2, 3, 4, 20, 64):
            ev, tot = [], []
            for r in range(15):
                st = torch.zeros(9, dtype=torch.int64, device=dev)
                cursor.zero_()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                eng.run_persistent(X, Y, n, 32, sampler, cursor, losses, stamps=st,
                                   idx=idx if given else None, cursor_j=0)
                b.record()
                b.synchronize()
                ev.append(1e3 * a.elapsed_time(b))
                tot.append(st[8].item() * 10e-3)  # 100 MHz ticks -> us
            print(json.dumps({"idx_given": given, "n": n, "event_us": round(med(ev), 2),
                              "wave0_after_prologue_us": round(med(tot), 2)}), flush=True)


if __name__ == "__main__":
    main()
