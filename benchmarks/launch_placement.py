#!/usr/bin/env python3
"""Single-shot latency of a short persistent-engine launch vs where it lands.

bench.py times ONE launch of K steps after warmup. A 1-workgroup kernel lands on
whichever XCD the dispatcher picks, so a single shot usually starts with cold
L2 (code, dataset rows, parameters) unless every launch is pinned to the same
CUs. Measures launch+sync wall time of n steps, hot (back-to-back) and after an
idle gap, on the default stream and on a CU-masked stream. One JSON line per case.
"""
from __future__ import annotations

import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def med(xs):
    xs = sorted(xs)
    return xs[len(xs) // 2]


def main():
    from pytorch_distributed_training_tutorials_amd import native
    from pytorch_distributed_training_tutorials_amd.data import DeviceTensorDataset
    from pytorch_distributed_training_tutorials_amd.data.device_sampler import DeviceDistributedSampler
    from pytorch_distributed_training_tutorials_amd.models.toy import ddp_toy_model
    from pytorch_distributed_training_tutorials_amd.ops.fused_step import FusedMLPStep

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    model = ddp_toy_model(20, 1).to(dev)
    ds = DeviceTensorDataset.synthetic_regression(2048, 20, 1, device=dev, seed=0)
    X, Y = ds.tensors
    eng = FusedMLPStep(model, loss="ce_soft", lr=1e-2)
    sampler = DeviceDistributedSampler(len(ds), 1, 0, seed=0, device=dev)
    cursor = torch.zeros(2, dtype=torch.int32, device=dev)
    losses = torch.zeros(64, device=dev)
    plan = eng.persistent_plan(X, Y, 32, sampler, cursor, losses)
    streams = {"default": torch.cuda.current_stream(dev),
               "cu0": torch.cuda.ExternalStream(native().cu_masked_stream(0, [0]), device=dev),
               "cu0-3": torch.cuda.ExternalStream(native().cu_masked_stream(0, [0, 1, 2, 3]), device=dev)}
    one = torch.zeros(1, device=dev)

    def spin(sec):
        t = time.perf_counter()
        while time.perf_counter() - t < sec:
            pass

    def wake():  # idle gap, then one tiny kernel + sync right before t0 (what bench's barrier does)
        time.sleep(0.002)
        one.add_(1.0)
        torch.cuda.synchronize(dev)

    gaps = {"none": None, "sleep2ms": lambda: time.sleep(0.002), "spin2ms": lambda: spin(0.002), "sleep+kernel": wake}
    for name, st in streams.items():
        with torch.cuda.stream(st):
            for n in (1, 20):
                for gap, gfn in gaps.items():
                    if name != "default" and gap not in ("none", "sleep2ms"):
                        continue
                    ts = []
                    for r in range(25):
                        torch.cuda.synchronize(dev)
                        if gfn is not None:
                            gfn()
                        t0 = time.perf_counter()
                        plan.launch(n)
                        torch.cuda.synchronize(dev)
                        ts.append(1e6 * (time.perf_counter() - t0))
                    print(json.dumps({"stream": name, "n": n, "gap": gap, "median_us": round(med(ts), 2),
                                      "min_us": round(min(ts), 2), "max_us": round(max(ts), 2)}), flush=True)


if __name__ == "__main__":
    main()
