#!/usr/bin/env python3
"""Where does the fixed cost of a short persistent-engine run go?

Splits the bench's timed region (bench.py _timed around run_persistent) into
host/launch/sync pieces on one GPU: synchronize alone, the world-1 barrier, the
Python wrapper, the launch, and the kernel itself (HIP events), at several
step counts. Prints one JSON line per measurement.
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
    from pytorch_distributed_training_tutorials_amd.data import DeviceTensorDataset
    from pytorch_distributed_training_tutorials_amd.data.device_sampler import DeviceDistributedSampler
    from pytorch_distributed_training_tutorials_amd.models.toy import ddp_toy_model, ToyMLP
    from pytorch_distributed_training_tutorials_amd.ops.fused_step import FusedMLPStep
    from pytorch_distributed_training_tutorials_amd.parallel import comm as comm_mod
    from pytorch_distributed_training_tutorials_amd.parallel import env

    sched = os.environ.get("PTDT_DEVICE_SCHED")  # 0 auto / 1 spin / 2 yield / 4 blocking (hipSetDeviceFlags)
    if sched is not None:
        from pytorch_distributed_training_tutorials_amd._ext import native

        native().set_device_flags(0, int(sched))
    env.init_process_group("nccl")
    dev = torch.device("cuda", 0)
    comm = comm_mod.get_default(dev)
    reps = 30

    def timeit(fn, n=reps):
        out = []
        for _ in range(n):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            fn()
            out.append(time.perf_counter() - t0)
        return 1e6 * med(out)

    one = torch.zeros(1, device=dev)

    def tiny():  # one 1-element ATen kernel: the launch + dispatch + sync floor
        one.add_(1.0)
        torch.cuda.synchronize(dev)

    res = {"sync_us": timeit(lambda: torch.cuda.synchronize(dev)),
           "barrier_us": timeit(lambda: comm.barrier()),
           "tiny_kernel_wall_us": timeit(tiny)}
    for model_kind in ("linear", "mlp"):
        torch.manual_seed(0)
        if model_kind == "linear":
            model, loss = ddp_toy_model(20, 1).to(dev), "ce_soft"
            ds = DeviceTensorDataset.synthetic_regression(2048, 20, 1, device=dev, seed=0)
        else:
            model, loss = ToyMLP(20, 64, 10).to(dev), "ce_index"
            ds = DeviceTensorDataset.synthetic_classification(2048, 20, 10, device=dev, seed=0)
        X, Y = ds.tensors
        eng = FusedMLPStep(model, loss=loss, lr=1e-2, comm=comm)
        sampler = DeviceDistributedSampler(len(ds), 1, 0, seed=0, device=dev)
        cursor = torch.zeros(2, dtype=torch.int32, device=dev)
        losses = torch.zeros(8192, device=dev)
        eng.run_persistent(X, Y, 64, 32, sampler, cursor, losses)
        torch.cuda.synchronize(dev)
        plan = eng.persistent_plan(X, Y, 32, sampler, cursor, losses)
        for n in (1, 20, 200, 2000):
            def run():
                plan.launch(n)

            wall = timeit(lambda: (run(), torch.cuda.synchronize(dev)))
            launch_only = timeit(run, n=10)
            torch.cuda.synchronize(dev)
            evs = []
            for _ in range(10):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                run()
                b.record()
                b.synchronize()
                evs.append(1e3 * a.elapsed_time(b))
            res[f"{model_kind}_n{n}"] = {"wall_us": round(wall, 2), "host_call_us": round(launch_only, 2),
                                         "event_us": round(med(evs), 2)}
            print(json.dumps({model_kind: n, **res[f"{model_kind}_n{n}"]}), flush=True)
    print(json.dumps(res), flush=True)
    env.destroy_process_group()


if __name__ == "__main__":
    main()
