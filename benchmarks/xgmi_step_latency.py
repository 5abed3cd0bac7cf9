#!/usr/bin/env python3
"""Per-step cost of the in-kernel one-shot all-reduce inside the persistent wave engine.

World-size-2 DDP steps of the flagship toy (Linear(20,1), soft CE, B=32 per rank) with two
processes sharing ONE GPU (``cuda:0``): both persistent kernels run concurrently and exchange
gradients through the same IPC-shared uncached LL buffers as on an 8-GPU node, only without
the xGMI hop. It isolates the protocol overhead (push, poll detection, rank-ordered sum) that
the driver's multi-GPU scaling run adds on top of the 1-GPU step; the xGMI link latency itself
is only measurable on a multi-GPU node.

    python benchmarks/xgmi_step_latency.py --steps 20000
Prints one JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def worker(rank, world, port, steps, warmup, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from pytorch_distributed_training_tutorials_amd.data.device_sampler import DeviceDistributedSampler
    from pytorch_distributed_training_tutorials_amd.models.toy import ddp_toy_model
    from pytorch_distributed_training_tutorials_amd.ops.fused_step import FusedMLPStep
    from pytorch_distributed_training_tutorials_amd.parallel.comm import Communicator
    from pytorch_distributed_training_tutorials_amd.parallel.xgmi import XgmiAllReduce

    dev = torch.device("cuda", 0)
    ctl = Communicator(device=torch.device("cpu"))
    xg = XgmiAllReduce(ctl, dev, max_elems=4096)
    assert xg.ok, "xGMI buffers unavailable"
    torch.manual_seed(0)
    X = torch.rand(2048, 20, device=dev)
    Y = torch.rand(2048, 1, device=dev)
    res = {}
    for w, tag in ((world, "allreduce"), (1, "local_only")):
        torch.manual_seed(0)
        eng = FusedMLPStep(ddp_toy_model().to(dev), loss="ce_soft", lr=1e-2, xgmi=xg if w > 1 else None)
        sampler = DeviceDistributedSampler(2048, w if w > 1 else 1, rank if w > 1 else 0, seed=0, device=dev)
        cursor = torch.zeros(2, dtype=torch.int32, device=dev)
        losses = torch.zeros(8192, device=dev)
        eng.run_persistent(X, Y, warmup, 32, sampler, cursor, losses)
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        eng.run_persistent(X, Y, steps, 32, sampler, cursor, losses)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        t = torch.tensor([el])
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        res[tag] = {"us_per_step": round(1e6 * float(t) / steps, 3),
                    "engine": eng.persistent_engine(32, sampler)}
        xg.check()
        dist.barrier()
    if rank == 0:
        with open(out, "w") as f:
            json.dump(res, f)
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--steps", type=int, default=20000)
    ap.add_argument("--warmup", type=int, default=1000)
    a = ap.parse_args()
    import tempfile

    from pytorch_distributed_training_tutorials_amd.parallel.env import free_port
    from pytorch_distributed_training_tutorials_amd.parallel.launcher import spawn

    out = os.path.join(tempfile.mkdtemp(), "res.json")
    spawn(worker, args=(2, free_port(), a.steps, a.warmup, out), nprocs=2)
    res = json.load(open(out))
    ar, lo = res["allreduce"]["us_per_step"], res["local_only"]["us_per_step"]
    print(json.dumps({"metric": "in-kernel all-reduce cost per DDP step (2 ranks sharing one MI355X)",
                      "us_per_step_world2": ar, "us_per_step_world1_concurrent": lo,
                      "allreduce_overhead_us": round(ar - lo, 3), "steps": a.steps,
                      "engine": res["allreduce"]["engine"],
                      "note": "both processes share one GPU: no xGMI hop; the local-only run has the "
                              "two kernels running concurrently as well"}), flush=True)


if __name__ == "__main__":
    main()
