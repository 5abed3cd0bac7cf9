#!/usr/bin/env python3
"""What the first multi-GPU run needs to know before its numbers can be read.

Run under ``python -m torch.distributed.run --nproc-per-node N`` (one rank per GPU). Rank 0 prints
ONE JSON line:

  * ``rccl_ranks``: ranks an RCCL all-reduce of ones actually summed over (== N, or the launch is
    not what it claims);
  * ``peer_access``: the hipDeviceCanAccessPeer matrix of the visible devices;
  * ``xgmi_ok`` / ``xgmi_why``: the one-shot in-kernel all-reduce's IPC setup and self-test across
    the devices (the bench's persistent engine needs it; without it the bench falls back to the
    fused engine + RCCL and says so in its own line);
  * ``barrier_skew_us``: how far apart the ranks leave the node-local spin barrier (the bench's
    timed-region release), max - min of CLOCK_MONOTONIC over 20 rounds (median);
  * ``allreduce_84B_us``: an 84-byte RCCL all-reduce (the reference's per-step bucket),
    median of 200 after warm-up.

Reference: ddp_gpus.py:12-17 (rendezvous + process group), SURVEY M5 / §5.8.
"""
from __future__ import annotations

import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from pytorch_distributed_training_tutorials_amd.parallel import comm as comm_mod
    from pytorch_distributed_training_tutorials_amd.parallel import env
    from pytorch_distributed_training_tutorials_amd.parallel.xgmi import XgmiAllReduce
    from pytorch_distributed_training_tutorials_amd.utils import spin_barrier

    env.init_process_group("nccl")
    rank, world = env.rank(), env.world_size()
    dev = env.device()
    comm = comm_mod.get_default(dev)
    out = {"n_gpus": world, "visible_devices": torch.cuda.device_count()}
    ones = torch.ones(1, device=dev)
    comm.all_reduce(ones, "sum")
    torch.cuda.synchronize(dev)
    out["rccl_ranks"] = int(ones.item())
    n = torch.cuda.device_count()
    out["peer_access"] = [[i == j or torch.cuda.can_device_access_peer(i, j) for j in range(n)] for i in range(n)]
    if world > 1:
        xg = XgmiAllReduce(comm, dev)
        out["xgmi_ok"], out["xgmi_why"] = bool(xg.ok), xg.why
        bar = spin_barrier.create(comm)
        skews = []
        for _ in range(20):
            comm.barrier()
            if bar is not None:
                bar.wait()
            t = time.clock_gettime_ns(time.CLOCK_MONOTONIC)
            stamps = comm.all_gather_object(t)
            skews.append((max(stamps) - min(stamps)) / 1e3)
        out["barrier_skew_us"] = round(statistics.median(skews), 2)
        out["release"] = "spin barrier (/dev/shm)" if bar is not None else "collective barrier"
    else:
        out["xgmi_ok"], out["xgmi_why"] = None, "world 1: no all-reduce"
    t84 = torch.zeros(21, device=dev)
    lat = []
    for i in range(240):
        torch.cuda.synchronize(dev)
        a = time.perf_counter()
        comm.all_reduce(t84, "sum")
        torch.cuda.synchronize(dev)
        if i >= 40:
            lat.append((time.perf_counter() - a) * 1e6)
    out["allreduce_84B_us"] = round(statistics.median(lat), 2)
    if rank == 0:
        print(json.dumps({"what": "multi_gpu_probe", **out}), flush=True)
    env.destroy_process_group()


if __name__ == "__main__":
    main()
