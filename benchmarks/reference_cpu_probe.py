#!/usr/bin/env python3
"""CPU/gloo comparator of the reference DDP toy loop (BASELINE.md "survey-local probe").

Re-measures the survey's method at W = 1, 2, 4 and adds W = 8: the
``ddp_gpus_torchrun.py`` job written out with stock torch (list-of-tuples
dataset of 2048 ``(rand(20), rand(1))`` samples, ``DataLoader(batch 32,
pin_memory, DistributedSampler)``, ``DistributedDataParallel(nn.Linear(20, 1))``,
``F.cross_entropy`` on float targets, ``SGD(lr=1e-2)``), gloo backend, one
process per rank with ``OMP_NUM_THREADS=1``, 1 warm-up epoch then 10 timed
epochs. Rank 0 prints whole-node samples/s. Launch:
``torchrun --standalone --nproc-per-node W benchmarks/reference_cpu_probe.py``.
"""
from __future__ import annotations

import json
import os
import time

import torch
import torch.distributed as dist
import torch.nn.functional as F
from torch.nn.parallel import DistributedDataParallel as DDP
from torch.utils.data import DataLoader, Dataset
from torch.utils.data.distributed import DistributedSampler


class _Synthetic(Dataset):
    def __init__(self, n):
        self.rows = [(torch.rand(20), torch.rand(1)) for _ in range(n)]

    def __len__(self):
        return len(self.rows)

    def __getitem__(self, i):
        return self.rows[i]


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    ds = _Synthetic(2048)
    sampler = DistributedSampler(ds)
    loader = DataLoader(ds, batch_size=32, pin_memory=True, shuffle=False, sampler=sampler)
    model = DDP(torch.nn.Linear(20, 1))
    opt = torch.optim.SGD(model.parameters(), lr=1e-2)

    def epoch(e):
        sampler.set_epoch(e)
        for xs, ys in loader:
            opt.zero_grad()
            F.cross_entropy(model(xs), ys).backward()
            opt.step()

    epoch(0)
    dist.barrier()
    t0 = time.perf_counter()
    for e in range(1, 11):
        epoch(e)
    dist.barrier()
    el = torch.tensor([time.perf_counter() - t0])
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    if rank == 0:
        samples = 10 * len(sampler) * world
        print(json.dumps({"world": world, "samples_per_s": round(samples / float(el), 1),
                          "steps_per_epoch": len(loader), "omp_threads": os.environ.get("OMP_NUM_THREADS")}),
              flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
