"""Distributed sampling with ``torch.utils.data.DistributedSampler`` semantics.

Reference: ``DataLoader(..., shuffle=False, sampler=DistributedSampler(ds))``
ddp_gpus.py:72-79 and ``sampler.set_epoch(epoch)`` ddp_gpus.py:45:
defaults ``shuffle=True, seed=0, drop_last=False``; rank ``r`` takes
``perm[r::W]`` of ``randperm(N, generator=seed+epoch)`` after padding the
permutation to a multiple of ``W`` by wrapping around.

The index sequence is bit-identical to torch's (tested). Besides the Python
iterator, :meth:`epoch_indices` returns the rank's whole epoch as one int32
tensor so the device loader uploads it once per epoch (no per-step host work).
"""
from __future__ import annotations

import math

import torch


class DistributedSampler(torch.utils.data.Sampler):
    def __init__(self, dataset, num_replicas: int | None = None, rank: int | None = None,
                 shuffle: bool = True, seed: int = 0, drop_last: bool = False):
        if num_replicas is None or rank is None:
            from ..parallel import env

            num_replicas = env.world_size() if num_replicas is None else num_replicas
            rank = env.rank() if rank is None else rank
        if rank >= num_replicas or rank < 0:
            raise ValueError(f"Invalid rank {rank}, rank should be in the interval [0, {num_replicas - 1}]")
        self.dataset = dataset
        self.num_replicas = num_replicas
        self.rank = rank
        self.epoch = 0
        self.drop_last = drop_last
        n = len(dataset)
        if drop_last and n % num_replicas != 0:
            self.num_samples = math.ceil((n - num_replicas) / num_replicas)
        else:
            self.num_samples = math.ceil(n / num_replicas)
        self.total_size = self.num_samples * num_replicas
        self.shuffle = shuffle
        self.seed = seed

    def _global_indices(self) -> torch.Tensor:
        n = len(self.dataset)
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            idx = torch.randperm(n, generator=g)
        else:
            idx = torch.arange(n)
        if not self.drop_last:
            pad = self.total_size - n
            if pad > 0:
                if pad <= n:
                    idx = torch.cat([idx, idx[:pad]])
                else:
                    idx = torch.cat([idx.repeat(math.ceil(pad / n) + 1)])[: self.total_size]
        else:
            idx = idx[: self.total_size]
        assert idx.numel() == self.total_size
        return idx

    def epoch_indices(self) -> torch.Tensor:
        """This rank's indices for the current epoch (int64, CPU)."""
        return self._global_indices()[self.rank:self.total_size:self.num_replicas]

    def __iter__(self):
        return iter(self.epoch_indices().tolist())

    def __len__(self) -> int:
        return self.num_samples

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch
