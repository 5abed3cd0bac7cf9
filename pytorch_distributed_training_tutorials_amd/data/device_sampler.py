"""Device-side DistributedSampler (``device_sampler`` kernel in csrc/kernels/rng.hip).

Same sharding and padding semantics as ``torch.utils.data.DistributedSampler``
(rank ``r`` takes positions ``r, r+W, ...`` of the epoch permutation padded to
``ceil(N/W)*W`` by wrap-around; ``drop_last`` truncates), but the epoch
permutation is a keyed Feistel bijection of ``[0, N)`` evaluated per element on
the GPU and the epoch number lives in device memory: one launch per epoch
writes this rank's whole index list, and that launch can sit inside a hipGraph
that replays many epochs with no host involvement (no randperm, no H2D).
All ranks derive the same permutation from ``(seed, epoch)``, so the shards
partition the dataset exactly like torch's sampler. (The permutation itself
differs from ``torch.randperm``; use :class:`.sampler.DistributedSampler` when
bit-identical order to torch is required.) :func:`reference_indices` is a
host implementation of the same function used by the tests.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from .._ext import native

_M64 = (1 << 64) - 1


def _splitmix64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & _M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & _M64
    return x ^ (x >> 31)


def _mix32(h: np.ndarray) -> np.ndarray:
    h = h.astype(np.uint64)
    h ^= h >> np.uint64(16)
    h = (h * np.uint64(0x7FEB352D)) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(15)
    h = (h * np.uint64(0x846CA68B)) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(16)
    return h


def _num_samples(n: int, w: int, drop_last: bool) -> int:
    if drop_last and n % w != 0:
        return math.ceil((n - w) / w)
    return math.ceil(n / w)


def reference_indices(n: int, world: int, rank: int, epoch: int, seed: int = 0, shuffle: bool = True,
                      drop_last: bool = False) -> np.ndarray:
    """Host model of the kernel (numpy)."""
    ns = _num_samples(n, world, drop_last)
    pos = (rank + world * np.arange(ns, dtype=np.int64)) % n
    if not shuffle:
        return pos.astype(np.int32)
    bits = 1
    while (1 << bits) < n:
        bits += 1
    hb = bits // 2  # unbalanced split: L has bits - hb bits, R has hb
    mask_r = np.uint64((1 << hb) - 1)
    mask_l = np.uint64((1 << (bits - hb)) - 1)
    base = _splitmix64((seed ^ _splitmix64((epoch + 0x1234567) & _M64)) & _M64)
    keys = [np.uint64(_splitmix64((base + r) & _M64) & 0xFFFFFFFF) for r in range(4)]
    x = pos.astype(np.uint64)
    out = np.empty_like(x)
    todo = np.ones(len(x), dtype=bool)
    cur = x.copy()
    while todo.any():
        L = cur >> np.uint64(hb)
        R = cur & mask_r
        L = L ^ (_mix32(R ^ keys[0]) & mask_l)
        R = R ^ (_mix32(L ^ keys[1]) & mask_r)
        L = L ^ (_mix32(R ^ keys[2]) & mask_l)
        R = R ^ (_mix32(L ^ keys[3]) & mask_r)
        cur = (L << np.uint64(hb)) | R
        done = todo & (cur < np.uint64(n))
        out[done] = cur[done]
        todo &= ~done
    return out.astype(np.int32)


class DeviceDistributedSampler:
    def __init__(self, num_items: int, num_replicas: int = 1, rank: int = 0, shuffle: bool = True,
                 seed: int = 0, drop_last: bool = False, device="cuda"):
        if not 0 <= rank < num_replicas:
            raise ValueError(f"Invalid rank {rank} for {num_replicas} replicas")
        self.n = num_items
        self.num_replicas = num_replicas
        self.rank = rank
        self.shuffle = shuffle
        self.seed = seed
        self.drop_last = drop_last
        self.num_samples = _num_samples(num_items, num_replicas, drop_last)
        self.total_size = self.num_samples * num_replicas
        self.device = torch.device(device)
        self._epoch = torch.full((1,), -1, dtype=torch.int32, device=self.device)

    def __len__(self):
        return self.num_samples

    def set_epoch(self, epoch: int) -> None:
        """The next :meth:`generate` produces ``epoch`` (host write; not inside graphs)."""
        self._epoch.fill_(epoch - 1)

    def generate(self, out: torch.Tensor) -> torch.Tensor:
        """Advance the device epoch counter and write this rank's indices into ``out``."""
        if self.device.type == "cuda":
            native().device_sampler_(out, self.n, self.num_replicas, self.rank, self.num_samples, self.seed,
                                     self._epoch, self.shuffle)
        else:
            e = int(self._epoch.item()) + 1
            out[: self.num_samples].copy_(torch.from_numpy(reference_indices(
                self.n, self.num_replicas, self.rank, e, self.seed, self.shuffle, self.drop_last)))
            self._epoch.fill_(e)
        return out

    def current_epoch(self) -> int:
        return int(self._epoch.item())
