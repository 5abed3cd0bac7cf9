"""Synthetic datasets of the reference, plus device-resident variants.

* :class:`MyTrainDataset` -- ``size`` pairs ``(rand(20), rand(1))`` (ddp_gpus.py:56-67,
  SURVEY R7). The reference draws them unseeded on every rank, so ranks train on
  different data (quirk Q3); here the default is a seeded dataset shared by all
  ranks (``per_rank_seed=True`` reproduces the reference's per-rank data).
* :class:`RandomDataset` -- ``randn(length, size)`` (NB01:118-127, R15).
* :class:`DeviceTensorDataset` -- the same tensors kept resident in HBM
  (generated on the GPU by the Philox kernel), served by
  :class:`..data.loader.DeviceDataLoader` with an on-device gather per step.
"""
from __future__ import annotations

import torch

from .._ext import native


class MyTrainDataset(torch.utils.data.Dataset):
    def __init__(self, size: int, in_features: int = 20, out_features: int = 1, seed: int | None = 0,
                 rank: int = 0, per_rank_seed: bool = False):
        super().__init__()
        self.size = size
        g = None
        if seed is not None:
            g = torch.Generator()
            g.manual_seed(seed + (rank if per_rank_seed else 0))
        x = torch.rand(size, in_features, generator=g)
        y = torch.rand(size, out_features, generator=g)
        self.x, self.y = x, y
        self.data = [(x[i], y[i]) for i in range(size)]

    def __len__(self):
        return self.size

    def __getitem__(self, index):
        return self.data[index]


class RandomDataset(torch.utils.data.Dataset):
    def __init__(self, size: int, length: int, seed: int | None = None):
        g = None
        if seed is not None:
            g = torch.Generator()
            g.manual_seed(seed)
        self.len = length
        self.data = torch.randn(length, size, generator=g)

    def __getitem__(self, index):
        return self.data[index]

    def __len__(self):
        return self.len


class DeviceTensorDataset(torch.utils.data.Dataset):
    """Tensors resident on one device; item i is ``tuple(t[i] for t in tensors)``."""

    def __init__(self, *tensors: torch.Tensor):
        if not tensors:
            raise ValueError("need at least one tensor")
        n = tensors[0].shape[0]
        if any(t.shape[0] != n for t in tensors):
            raise ValueError("all tensors need the same first dimension")
        self.tensors = tuple(t.contiguous() for t in tensors)

    @property
    def device(self):
        return self.tensors[0].device

    def __len__(self):
        return self.tensors[0].shape[0]

    def __getitem__(self, i):
        return tuple(t[i] for t in self.tensors)

    @classmethod
    def synthetic_regression(cls, size: int, in_features: int = 20, out_features: int = 1,
                             device="cpu", seed: int = 0):
        """``MyTrainDataset`` equivalent generated in place: uniform [0,1) features
        and targets (Philox on the GPU; torch's CPU generator on CPU)."""
        device = torch.device(device)
        x = torch.empty(size, in_features, device=device)
        y = torch.empty(size, out_features, device=device)
        if device.type == "cuda":
            C = native()
            C.philox_(x, seed, 0, 0)
            C.philox_(y, seed, (x.numel() + 3) // 4, 0)
        else:
            g = torch.Generator().manual_seed(seed)
            x.copy_(torch.rand(size, in_features, generator=g))
            y.copy_(torch.rand(size, out_features, generator=g))
        return cls(x, y)

    @classmethod
    def synthetic_classification(cls, size: int, in_features: int, num_classes: int, device="cpu",
                                 seed: int = 0):
        device = torch.device(device)
        x = torch.empty(size, in_features, device=device)
        g = torch.Generator().manual_seed(seed)
        labels = torch.randint(0, num_classes, (size,), generator=g).to(device)
        if device.type == "cuda":
            native().philox_(x, seed, 0, 1)
        else:
            x.copy_(torch.randn(size, in_features, generator=g))
        return cls(x, labels)
