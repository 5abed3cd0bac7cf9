"""The reference's toy models, built on the native Linear.

* :func:`ddp_toy_model` -- ``torch.nn.Linear(20, 1)`` trained with CE on float
  targets (ddp_gpus.py:81-82). 21 parameters.
* :class:`SampleModel` -- ``Linear(32 -> 2)`` that prints the per-replica input
  shape (NB01:168-175, R16) to make the DataParallel split visible.
* :class:`ToyModel` -- ``net1 = Linear(10000, 10)`` + ReLU on ``dev0``,
  ``net2 = Linear(10, 5)`` on ``dev1`` (NB03:440-450, R19): the naive
  model-parallel toy. 100,065 parameters.
* :class:`ToyMLP` -- ``Linear(in, hidden) -> ReLU -> Linear(hidden, classes)``,
  the "toy MLP mode"  so kernels do real work.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ..ops.linear import Linear


def ddp_toy_model(in_features: int = 20, out_features: int = 1, device=None) -> nn.Module:
    """Reference DDP toy: a single ``Linear(20, 1)`` (state_dict keys ``weight``, ``bias``)."""
    return Linear(in_features, out_features, device=device)


class SampleModel(nn.Module):
    def __init__(self, input_size: int = 32, output_size: int = 2, verbose: bool = True):
        super().__init__()
        self.fc = Linear(input_size, output_size)
        self.verbose = verbose

    def forward(self, x):
        if self.verbose:
            print(f"Input shape: {x.shape}")  # per replica, as in NB01:174
        return self.fc(x)


class ToyModel(nn.Module):
    def __init__(self, dev0="cuda:0", dev1="cuda:1", in_features: int = 10000, hidden: int = 10, out: int = 5):
        super().__init__()
        self.dev0 = torch.device(dev0)
        self.dev1 = torch.device(dev1)
        self.net1 = Linear(in_features, hidden, relu=True).to(self.dev0)  # ReLU fused into net1's epilogue
        self.relu = nn.Identity()  # kept for module-tree parity with the reference (ReLU lives in net1)
        self.net2 = Linear(hidden, out).to(self.dev1)

    def forward(self, x):
        x = self.relu(self.net1(x.to(self.dev0)))
        return self.net2(x.to(self.dev1))


class ToyMLP(nn.Sequential):
    def __init__(self, in_features: int = 20, hidden: int = 64, out_features: int = 10, device=None):
        super().__init__(Linear(in_features, hidden, device=device), nn.ReLU(),
                         Linear(hidden, out_features, device=device))


def model_size(model: nn.Module) -> int:
    """Reference helper ``model_size`` (NB03:844-845): number of parameters
    (deduplicated, so aliased stage modules count once)."""
    return sum(p.numel() for p in model.parameters())
