"""Cross-entropy and MSE on native kernels (csrc/kernels/loss.hip).

Reference: ``F.cross_entropy(output, ys)`` ddp_gpus.py:37 -- with ``output``
[B,1] and float ``ys`` [B,1] this is *soft-target* CE over a single class, so
the loss and every gradient are exactly zero; the kernels compute
it faithfully (parity mode) and also support class-index targets with
``ignore_index`` and label smoothing. ``nn.MSELoss`` NB03:533,976.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .._ext import native, use_native


class _CrossEntropyFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, ignore_index: int, label_smoothing: float):
        soft = target if target.is_floating_point() else None
        index = None if soft is not None else target
        if soft is not None and soft.dtype != torch.float32:
            soft = soft.float()
        loss, lse, valid = native().ce_fwd(logits.contiguous(), soft.contiguous() if soft is not None else None,
                                           index.contiguous() if index is not None else None,
                                           ignore_index, label_smoothing)
        ctx.save_for_backward(logits, soft if soft is not None else index, lse, valid)
        ctx.is_soft = soft is not None
        ctx.ignore_index = ignore_index
        ctx.ls = label_smoothing
        return loss

    @staticmethod
    def backward(ctx, g):
        logits, tgt, lse, valid = ctx.saved_tensors
        soft = tgt if ctx.is_soft else None
        index = None if ctx.is_soft else tgt
        g = g.reshape(1).float().contiguous()
        d = native().ce_bwd(logits.contiguous(), soft, index, lse, valid, g, ctx.ignore_index, ctx.ls)
        return d, None, None, None


def cross_entropy(input: torch.Tensor, target: torch.Tensor, ignore_index: int = -100,
                  label_smoothing: float = 0.0, reduction: str = "mean") -> torch.Tensor:
    """Mean-reduced cross entropy over ``[B, C]`` logits with soft (float
    ``[B, C]``) or class-index (int64 ``[B]``) targets."""
    if use_native(input) and input.dim() == 2 and reduction == "mean":
        if target.is_floating_point() and target.shape != input.shape:
            raise ValueError(f"soft targets must match logits {tuple(input.shape)}, got {tuple(target.shape)}")
        return _CrossEntropyFn.apply(input, target, ignore_index, float(label_smoothing))
    return F.cross_entropy(input, target, ignore_index=ignore_index, label_smoothing=label_smoothing,
                           reduction=reduction)


class _MSEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, y):
        ctx.save_for_backward(x, y)
        return native().mse_fwd(x.contiguous(), y.contiguous())

    @staticmethod
    def backward(ctx, g):
        x, y = ctx.saved_tensors
        dx, dy = native().mse_bwd(x.contiguous(), y.contiguous(), g.reshape(1).float().contiguous(),
                                  ctx.needs_input_grad[0], ctx.needs_input_grad[1])
        return (dx if ctx.needs_input_grad[0] else None), (dy if ctx.needs_input_grad[1] else None)


def mse_loss(input: torch.Tensor, target: torch.Tensor, reduction: str = "mean") -> torch.Tensor:
    if use_native(input, target) and reduction == "mean" and input.dtype == target.dtype \
            and input.dtype in (torch.float32, torch.bfloat16):
        if input.shape != target.shape:
            raise ValueError(f"mse_loss shape mismatch {tuple(input.shape)} vs {tuple(target.shape)}")
        return _MSEFn.apply(input, target)
    return F.mse_loss(input, target, reduction=reduction)


class CrossEntropyLoss(nn.Module):
    def __init__(self, ignore_index: int = -100, label_smoothing: float = 0.0):
        super().__init__()
        self.ignore_index = ignore_index
        self.label_smoothing = label_smoothing

    def forward(self, input, target):
        return cross_entropy(input, target, self.ignore_index, self.label_smoothing)


class MSELoss(nn.Module):
    def forward(self, input, target):
        return mse_loss(input, target)


class _SumFn(torch.autograd.Function):
    """``x.sum()`` -> fp32 scalar by one native reduction launch; the backward is
    the upstream scalar broadcast as a stride-0 view (no fill kernel at all)."""

    @staticmethod
    def forward(ctx, x):
        ctx.shape, ctx.dtype = x.shape, x.dtype
        return native().sum_all(x.contiguous()).to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        return g.to(ctx.dtype).expand(ctx.shape)


def sum_loss(x: torch.Tensor) -> torch.Tensor:
    """The DP toy's ``loss = output.sum()`` (NB01:485): native on the GPU."""
    if use_native(x) and x.dtype in (torch.float32, torch.bfloat16):
        return _SumFn.apply(x)
    return x.sum()
