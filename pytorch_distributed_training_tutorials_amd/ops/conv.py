"""Conv2d whose mixed-precision weight cast writes its gradient straight into
the DDP gradient bucket.

Under ``torch.autocast("cuda", torch.bfloat16)`` every convolution casts its
fp32 master weight to bf16 in the forward; in the backward the bf16 weight
gradient is cast back to fp32 (one kernel) and then accumulated into the
parameter's ``.grad`` -- a bucket view of the DDP reducer -- by a second
elementwise kernel (``AccumulateGrad``'s ``grad += new``). In the ResNet-50 DDP
step that is 2 x 161 kernels (profiles/r1_resnet_window.md: the bf16->fp32
copies and the ``add<float>`` kernels).

``Conv2d`` here performs that cast through :class:`SinkCast`: when the
parameter carries a *grad sink* (installed by ``parallel.ddp``; returns a fresh
view of the parameter's bucket slot) and its ``.grad`` is ``None`` (DDP's
``zero_grad`` clears it), the backward converts the bf16 gradient directly into
the bucket slot with one copy kernel and hands that view to autograd, which
adopts it as ``.grad`` without another kernel. With DDP's deferred casts (the
default on GPU) even that copy is batched: the sink records (slot, bf16 gradient)
and the wrapper converts a whole bucket's pending gradients in ONE multi-tensor
launch (``cast_multi_``) right before that bucket's all-reduce is issued (or at
the end of backward), 53 launches per ResNet-50 step -> one per bucket. Without a sink, outside autocast,
or while gradients accumulate (``no_sync``) it behaves exactly like the
autocast cast. Parameters and state_dict are ``nn.Conv2d``'s.

Reference call sites: the 53 convolutions of torchvision's ResNet-50
(NB03:560-570, NB03:807-833).
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn


class SinkCast(torch.autograd.Function):
    """``w.to(dtype)`` whose backward can land the gradient in ``w``'s DDP bucket slot."""

    @staticmethod
    def forward(ctx, w, dtype, shadow=None):
        ctx.w = w
        return shadow.detach() if shadow is not None else w.to(dtype)

    @staticmethod
    def backward(ctx, g):
        w = ctx.w
        sink = getattr(w, "_ptdt_grad_sink", None)
        out = sink() if (sink is not None and w.grad is None) else None  # None: slot already claimed
        defer = getattr(w, "_ptdt_grad_defer", None)
        if out is not None:
            if defer is None or not defer(out, g):
                out.copy_(g)  # bf16 -> fp32 conversion straight into the bucket
            return out, None, None
        if defer is not None and sink is not None and w.grad is None:
            defer(None, None)  # a tied weight's other use deferred its cast: land it before autograd adds
        return g.to(w.dtype), None, None


def cast_weight(w: torch.Tensor) -> torch.Tensor:
    """The autocast dtype copy of an fp32 parameter (through SinkCast when it needs a gradient)."""
    if not (w.is_cuda and w.dtype == torch.float32 and torch.is_autocast_enabled("cuda")):
        return w
    dt = torch.get_autocast_dtype("cuda")
    if dt not in (torch.bfloat16, torch.float16):
        return w
    # the optimizer's bf16 copy of the current weight (FusedSGD(bf16_shadow=True)), if still current
    sh = getattr(w, "_ptdt_bf16", None)
    if sh is not None and (dt != torch.bfloat16 or getattr(w, "_ptdt_bf16_version", -1) != w._version):
        sh = None
    if w.requires_grad and torch.is_grad_enabled():
        return SinkCast.apply(w, dt, sh)
    return sh if sh is not None else w.to(dt)


def _pad_rgb(x: torch.Tensor, w: torch.Tensor):
    """3 input channels -> 4 (zero channel in the input, zero slice in the weight: the same
    convolution). MIOpen's NHWC bf16 solvers handle a 7x7/2 stem on 3 channels poorly (C = 3 does
    not fill an MFMA K step): at batch 128 forward + weight gradient take 450 us on 3 channels and
    342 us on 4, the pad included (benchmarks/stem_probe.py, profiles/r3_stem_probe.jsonl). The
    input's cast to the compute dtype happens in the same copy."""
    if x.requires_grad or w.dtype != torch.bfloat16 or x.dtype not in (torch.float32, torch.bfloat16):
        n, _, h, wd = x.shape
        xp = torch.zeros((n, 4, h, wd), device=x.device, dtype=w.dtype, memory_format=torch.channels_last)
        xp[:, :3] = x
    else:  # one native pass: cast + pad (csrc/kernels/elementwise.hip rgb4_pack)
        from .._ext import native

        xp = native().rgb4_pack(x)
    return xp, torch.nn.functional.pad(w, (0, 0, 0, 0, 0, 1))


class Conv2d(nn.Conv2d):
    """Drop-in ``nn.Conv2d`` (same parameters, init, state_dict) with the grad-sink weight cast.
    Under bf16 autocast a 3-channel channels_last input (an RGB stem) runs as a 4-channel
    convolution (``PTDT_PAD_RGB=0`` disables it)."""

    def forward(self, x):
        w = cast_weight(self.weight)
        if w is not self.weight:
            b = self.bias.to(w.dtype) if self.bias is not None else None
            if (self.in_channels == 3 and self.groups == 1 and x.dim() == 4 and self.padding_mode == "zeros"
                    and x.is_contiguous(memory_format=torch.channels_last) and _PAD_RGB):
                x, w = _pad_rgb(x, w)
            else:
                x = x.to(w.dtype)
            return self._conv_forward(x, w, b)
        return self._conv_forward(x, self.weight, self.bias)


_PAD_RGB = os.environ.get("PTDT_PAD_RGB", "1") != "0"
