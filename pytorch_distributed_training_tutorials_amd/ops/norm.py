"""BatchNorm with the ResNet epilogues fused: ``y = ReLU?(BN(x) + residual?)``,
and NHWC max pooling (the ResNet stem pool).

Reference call sites: every ``nn.BatchNorm2d`` of torchvision's ResNet-50
(NB03:560-570, ``ModelParallelResNet50`` NB03:807-833), each
followed by ``ReLU`` and, at the end of a Bottleneck, by the residual add.

On GPU with channels_last (NHWC) activations the training forward and backward
run on csrc/kernels/batchnorm.hip: statistics and the normalise / residual /
ReLU epilogue in two launches, the ReLU mask, both parameter gradients, the
input gradient and the residual gradient in two more -- instead of MIOpen's BN
kernels plus separate clamp, add, threshold-backward and tensor-op passes.
With a residual, the forward also writes the ReLU mask as bits (1/16 of the
activation in bf16) and the backward's reduce pass writes the masked gradient
(the residual gradient itself), so its apply pass reads that and x only.
Eval mode applies the running statistics in one launch. Anything else (NCHW,
CPU, momentum=None, odd channel counts) uses PyTorch's batch_norm with the same
semantics. Parameters, buffers and state_dict keys are nn.BatchNorm2d's.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .._ext import native


def _rows_layout_ok(x: torch.Tensor) -> bool:
    if not x.is_cuda or x.dtype not in (torch.float32, torch.bfloat16):
        return False
    vec = 4 if x.dtype == torch.float32 else 8
    if x.dim() < 2 or x.shape[1] % vec or x.data_ptr() % 16 or x.numel() == 0:
        return False
    if x.dim() == 2:
        return x.is_contiguous()
    return x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last)


def _like(t: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """t in x's memory layout (autograd hands back whatever the consumer produced)."""
    if t.stride() == x.stride():
        return t
    out = t.contiguous(memory_format=torch.channels_last) if x.dim() == 4 else t.contiguous()
    if out.stride() != x.stride():
        # size-1 dims (e.g. [B, C, 1, 1] after layer4 of a small-image ResNet) make several stride
        # tuples "contiguous" for one layout, and .contiguous() keeps t's: copy into x's exact strides
        out = torch.empty_strided(x.shape, x.stride(), dtype=t.dtype, device=t.device).copy_(t)
    return out


class ResidualLink:
    """Hand-over of a residual gradient between two fused BNs (a ResNet identity
    shortcut): the BN that adds ``residual`` (block k+1's bn3) stores the
    residual's gradient here instead of returning it to autograd, and the BN that
    produced ``residual`` (block k's bn3) adds it to its incoming gradient inside
    its backward kernels -- replacing autograd's separate add of the two
    gradients of the shared activation (two reads and a write of it).

    Ordering is autograd's own: the producer's backward runs only after every
    consumer of its output, the linking BN included, has run its backward. Each
    backward pass (a retained graph may run several) re-delivers: the consumer
    stores, the producer takes and clears; None means the consumer did not run.

    Streams: autograd runs each backward on its forward's stream and synchronises the
    gradients it passes along graph edges, but not this side channel. A link can span two
    streams (a pipeline's stage streams on one device, where the stage hop ``a.to(dev)`` is
    the same tensor and keeps its link), so the stream that produced the stored value is
    recorded and the taker waits for it when it runs elsewhere (``take``). A second delivery
    adds on ITS stream after waiting for the first one's, and the sum's stream becomes the
    recorded one (the round-5 version kept the first deliverer's: a taker on that stream skipped
    the wait for the add, one on a third stream waited on the wrong stream)."""

    __slots__ = ("dres", "stream")

    def __init__(self):
        self.dres = None
        self.stream = None

    def put(self, g):
        """Store (or, when already delivered, add) a consumer's residual gradient."""
        if self.dres is None:
            self.dres = g
            self.stream = torch.cuda.current_stream(g.device) if g.is_cuda else None
        else:
            self._sync(g.device)
            self.dres = self.dres + g
            self.stream = torch.cuda.current_stream(g.device) if g.is_cuda else None  # the sum's producer

    def take(self, device):
        """The delivered gradient (None if no consumer ran), ordered after its producer's stream."""
        g, self.dres = self.dres, None
        if g is not None:
            self._sync(device, g)
        self.stream = None
        return g

    def _sync(self, device, g=None):
        if self.stream is None or device.type != "cuda":
            return
        cur = torch.cuda.current_stream(device)
        if cur != self.stream:
            cur.wait_stream(self.stream)
            t = g if g is not None else self.dres
            t.record_stream(cur)


class _BatchNormActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, residual, running_mean, running_var, nbt, relu: bool, momentum: float,
                eps: float, tickets, link_in, link_out, stats_in=None, conv_link=None):
        # with a residual the ReLU mask travels as bits (one byte per 16-B vector, 1/16 of y in
        # bf16); without one it is recomputed from x and the saved scale/shift (bit-exact)
        want_mask = relu and residual is not None
        if stats_in is not None:  # statistics from the producing 1x1 conv's epilogue (ops/convbn.py)
            stats = stats_in
            y, mask = native().bn_fwd_apply(x, stats, residual, relu, want_mask)
        else:
            y, stats, mask = native().bn_fwd_train(x, weight, bias, running_mean, running_var, nbt, residual, relu,
                                                   momentum, eps, tickets, want_mask)
        ctx.tickets = tickets
        ctx.params = (weight, bias)
        ctx.relu = relu
        ctx.has_res = residual is not None
        ctx.link_in, ctx.link_out = link_in, link_out
        ctx.conv_link = conv_link
        ctx.save_for_backward(x, mask if want_mask else None, weight, stats)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mask, weight, stats = ctx.saved_tensors
        want_dw = weight is not None and (ctx.needs_input_grad[1] or ctx.needs_input_grad[2])
        link_in, link_out = ctx.link_in, ctx.link_out
        # a bit mask is read by the backward's materialised-gradient path, which writes the
        # residual gradient: request it whenever the mask exists
        want_dres = ctx.has_res and (ctx.needs_input_grad[3] or link_in is not None or mask is not None)
        dy = _like(dy, x)
        dy2 = None
        if link_out is not None:  # a later block's residual gradient of our output
            # (None: that block's backward did not run -- its output does not reach the loss)
            dy2 = link_out.take(dy.device)
            if dy2 is not None and dy2.stride() != dy.stride():
                dy, dy2 = dy + dy2, None
        sinks = [None, None]
        if want_dw:  # DDP grad sinks (ops/conv.py): write dweight/dbias straight into the bucket slots
            for k, p in enumerate(ctx.params):
                if p is not None and p.grad is None and getattr(p, "_ptdt_grad_sink", None) is not None:
                    sinks[k] = p._ptdt_grad_sink()
        clink = ctx.conv_link
        if clink is not None and ctx.needs_input_grad[0]:
            # reduce pass only: the producing 1x1 conv applies dY = A g + B x + C inside its fused
            # backward (ops/convbn.py ConvBwdLink); g doubles as the residual gradient
            g, dw, db, clink.coef = native().bn_bwd_reduce(dy, x, weight, stats, ctx.relu, want_dw, ctx.tickets,
                                                           sinks[0], sinks[1], dy2, mask)
            dx, dres = g, (g.view_as(g) if want_dres else None)
        else:
            dx, dw, db, dres = native().bn_bwd(dy, x, None, weight, stats, ctx.relu, want_dres, want_dw,
                                               ctx.tickets, sinks[0], sinks[1], dy2, mask)
        if link_in is not None and dres is not None:  # delivered to the residual's producer instead of autograd
            if link_in.dres is None:
                link_in.put(dres)
                dres = None
            elif not ctx.needs_input_grad[3]:  # the link is taken (another consumer delivered): sum into it
                link_in.put(dres)
                dres = None
            # else: autograd adds this one (returned below), as _GradLinkFn does
        return (dx if ctx.needs_input_grad[0] else None, dw if want_dw else None, db if want_dw else None,
                dres if (dres is not None and ctx.needs_input_grad[3]) else None, *([None] * 11))


class _GradLinkFn(torch.autograd.Function):
    """Identity whose backward hands its gradient to ``x``'s producing fused BN (the same
    :class:`ResidualLink` an identity shortcut uses) instead of returning it to autograd."""

    @staticmethod
    def forward(ctx, x, link):
        ctx.link = link
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        link = ctx.link
        if link.dres is None:  # delivered: the producer adds it as dy2 inside its backward kernels
            link.put(g)
            return None, None
        return g, None  # the link is taken (another consumer delivered): autograd adds this one


def grad_link(x: torch.Tensor) -> torch.Tensor:
    """``x`` for a second consumer branch whose gradient should be summed inside the backward of
    the fused BN that produced ``x`` (one extra read there) rather than by autograd's add kernel
    (two reads and a write of an activation). ResNet's downsample blocks feed their input to conv1
    and to the downsample conv; with the link the two input gradients meet in the previous block's
    bn3 backward. A tensor without a producing fused BN (or outside autograd) passes through."""
    link = getattr(x, "_ptdt_res_link", None)
    if link is None or not torch.is_grad_enabled() or not x.requires_grad:
        return x
    return _GradLinkFn.apply(x, link)


def _tickets_of(bn, x):
    """The module's zeroed ticket array for the kernels' last-block hand-off (None: per-device one)."""
    t = getattr(bn, "_bn_tickets", None)
    if t is None or t.device != x.device:
        return None
    return t


def batch_norm_act(x: torch.Tensor, bn: nn.modules.batchnorm._BatchNorm, residual: torch.Tensor | None = None,
                   relu: bool = False, link: bool = False, stats: torch.Tensor | None = None,
                   conv_link=None) -> torch.Tensor:
    """``ReLU?(bn(x) + residual)`` with ``bn``'s parameters, buffers and train/eval mode.

    ``link=True``: when ``residual`` is the output of another fused BN, its gradient
    is handed to that BN's backward kernels (:class:`ResidualLink`) instead of being
    added to the residual's other gradients by autograd. Only for a residual whose
    producer is a fused BN (a ResNet identity shortcut).

    ``stats``: this batch's [4, C] statistics (mean, invstd, scale, shift) already computed --
    and the running statistics already updated -- by the kernel that produced ``x``
    (ops/convbn.py); only the apply pass runs. Training mode, native layout only."""
    fast = _rows_layout_ok(x) and (residual is None or (residual.dtype == x.dtype and residual.shape == x.shape
                                                        and residual.stride() == x.stride()
                                                        and residual.data_ptr() % 16 == 0))
    use_batch_stats = bn.training or not bn.track_running_stats
    if fast and use_batch_stats and bn.momentum is not None:
        track = bn.training and bn.track_running_stats
        link_in = getattr(residual, "_ptdt_res_link", None) if (link and residual is not None) else None
        link_out = ResidualLink() if torch.is_grad_enabled() else None
        y = _BatchNormActFn.apply(x, bn.weight, bn.bias, residual, bn.running_mean if track else None,
                                  bn.running_var if track else None, bn.num_batches_tracked if track else None,
                                  relu, float(bn.momentum), float(bn.eps), _tickets_of(bn, x), link_in, link_out,
                                  stats, conv_link)
        if link_out is not None:
            y._ptdt_res_link = link_out
        return y
    if stats is not None:
        raise RuntimeError("batch_norm_act: precomputed statistics need the native training path")
    needs_grad = torch.is_grad_enabled() and (x.requires_grad or (residual is not None and residual.requires_grad))
    if fast and not use_batch_stats and not needs_grad:  # eval: one launch with the running statistics
        scale = torch.rsqrt(bn.running_var.float() + bn.eps)
        if bn.weight is not None:
            scale = scale * bn.weight.float()
        shift = -bn.running_mean.float() * scale
        if bn.bias is not None:
            shift = shift + bn.bias.float()
        return native().bn_apply(x, residual, scale.contiguous(), shift.contiguous(), relu)
    if bn.training and bn.track_running_stats and bn.num_batches_tracked is not None:
        bn.num_batches_tracked.add_(1)
    momentum = bn.momentum
    if bn.training and bn.track_running_stats and momentum is None:  # cumulative moving average
        momentum = 1.0 / float(bn.num_batches_tracked)
    y = F.batch_norm(x, bn.running_mean if not bn.training or bn.track_running_stats else None,
                     bn.running_var if not bn.training or bn.track_running_stats else None, bn.weight, bn.bias,
                     use_batch_stats, momentum if momentum is not None else 0.0, bn.eps)
    if residual is not None:
        y = y + residual
    return F.relu(y) if relu else y


class BatchNorm2d(nn.BatchNorm2d):
    """Drop-in ``nn.BatchNorm2d`` (same parameters, buffers, state_dict keys) whose
    ``forward(x, residual=None, relu=False)`` fuses the residual add and ReLU and
    runs on the native NHWC kernels for channels_last GPU activations."""

    def __init__(self, num_features: int, *args, **kwargs):
        super().__init__(num_features, *args, **kwargs)
        # zeroed int32 tickets for the kernels' last-block hand-off (re-armed in-kernel), one per
        # channel tile (>= 32 channels); non-persistent: not part of the state_dict
        self.register_buffer("_bn_tickets", torch.zeros(max(1, -(-num_features // 32)), dtype=torch.int32),
                             persistent=False)
        # tickets of the statistics merge when a 1x1 conv's epilogue computes this BN's statistics
        # (ops/convbn.py; (merge groups + 1) x column tiles, re-armed in-kernel)
        self.register_buffer("_gemm_tickets", torch.zeros(1024, dtype=torch.int32), persistent=False)

    def forward(self, x, residual=None, relu: bool = False, link: bool = False):
        self._check_input_dim(x)
        return batch_norm_act(x, self, residual, relu, link)


# ----------------------------------------------------------------------------- pooling
class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        y, arg = native().maxpool2d_fwd(x, k, s, p)
        ctx.save_for_backward(arg)
        ctx.cfg = (list(x.shape), k, s, p)
        return y

    @staticmethod
    def backward(ctx, gy):
        (arg,) = ctx.saved_tensors
        size, k, s, p = ctx.cfg
        gy = gy.contiguous(memory_format=torch.channels_last)
        return native().maxpool2d_bwd(gy, arg, size, k, s, p), None, None, None


def _pair(v):
    return [int(v), int(v)] if isinstance(v, int) else [int(t) for t in v]


def _pool_cfg(pool: nn.MaxPool2d, x: torch.Tensor):
    """(k, s, p) when the native NHWC pool applies to ``x``, else None."""
    k, s, p = _pair(pool.kernel_size), _pair(pool.stride or pool.kernel_size), _pair(pool.padding)
    d = _pair(pool.dilation)
    vec = 4 if x.dtype == torch.float32 else 8
    if (x.is_cuda and x.dim() == 4 and x.dtype in (torch.float32, torch.bfloat16) and d == [1, 1]
            and not pool.ceil_mode and not pool.return_indices and x.shape[1] % vec == 0
            and x.is_contiguous(memory_format=torch.channels_last) and x.data_ptr() % 16 == 0
            and 2 * p[0] <= k[0] and 2 * p[1] <= k[1]):
        return k, s, p
    return None


class _BnReluPoolFn(torch.autograd.Function):
    """maxpool(ReLU(BN(x))) in two launches: the BN statistics, then the pool applying
    ReLU(x * scale + shift) to every value it loads -- the normalised activation (the ResNet stem's
    [B, 64, 112, 112]) is never written or re-read. Backward: the pool's gather, then the BN backward
    with the ReLU mask recomputed from x (bit-exact with the fused apply)."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, nbt, momentum: float, eps: float, tickets, k, s, p):
        _, stats, _ = native().bn_fwd_train(x, weight, bias, running_mean, running_var, nbt, None, True, momentum,
                                            eps, tickets, False, True)
        y, arg = native().maxpool2d_fwd(x, k, s, p, stats[2], stats[3], True)
        ctx.save_for_backward(x, arg, weight, stats)
        ctx.cfg = (k, s, p)
        ctx.tickets = tickets
        ctx.params = (weight, bias)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, arg, weight, stats = ctx.saved_tensors
        k, s, p = ctx.cfg
        dy = native().maxpool2d_bwd(gy.contiguous(memory_format=torch.channels_last), arg, list(x.shape), k, s, p)
        want_dw = weight is not None and (ctx.needs_input_grad[1] or ctx.needs_input_grad[2])
        sinks = [None, None]
        if want_dw:  # DDP grad sinks: dweight/dbias straight into the bucket slots
            for i, prm in enumerate(ctx.params):
                if prm is not None and prm.grad is None and getattr(prm, "_ptdt_grad_sink", None) is not None:
                    sinks[i] = prm._ptdt_grad_sink()
        dx, dw, db, _ = native().bn_bwd(dy, x, None, weight, stats, True, False, want_dw, ctx.tickets, sinks[0],
                                        sinks[1], None, None)
        return (dx if ctx.needs_input_grad[0] else None, dw if want_dw else None, db if want_dw else None,
                *([None] * 9))


def bn_relu_maxpool(x: torch.Tensor, bn: nn.Module, pool: nn.MaxPool2d) -> torch.Tensor:
    """``pool(ReLU(bn(x)))`` (the ResNet stem): fused for an ops.norm.BatchNorm2d in training over a
    channels_last GPU activation (PTDT_BN_POOL=0 disables), composed otherwise."""
    cfg = _pool_cfg(pool, x) if _BN_POOL else None
    if (cfg is None or not isinstance(bn, BatchNorm2d) or not bn.training or bn.momentum is None
            or not _rows_layout_ok(x)):
        y = bn(x, relu=True) if isinstance(bn, BatchNorm2d) else torch.relu(bn(x))
        return pool(y)
    track = bn.track_running_stats
    return _BnReluPoolFn.apply(x, bn.weight, bn.bias, bn.running_mean if track else None,
                               bn.running_var if track else None, bn.num_batches_tracked if track else None,
                               float(bn.momentum), float(bn.eps), _tickets_of(bn, x), *cfg)


_BN_POOL = __import__("os").environ.get("PTDT_BN_POOL", "1") != "0"


class MaxPool2d(nn.MaxPool2d):
    """Drop-in ``nn.MaxPool2d``; channels_last GPU activations run on the native NHWC
    kernels (csrc/kernels/pool.hip: one-byte window argmax, gather backward)."""

    def forward(self, x):
        cfg = _pool_cfg(self, x)
        if cfg is not None:
            return _MaxPoolFn.apply(x, *cfg)
        return super().forward(x)
