"""1x1 convolution + training BatchNorm with the statistics computed in the convolution's
epilogue: ``ReLU?(BN(conv1x1(x)) + residual?)``.

A stride-1 1x1 convolution over an NHWC (channels_last) activation is a GEMM,
``Y[N*H*W, Cout] = X[N*H*W, Cin] . W[Cout, Cin]^T``, with both operands already
K-contiguous in memory. Two native kernels run it and, while each output value is
still in registers, reduce the output to per-channel sums for the BatchNorm:

* ``conv1x1_bn.hip`` (streaming; ResNet-50's layer1 shapes and, with the weights in
  <= 64 KiB slabs, 128 -> 512 and 256 -> 1024): persistent workgroups, weights
  resident in LDS, activation row blocks LDS-DMA'd ahead, 16-B output stores,
  per-lane sums about running-mean pivots;
* ``gemm_bn_stats`` in ``gemm_big.hip`` (tiled, any K % 64 == 0 shape): the
  LDS-DMA GEMM with centred per-wave partials in its epilogue.

Partials are merged in fixed order by the last workgroups to finish (two ticket
levels, sc1 hand-off), which also write the BN coefficients and update the running
statistics. The BN then runs only its apply pass (``bn_fwd_apply``): the separate
statistics pass -- a full read of the conv output -- is gone (bf16, batch 128:
-214 us per ResNet-50 step, profiles/r3_convbn.md).

Backward is unchanged: the BN's native backward, then the convolution's data and
weight gradients on MIOpen (``aten.convolution_backward``, as autograd would
call it). Forward numerics: the statistics are those of the stored bf16 output
(what the separate pass would read), merged in double.

Anything else -- stride 2, eval mode, fp32, NCHW, odd channel counts, CPU --
takes the unfused ``bn_act(bn, conv(x))``. Where both apply, ``PTDT_CONVBN=auto`` (default)
times the two once per shape on the live operands and keeps the faster (MIOpen's 1x1
forward kernels run close to HBM speed on some shapes, profiles/r3_convbn.md); ``on``
always fuses, ``off`` never does.

Reference call sites: the Bottleneck convolutions + BatchNorms of torchvision's
ResNet-50 (NB03:560-570, NB03:807-833).
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from .._ext import native
from .conv import cast_weight
from .norm import BatchNorm2d, batch_norm_act

_MODE = os.environ.get("PTDT_CONVBN", "auto")  # auto: per-shape timing decides; on / 1: always; off / 0: never
_ENABLED = _MODE not in ("0", "off")
_STREAM = os.environ.get("PTDT_CONVBN_STREAM", "1") != "0"
# fused backward (BN apply + 1x1 data and weight gradients, csrc/kernels/conv1x1_bwd.hip) where an
# instance exists; 0: the BN's full backward, then MIOpen's convolution_backward
_BWD = os.environ.get("PTDT_CONVBN_BWD", "1") != "0"
# A/B of single shapes: "KxN,KxN" (input x output channels) keep the unfused backward
_BWD_SKIP = {tuple(int(v) for v in t.split("x")) for t in os.environ.get("PTDT_CONVBN_BWD_SKIP", "").split(",") if t}
_CHOICE: dict[tuple, bool] = {}  # (M, K, N, tile) -> fused is faster (PTDT_CONVBN=auto)


def _tile(M: int, N: int, K: int) -> int:
    """0: the streaming kernel (memory-bound (K, N) instances: weights resident in LDS); else the
    tiled GEMM's block tile: 256x256 when those tiles fill the chip (>= 192 of them), else 128x128."""
    if _STREAM and native().conv1x1_bn_stream_supported(K, N):
        return 0
    return 256 if (-(-M // 256)) * (-(-N // 256)) >= 192 else 128


class ConvBwdLink:
    """Hand-over from a fused BN's backward to its producing 1x1 conv's backward (the fused backward,
    csrc/kernels/conv1x1_bwd.hip): the BN runs only its reduce pass and passes the masked gradient g
    down as "the gradient of y", leaving here the coefficients of its apply (dY = A g + B y + C); the
    conv's backward then computes dY on the fly inside its data- and weight-gradient GEMMs. None:
    the BN ran its full backward (the conv receives dY itself)."""

    __slots__ = ("coef",)

    def __init__(self):
        self.coef = None


class _Conv1x1StatsFn(torch.autograd.Function):
    """y = conv1x1(x, w) (NHWC bf16) and the [4, Cout] BN statistics of y (non-differentiable)."""

    @staticmethod
    def forward(ctx, x, w, bn_weight, bn_bias, running_mean, running_var, nbt, momentum: float, eps: float,
                tickets, tile: int, link=None):
        n, cin, h, wd = x.shape
        cout = w.shape[0]
        x2 = x.permute(0, 2, 3, 1).reshape(n * h * wd, cin)  # channels_last storage: a view
        y2, stats = native().conv1x1_bn_stats(x2, w.reshape(cout, cin), bn_weight, bn_bias, running_mean,
                                              running_var, nbt, momentum, eps, tickets, tile)
        ctx.link = link
        ctx.save_for_backward(x, w, y2 if link is not None else None)
        ctx.mark_non_differentiable(stats)
        return y2.view(n, h, wd, cout).permute(0, 3, 1, 2), stats

    @staticmethod
    def backward(ctx, gy, _gstats):
        x, w, y2 = ctx.saved_tensors
        link = ctx.link
        if link is not None and link.coef is not None:  # gy is the BN's masked gradient g (ConvBwdLink)
            coef, link.coef = link.coef, None
            n, cin, h, wd = x.shape
            cout = w.shape[0]
            g2 = gy.permute(0, 2, 3, 1).reshape(-1, cout)
            if not g2.is_contiguous():
                g2 = g2.contiguous()
            x2 = x.permute(0, 2, 3, 1).reshape(-1, cin)
            dx2, dw2 = native().conv1x1_bwd(g2, y2, x2, w.reshape(cout, cin), coef)
            dx = dx2.view(n, h, wd, cin).permute(0, 3, 1, 2) if ctx.needs_input_grad[0] else None
            dw = dw2.view(cout, cin, 1, 1) if ctx.needs_input_grad[1] else None
            return dx, dw, *([None] * 10)
        gy = gy.contiguous(memory_format=torch.channels_last)
        mask = [ctx.needs_input_grad[0], ctx.needs_input_grad[1], False]
        dx, dw, _ = torch.ops.aten.convolution_backward(gy, x, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1,
                                                        mask)
        return dx, dw, *([None] * 10)


def _fusable(conv: nn.Conv2d, bn: nn.Module, x: torch.Tensor, residual) -> bool:
    if not (_ENABLED and isinstance(bn, BatchNorm2d) and bn.training and bn.momentum is not None):
        return False
    if not (isinstance(conv, nn.Conv2d) and conv.kernel_size == (1, 1) and conv.stride == (1, 1)
            and conv.padding == (0, 0) and conv.dilation == (1, 1) and conv.groups == 1 and conv.bias is None
            and conv.padding_mode == "zeros"):
        return False
    if not (x.is_cuda and x.dim() == 4 and torch.is_autocast_enabled("cuda")
            and torch.get_autocast_dtype("cuda") == torch.bfloat16 and x.dtype == torch.bfloat16
            and x.is_contiguous(memory_format=torch.channels_last) and x.data_ptr() % 16 == 0):
        return False
    cin, cout = conv.in_channels, conv.out_channels
    if cin % 64 or cout % 8 or x.shape[0] * x.shape[2] * x.shape[3] >= 2 ** 31:
        return False
    if residual is not None:  # the BN's native path needs the residual in the output's layout
        n, _, h, w = x.shape
        if not (residual.dtype == torch.bfloat16 and tuple(residual.shape) == (n, cout, h, w)
                and residual.is_contiguous(memory_format=torch.channels_last) and residual.data_ptr() % 16 == 0):
            return False
    return True


def _time_us(fn, reps: int = 3) -> float:
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    best = float("inf")
    for _ in range(reps):
        s.record()
        fn()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) * 1e3)
    return best


def _fused_wins(x: torch.Tensor, w: torch.Tensor, tile: int) -> bool:
    """PTDT_CONVBN=auto: time, once per (M, K, N), the fused conv + statistics kernel + the BN apply
    pass against MIOpen's convolution + the BN's statistics and apply passes on the live operands
    (scratch statistics, no running-stat side effects), and keep the faster. Inside a graph capture an
    unseen shape keeps the unfused path."""
    n, cin, h, wd = x.shape
    cout = w.shape[0]
    key = (n * h * wd, cin, cout, tile)
    if _MODE in ("1", "on"):
        return True
    from ..utils import tuning

    hit = tuning.lookup("convbn", key)  # (a decision valid here: see tuning.lookup)
    if hit is not None:
        return hit == "fused"
    pin = tuning.pinned("convbn", key)
    if pin is not None:
        return pin == "fused"
    if torch.cuda.is_current_stream_capturing():
        return False
    local = tuning.local_choice("convbn", key)
    if local is not None:  # timed before outside any scope: agree it, no second timing
        return tuning.agree("convbn", key, local, ("unfused", "fused"), x.device) == "fused"
    C = native()
    x2 = x.detach().permute(0, 2, 3, 1).reshape(-1, cin)
    w2 = w.detach().reshape(cout, cin)
    tickets = torch.zeros(C.conv1x1_bn_num_tickets(key[0], cout, tile, cin), dtype=torch.int32, device=x.device)

    def fused():
        y2, st = C.conv1x1_bn_stats(x2, w2, None, None, None, None, None, 0.1, 1e-5, tickets, tile)
        C.bn_fwd_apply(y2, st, None, True, False)

    def plain():
        y = torch.nn.functional.conv2d(x.detach(), w.detach())
        C.bn_fwd_train(y, None, None, None, None, None, None, True, 0.1, 1e-5, None, False)

    with torch.no_grad():  # interleaved, best of 5 each; near-ties (< 3 %) keep MIOpen's path
        tf, tp = float("inf"), float("inf")
        for _ in range(5):
            tf, tp = min(tf, _time_us(fused, 1)), min(tp, _time_us(plain, 1))
    local = "fused" if tf < 0.97 * tp else "unfused"
    # rank 0's choice on every rank: DDP replicas must run the same BN statistics path (utils/tuning.py)
    return tuning.agree("convbn", key, local, ("unfused", "fused"), x.device) == "fused"


def conv_bn_act(conv: nn.Conv2d, bn: nn.Module, x: torch.Tensor, residual: torch.Tensor | None = None,
                relu: bool = False, link: bool = False) -> torch.Tensor:
    """``ReLU?(bn(conv(x)) + residual)``; a stride-1 1x1 ``conv`` feeding an ops.norm.BatchNorm2d in
    training under bf16 autocast computes the BN statistics in its GEMM epilogue."""
    if not _fusable(conv, bn, x, residual):
        from ..models.resnet import bn_act

        return bn_act(bn, conv(x), residual, relu, link)
    M = x.shape[0] * x.shape[2] * x.shape[3]
    tile = _tile(M, conv.out_channels, conv.in_channels)
    w = cast_weight(conv.weight)
    if not _fused_wins(x, w, tile):
        from ..models.resnet import bn_act

        return bn_act(bn, conv._conv_forward(x, w, None), residual, relu, link)
    track = bn.track_running_stats
    tickets = bn._gemm_tickets
    need = native().conv1x1_bn_num_tickets(M, conv.out_channels, tile, conv.in_channels)
    if tickets.numel() < need or tickets.device != x.device:
        raise RuntimeError(f"conv_bn_act: BN ticket buffer too small ({tickets.numel()} < {need}) or off-device")
    cin, cout = conv.in_channels, conv.out_channels
    clink = None
    if _BWD and torch.is_grad_enabled() and (cin, cout) not in _BWD_SKIP and native().conv1x1_bwd_supported(cin, cout):
        clink = ConvBwdLink()
    y, stats = _Conv1x1StatsFn.apply(x, w, bn.weight, bn.bias, bn.running_mean if track else None,
                                     bn.running_var if track else None, bn.num_batches_tracked if track else None,
                                     float(bn.momentum), float(bn.eps), tickets, tile, clink)
    return batch_norm_act(y, bn, residual, relu, link, stats=stats, conv_link=clink)


def conv1x1_stats_probe(x2: torch.Tensor, w2: torch.Tensor, tile: int | None = None):
    """Callable running the fused GEMM + statistics kernel alone on [M, K] x [N, K]^T (benchmarks)."""
    M, N, K = x2.shape[0], w2.shape[0], x2.shape[1]
    t = _tile(M, N, K) if tile is None else tile
    tickets = torch.zeros(native().conv1x1_bn_num_tickets(M, N, t, K), dtype=torch.int32, device=x2.device)
    return lambda: native().conv1x1_bn_stats(x2, w2, None, None, None, None, None, 0.1, 1e-5, tickets, t)
