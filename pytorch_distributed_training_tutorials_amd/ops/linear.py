"""Linear layer on the native MFMA GEMM (csrc/kernels/gemm.hip).

Reference call sites: ``torch.nn.Linear`` in every model of the reference
(``ddp_gpus.py:81`` Linear(20,1); ``SampleModel`` Linear(32,2) NB01:168-175;
``ToyModel`` Linear(10000,10)+ReLU+Linear(10,5) NB03:440-450; ResNet-50 ``fc``
2048->1000 NB03:560). SURVEY K1/K3/K6/K8/K10/K11/K13.

Forward  : y = act(x W^T + b)         -- one launch, bias + ReLU in the epilogue
Backward : dx = (dy * relu'(y)) W      -- ReLU mask applied while staging dy
           dW = (dy * relu'(y))^T x    -- same mask, bias grad = row sums of the
           db = sum_rows(dy * relu'(y))   staged operand, fused in the dW launch
Long-K / tiny-MN shapes (ToyModel's K=10000, M=20, N=10) run split-K over
workgroups with fp32 atomics so the launch has enough workgroups to fill the
chip instead of one workgroup walking 10000 columns.
Large bf16 shapes (K % 64 == 0, >= 2^24 MACs) run the LDS-DMA kernel
(csrc/kernels/gemm_big.hip: 256x256 tiles ~1.1 PFLOP/s at 4096^3, 128x128 tiles
and split-K when fewer tiles than CUs, ``plan_big``): the forward directly on
nn.Linear's [out, in] weight, the backward GEMMs on K-contiguous copies (the
transposes cost a few % of the GEMM), with the ReLU mask and bias gradient as
separate elementwise / column-sum kernels.
CPU tensors use ``torch.nn.functional.linear`` (plumbing tests only).

Library GEMMs: the task's rule is "hand-written kernels for the fused hot ops,
hipBLASLt only for plain library GEMMs". A large bf16 GEMM whose only epilogue is
a bias (or nothing) is such a plain GEMM, and on those hipBLASLt measures ahead of
gemm_big.hip (profiles/r2_gemm_bench.jsonl: 1.45-1.59 vs 1.14-1.20 PFLOP/s at
4096^3 / 8192^3, 766 vs 560 TFLOP/s at 2048^3). It is not ahead everywhere:
hipBLASLt picks a weak tiling for 4096x11008x4096 (917 vs 1070 TFLOP/s native) and
ties at 1024^3. ``PTDT_LINEAR_GEMM`` picks the engine for plain bf16 GEMMs of
>= 2^24 MACs: ``auto`` (default) times both engines once per (M, N, K, transpose
form) on first use -- like MIOpen's find / cudnn.benchmark -- and keeps the faster
(during hipGraph capture an untuned shape takes hipBLASLt); ``native`` (always
gemm_big.hip) or ``library`` (always hipBLASLt). Everything fused or small stays on
the native kernels: fp32, ReLU epilogues and masks, split-K toy shapes.
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from .._ext import native, use_native

_KTILE = {torch.float32: 16, torch.bfloat16: 32}
_CUS = 256


def _split_k(M: int, N: int, K: int, dtype) -> int:
    """Split K when the output tile grid cannot fill the chip and K is long."""
    tiles = math.ceil(M / 64) * math.ceil(N / 64)
    ktiles = math.ceil(K / _KTILE.get(dtype, 32))
    if tiles >= 64 or ktiles < 8:
        return 1
    want = max(1, min(ktiles // 4, _CUS // tiles))
    return int(want)


_BIG_MIN_MACS = 1 << 24


def _big(M: int, N: int, K: int, dtype) -> bool:
    """Use the LDS-DMA kernel: bf16 with enough work (K not a multiple of its 64-deep
    K-tile is zero-padded by gemm_nt_big, e.g. ResNet fc's dx with K = 1000 classes)."""
    return dtype == torch.bfloat16 and K >= 64 and M * N * K >= _BIG_MIN_MACS


def _engine() -> str:
    e = os.environ.get("PTDT_LINEAR_GEMM", "auto").lower()
    if e not in ("auto", "native", "library"):
        raise ValueError(f"PTDT_LINEAR_GEMM must be auto, native or library, got {e!r}")
    return e


_TUNED: dict = {}


def _time(fn, reps: int = 3) -> float:
    fn()  # warm-up (and the hipBLASLt heuristic query)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e)


def _library(relu: bool = False, key=None, native_fn=None, library_fn=None) -> bool:
    """Plain big bf16 GEMM on hipBLASLt? (``_big`` is checked by the caller.) Under ``auto`` a
    shape ``key`` with both engines' thunks is timed once and the winner cached."""
    e = _engine()
    if e != "auto":
        return e == "library"
    if relu:
        return False
    if key is None or native_fn is None or library_fn is None:
        return True
    from ..utils import tuning

    hit = tuning.lookup("linear", key)  # (a decision valid here: see tuning.lookup)
    if hit is not None:
        return hit == "library"
    pin = tuning.pinned("linear", key)
    if pin is not None:
        return pin == "library"
    if torch.cuda.is_current_stream_capturing():
        return True  # no timing inside a capture; the shape stays untuned
    local = tuning.local_choice("linear", key)
    if local is None:
        local = "library" if _time(library_fn) <= _time(native_fn) else "native"
    # every DDP rank takes rank 0's engine (replicas must stay bit-identical; utils/tuning.py)
    return tuning.agree("linear", key, local, ("native", "library"), torch.cuda.current_device()) == "library"


def plan_big(M: int, N: int, K: int) -> tuple[int, int]:
    """(block tile, split-K) for gemm_big.hip, from profiles/r1_gemm_bench_v2.jsonl:
    256x256 tiles when they fill the 256 CUs; else 128x128 tiles (two workgroups
    per CU); split-K only when one slice-less 128 pass would run long (the zero
    fill + f32 atomics + cast cost ~10 us), at most one workgroup per CU and
    >= 4 K-tiles per slice."""
    nk = K // 64
    t256 = math.ceil(M / 256) * math.ceil(N / 256)
    if t256 >= _BIG256_MIN_TILES:
        return 256, 1
    t128 = math.ceil(M / 128) * math.ceil(N / 128)
    waves = math.ceil(t128 / (2 * _CUS))
    est_us = _KTILE_US * nk * waves
    if t128 >= _CUS or est_us < _SPLIT_MIN_US:
        return 128, 1
    split = max(1, min(_CUS // t128, nk // 4, 16))
    return 128, split


_BIG256_MIN_TILES = 192
_KTILE_US = 0.85      # one 128x128x64 K-tile step of a workgroup (measured, 2048^3)
_SPLIT_MIN_US = 25.0


def gemm_nt_big(A: torch.Tensor, Bt: torch.Tensor, out_dtype, bias=None, relu: bool = False,
                plan: tuple[int, int] | None = None) -> torch.Tensor:
    """C = A @ Bt^T on the LDS-DMA kernel (A [M,K], Bt [N,K], both made K-contiguous)."""
    K = A.shape[1]
    if K % 64:  # zero-pad K to the kernel's K-tile (one copy of each operand, made anyway when strided)
        A = F.pad(A, (0, 64 - K % 64))
        Bt = F.pad(Bt, (0, 64 - K % 64))
    A = A if A.stride(-1) == 1 and A.stride(0) % 8 == 0 else A.contiguous()
    Bt = Bt if Bt.stride(-1) == 1 and Bt.stride(0) % 8 == 0 else Bt.contiguous()
    M, N = A.shape[0], Bt.shape[0]
    tile, split = plan or plan_big(M, N, A.shape[1])
    if split > 1:  # fp32 atomics into a zeroed accumulator, ReLU/cast after
        acc = torch.zeros((M, N), device=A.device, dtype=torch.float32)
        native().gemm_big_(A, Bt, acc, bias, False, tile=tile, split_k=split)
        if relu:
            acc.relu_()
        return acc if out_dtype == torch.float32 else acc.to(out_dtype)
    C = torch.empty((M, N), device=A.device, dtype=out_dtype)
    native().gemm_big_(A, Bt, C, bias, relu, tile=tile)
    return C


def gemm(A: torch.Tensor, B: torch.Tensor, out: torch.Tensor | None = None, *, bias=None, amask=None,
         relu: bool = False, alpha: float = 1.0, beta: float = 0.0, colsum=None, out_dtype=None):
    """C = alpha*A@B (+beta*C) (+bias) (relu) on MFMA, with optional split-K."""
    M, K = A.shape
    N = B.shape[1]
    odt = out_dtype or (out.dtype if out is not None else A.dtype)
    split = _split_k(M, N, K, A.dtype) if beta == 0.0 else 1
    C = _ext_gemm(A, B, out, odt, bias, amask, relu, alpha, beta, colsum, split)
    return C


def _ext_gemm(A, B, out, odt, bias, amask, relu, alpha, beta, colsum, split):
    C_ = native()
    if split > 1:
        acc = torch.zeros((A.shape[0], B.shape[1]), device=A.device, dtype=torch.float32)
        C_.gemm_(A, B, acc, bias, amask, False, alpha, 0.0, colsum, split)
        if relu:
            acc.relu_()
        if out is None:
            return acc if odt == torch.float32 else acc.to(odt)
        out.copy_(acc)
        return out
    if out is None:
        out = torch.empty((A.shape[0], B.shape[1]), device=A.device, dtype=odt)
    C_.gemm_(A, B, out, bias, amask, relu, alpha, beta, colsum, 1)
    return out


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, relu: bool):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1])
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        M, K = x2.shape
        big = _big(M, weight.shape[0], K, x2.dtype)
        lib_b = bias.to(x2.dtype) if (big and bias is not None) else bias
        if big and _library(relu, ("nt", M, weight.shape[0], K),
                            lambda: gemm_nt_big(x2, weight, x.dtype, bias=bias),
                            lambda: F.linear(x2, weight, lib_b)):
            y = F.linear(x2, weight, lib_b)  # hipBLASLt (+bias epilogue)
            if relu:
                y = y.relu_()
        elif big:
            y = gemm_nt_big(x2, weight, x.dtype, bias=bias, relu=relu)
        else:
            y = gemm(x2, weight.t(), bias=bias, relu=relu, out_dtype=x.dtype)
        ctx.relu = relu
        ctx.has_bias = bias is not None
        ctx.bias_dtype = bias.dtype if bias is not None else None
        ctx.in_shape = shape
        ctx.save_for_backward(x2, weight, y if relu else None)
        return y.reshape(*shape[:-1], weight.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, weight, y = ctx.saved_tensors
        dy2 = dy.reshape(-1, weight.shape[0])
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        mask = y if ctx.relu else None
        dx = dw = db = None
        M, Nout, Kin = dy2.shape[0], weight.shape[0], weight.shape[1]
        big_dx = _big(M, Kin, Nout, dy2.dtype)
        big_dw = _big(Nout, Kin, M, dy2.dtype)
        if big_dx or big_dw:
            C_ = native()
            g = C_.relu_bwd(dy2, mask) if mask is not None else dy2
            if ctx.needs_input_grad[0]:
                if big_dx and _library(False, ("nn", M, Kin, Nout), lambda: gemm_nt_big(g, weight.t(), x2.dtype),
                                       lambda: torch.matmul(g, weight)):
                    dx = torch.matmul(g, weight).reshape(ctx.in_shape)
                else:
                    dx = (gemm_nt_big(g, weight.t(), x2.dtype) if big_dx else
                          gemm(g, weight, out_dtype=x2.dtype)).reshape(ctx.in_shape)
            if ctx.needs_input_grad[1]:
                if big_dw and _library(False, ("tn", Nout, Kin, M), lambda: gemm_nt_big(g.t(), x2.t(), weight.dtype),
                                       lambda: torch.matmul(g.t(), x2)):
                    dw = torch.matmul(g.t(), x2)
                else:
                    dw = gemm_nt_big(g.t(), x2.t(), weight.dtype) if big_dw else gemm(g.t(), x2, out_dtype=weight.dtype)
            if ctx.has_bias and ctx.needs_input_grad[2]:
                cs = torch.empty(Nout, device=dy.device, dtype=torch.float32)
                C_.col_sum_(g, cs, False)
                db = cs if ctx.bias_dtype == torch.float32 else cs.to(ctx.bias_dtype)
            return dx, dw, db, None
        if ctx.needs_input_grad[0]:
            dx = gemm(dy2, weight, amask=mask, out_dtype=x2.dtype).reshape(ctx.in_shape)
        if ctx.needs_input_grad[1] or (ctx.has_bias and ctx.needs_input_grad[2]):
            colsum = None
            if ctx.has_bias and ctx.needs_input_grad[2]:
                colsum = torch.zeros(weight.shape[0], device=dy.device, dtype=torch.float32)
            dw = gemm(dy2.t(), x2, amask=mask.t() if mask is not None else None, colsum=colsum,
                      out_dtype=weight.dtype)
            if colsum is not None:
                db = colsum if ctx.bias_dtype == torch.float32 else colsum.to(ctx.bias_dtype)
            if not ctx.needs_input_grad[1]:
                dw = None
        return dx, dw, db, None


def linear(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None = None, relu: bool = False):
    """``relu?(x @ weight.T + bias)``: native MFMA path on GPU, ATen on CPU."""
    if use_native(x, weight):
        if torch.is_autocast_enabled("cuda"):
            # autocast region: compute in the autocast dtype on MFMA, grads flow
            # back to the fp32 master weight through the differentiable casts
            # (the weight's through ops.conv.cast_weight: DDP bucket grad sink)
            dt = torch.get_autocast_dtype("cuda")
            if dt == torch.bfloat16:
                from .conv import cast_weight

                x, weight = x.to(dt), cast_weight(weight)
        if x.dtype not in (torch.float32, torch.bfloat16) or weight.dtype != x.dtype:
            raise TypeError(f"native linear supports fp32/bf16 with matching dtypes, got {x.dtype}/{weight.dtype}")
        return _LinearFn.apply(x, weight, bias, relu)
    y = F.linear(x, weight, bias)
    return F.relu(y) if relu else y


class Linear(nn.Linear):
    """Drop-in ``nn.Linear`` (same parameters, init and state_dict keys) whose
    GPU forward/backward run on the native MFMA kernels; ``relu=True`` fuses
    the activation into the epilogue."""

    def __init__(self, in_features: int, out_features: int, bias: bool = True, relu: bool = False,
                 device=None, dtype=None):
        super().__init__(in_features, out_features, bias=bias, device=device, dtype=dtype)
        self.relu = relu

    def forward(self, x):
        return linear(x, self.weight, self.bias, self.relu)

    def extra_repr(self) -> str:
        return super().extra_repr() + (", relu=True" if self.relu else "")
