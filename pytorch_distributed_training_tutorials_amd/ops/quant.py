"""Int8 weight-only linear layers (LLM.int8-style row-wise absmax).

Reference: ``BitsAndBytesConfig(load_in_8bit=True)`` NB03:52-56 (SURVEY R24,
N8, K20): the 7 projection weights of every Llama layer are quantised to int8
when moved to the GPU; RMSNorm, embeddings and lm_head stay in 16-bit.

:class:`Int8Linear` stores ``weight_q`` (int8 ``[out, in]``) and per-row
``weight_scale`` (fp32); on GPU the forward is the native
``int8_weight_gemm`` kernel (int8 tile widened to bf16 in LDS, MFMA, scale in
the fp32 epilogue -- 1 byte per weight read from HBM).

``llm_int8=True`` reproduces bitsandbytes' LLM.int8 matmul instead: the input
features with an activation above ``threshold`` (6.0, bitsandbytes' default) in
the batch are outliers and stay in 16/32-bit against the dequantised weight
columns; every other feature is quantised row-wise (absmax per token) to int8
and multiplied int8 x int8 -> int32 on MFMA (``v_mfma_i32_16x16x64_i8``,
csrc/kernels/int8_mm.hip), dequantised in the epilogue where the outlier product
and the bias are added. (Gathering the outlier columns reads their indices on
the host, as bitsandbytes does -- except at decode shapes, <= 32 tokens, where
csrc/kernels/int8_decode.hip fuses the outlier columns into an int8 GEMV: three
launches -- column statistics, row quantisation, GEMV -- and no host read.) fp32, bf16 and fp16 activations run natively
(the reference's load_in_8bit Llama is fp16); the plain-PyTorch
``llm_int8_reference`` is the CPU path and the numerics reference only.
"""
from __future__ import annotations

import weakref

import torch
import torch.nn as nn

from .._ext import native, use_native

_NATIVE_DTYPES = (torch.float32, torch.bfloat16, torch.float16)
_DECODE = __import__("os").environ.get("PTDT_INT8_DECODE", "1") != "0"  # 0: decode shapes take the GEMM path
_DTYPE_NAME = {torch.float32: "float32", torch.bfloat16: "bfloat16", torch.float16: "float16"}
# 0: the decode GEMV reads the row-major int8 weights instead of a pre-shuffled copy (A/B)
_PACKED = __import__("os").environ.get("PTDT_I8_PACKED", "1") != "0"


def quantize_rowwise(w: torch.Tensor):
    """(int8 q, fp32 scale) with ``w ~= q * scale[:, None]``."""
    if use_native(w) and w.dtype in _NATIVE_DTYPES:
        wq = w.float() if w.dtype == torch.float16 else w  # exact widening: same absmax and rounding
        return tuple(native().quantize_int8(wq.contiguous()))
    wf = w.float()
    amax = wf.abs().amax(dim=1)
    scale = torch.where(amax > 0, amax / 127.0, torch.ones_like(amax))
    q = torch.clamp(torch.round(wf / scale[:, None]), -127, 127).to(torch.int8)
    return q, scale


def llm_int8_reference(x: torch.Tensor, q: torch.Tensor, scale: torch.Tensor, bias: torch.Tensor | None,
                       threshold: float) -> torch.Tensor:
    """The LLM.int8 product in plain PyTorch (fp32 math, exact int32 products):
    the CPU path and the numerics reference of the native kernels."""
    xf = x.float()
    out_cols = xf.abs().amax(dim=0) > threshold
    xin = xf.masked_fill(out_cols[None, :], 0.0)
    amax = xin.abs().amax(dim=1)
    sx = torch.where(amax > 0, amax / 127.0, torch.ones_like(amax))
    xq = torch.clamp(torch.round(xin / sx[:, None]), -127, 127)
    prod = (xq.long().cpu() @ q.long().cpu().t()).to(torch.float32).to(x.device)
    y = prod * sx[:, None] * scale.float()[None, :]
    if bool(out_cols.any()):
        wdq = q[:, out_cols].float() * scale.float()[:, None]
        y = y + xf[:, out_cols] @ wdq.t()
    if bias is not None:
        y = y + bias.float()
    return y.to(x.dtype)


class Int8Linear(nn.Module):
    def __init__(self, in_features: int, out_features: int, bias: bool = True, dtype=torch.bfloat16, device=None,
                 llm_int8: bool = False, threshold: float = 6.0):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.llm_int8, self.threshold = llm_int8, float(threshold)
        self.register_buffer("weight_q", torch.zeros(out_features, in_features, dtype=torch.int8, device=device))
        self.register_buffer("weight_scale", torch.ones(out_features, dtype=torch.float32, device=device))
        if bias:
            self.register_buffer("bias", torch.zeros(out_features, dtype=dtype, device=device))
        else:
            self.bias = None

    @classmethod
    def from_linear(cls, lin: nn.Linear, llm_int8: bool = False, threshold: float = 6.0) -> "Int8Linear":
        m = cls(lin.in_features, lin.out_features, lin.bias is not None, dtype=lin.weight.dtype,
                device=lin.weight.device, llm_int8=llm_int8, threshold=threshold)
        q, s = quantize_rowwise(lin.weight.detach())
        m.weight_q.copy_(q)
        m.weight_scale.copy_(s)
        if lin.bias is not None:
            m.bias.copy_(lin.bias.detach())
        return m

    def dequantized_weight(self) -> torch.Tensor:
        return self.weight_q.float() * self.weight_scale[:, None]

    def invalidate_packed(self) -> None:
        """Drop the decode GEMV's pre-shuffled weight copy (rebuilt on the next decode call).
        Needed only after writes the version counter cannot see -- through ``weight_q.data``
        or another alias of the storage; ``load_state_dict`` calls it itself."""
        self._packed_cache = None

    def _load_from_state_dict(self, *args, **kwargs):
        super()._load_from_state_dict(*args, **kwargs)
        self.invalidate_packed()

    def _decode_packed(self, C):
        """The decode GEMV's pre-shuffled copy of ``weight_q`` (one contiguous KiB per wave load),
        rebuilt when the weights change: another tensor (a weak reference, so a recycled address
        cannot alias), an in-place update of ``weight_q`` itself (version counter), or an explicit
        :meth:`invalidate_packed` / ``load_state_dict``. Writes through ``weight_q.data`` bump a
        different version counter: call :meth:`invalidate_packed` after them."""
        w = self.weight_q
        cache = getattr(self, "_packed_cache", None)
        if cache is None or cache[0]() is not w or cache[1] != w._version or cache[2] != w.data_ptr():
            cache = (weakref.ref(w), w._version, w.data_ptr(), C.int8_decode_pack(w))
            self._packed_cache = cache
        return cache[3]

    def _llm_int8(self, x2: torch.Tensor) -> torch.Tensor:
        b = self.bias
        if not use_native(x2) or x2.dtype not in _NATIVE_DTYPES or self.in_features % 16 != 0:
            # CPU tensors, and GPU shapes / dtypes the int8 MFMA kernel has no instance for (its K step
            # is 16: e.g. in_features = 40): the plain-PyTorch LLM.int8 product, same numerics
            return llm_int8_reference(x2, self.weight_q, self.weight_scale, b, self.threshold)
        C = native()
        x2 = x2.contiguous()
        if _DECODE and C.int8_decode_supported(x2.shape[0], self.out_features, self.in_features):
            # decode shapes (<= 32 tokens): outliers, quantisation and the int8 GEMV with the outlier
            # columns fused, three launches, no host read (csrc/kernels/int8_decode.hip)
            return C.int8_decode(x2, self.weight_q, self.weight_scale, b, self.threshold, _DTYPE_NAME[x2.dtype],
                                 self._decode_packed(C) if _PACKED else None)
        mask = C.int8_col_outliers(x2, self.threshold)
        cols = mask.nonzero().flatten()  # host read: usually a handful of features
        xq, sx = C.int8_quant_rows(x2, mask if cols.numel() else None)
        addend = None
        if cols.numel():
            wdq = self.weight_q.index_select(1, cols).float() * self.weight_scale[:, None]
            addend = (x2.index_select(1, cols).float() @ wdq.t()).contiguous()
        return C.int8_mm(xq, sx, self.weight_q, self.weight_scale, addend, b, _DTYPE_NAME[x2.dtype])

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        shape = x.shape
        x2 = x.reshape(-1, shape[-1])
        if self.llm_int8:
            return self._llm_int8(x2).reshape(*shape[:-1], self.out_features)
        if use_native(x2) and x2.dtype in _NATIVE_DTYPES:
            # weight-only kernel: fp32 / bf16 activations; fp16 runs it in fp32 (exact widening) and
            # rounds the output back to fp16
            xin = x2.float() if x2.dtype == torch.float16 else x2
            b = self.bias if self.bias is None or self.bias.dtype == xin.dtype else self.bias.to(xin.dtype)
            y = native().int8_linear(xin.contiguous(), self.weight_q, self.weight_scale, b).to(x2.dtype)
        else:
            y = (x2.float() @ self.dequantized_weight().t()).to(x.dtype)
            if self.bias is not None:
                y = y + self.bias.to(y.dtype)
        return y.reshape(*shape[:-1], self.out_features)

    def extra_repr(self) -> str:
        mode = f"LLM.int8 threshold={self.threshold}" if self.llm_int8 else "int8 row-wise weights"
        return f"in_features={self.in_features}, out_features={self.out_features}, {mode}"


def quantize_int8_(model: nn.Module, skip=("lm_head",), llm_int8: bool = False, threshold: float = 6.0) -> nn.Module:
    """Replace every ``nn.Linear`` (except names ending in ``skip``) by Int8Linear, in place
    (``llm_int8``: bitsandbytes' LLM.int8 matmul with outlier decomposition)."""
    for name, mod in list(model.named_modules()):
        for cname, child in list(mod.named_children()):
            full = f"{name}.{cname}" if name else cname
            if isinstance(child, nn.Linear) and not any(full.endswith(s) for s in skip):
                setattr(mod, cname, Int8Linear.from_linear(child, llm_int8=llm_int8, threshold=threshold))
    return model
