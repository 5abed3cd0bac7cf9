"""Int8 weight-only linear layers (LLM.int8-style row-wise absmax).

Reference: ``BitsAndBytesConfig(load_in_8bit=True)`` NB03:52-56 (SURVEY R24,
N8, K20): the 7 projection weights of every Llama layer are quantised to int8
when moved to the GPU; RMSNorm, embeddings and lm_head stay in 16-bit.

:class:`Int8Linear` stores ``weight_q`` (int8 ``[out, in]``) and per-row
``weight_scale`` (fp32); on GPU the forward is the native
``int8_weight_gemm`` kernel (int8 tile widened to bf16 in LDS, MFMA, scale in
the fp32 epilogue -- 1 byte per weight read from HBM). bitsandbytes' fp16
outlier decomposition is not reproduced: activations stay bf16/fp32, so no
activation quantisation error exists to decompose.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .._ext import native, use_native


def quantize_rowwise(w: torch.Tensor):
    """(int8 q, fp32 scale) with ``w ~= q * scale[:, None]``."""
    if use_native(w) and w.dtype in (torch.float32, torch.bfloat16):
        return tuple(native().quantize_int8(w.contiguous()))
    wf = w.float()
    amax = wf.abs().amax(dim=1)
    scale = torch.where(amax > 0, amax / 127.0, torch.ones_like(amax))
    q = torch.clamp(torch.round(wf / scale[:, None]), -127, 127).to(torch.int8)
    return q, scale


class Int8Linear(nn.Module):
    def __init__(self, in_features: int, out_features: int, bias: bool = True, dtype=torch.bfloat16, device=None):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.register_buffer("weight_q", torch.zeros(out_features, in_features, dtype=torch.int8, device=device))
        self.register_buffer("weight_scale", torch.ones(out_features, dtype=torch.float32, device=device))
        if bias:
            self.register_buffer("bias", torch.zeros(out_features, dtype=dtype, device=device))
        else:
            self.bias = None

    @classmethod
    def from_linear(cls, lin: nn.Linear) -> "Int8Linear":
        m = cls(lin.in_features, lin.out_features, lin.bias is not None, dtype=lin.weight.dtype,
                device=lin.weight.device)
        q, s = quantize_rowwise(lin.weight.detach())
        m.weight_q.copy_(q)
        m.weight_scale.copy_(s)
        if lin.bias is not None:
            m.bias.copy_(lin.bias.detach())
        return m

    def dequantized_weight(self) -> torch.Tensor:
        return self.weight_q.float() * self.weight_scale[:, None]

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        shape = x.shape
        x2 = x.reshape(-1, shape[-1])
        if use_native(x2) and x2.dtype in (torch.float32, torch.bfloat16):
            b = self.bias if self.bias is None or self.bias.dtype == x2.dtype else self.bias.to(x2.dtype)
            y = native().int8_linear(x2.contiguous(), self.weight_q, self.weight_scale, b)
        else:
            y = (x2.float() @ self.dequantized_weight().t()).to(x.dtype)
            if self.bias is not None:
                y = y + self.bias.to(y.dtype)
        return y.reshape(*shape[:-1], self.out_features)

    def extra_repr(self) -> str:
        return f"in_features={self.in_features}, out_features={self.out_features}, int8 row-wise"


def quantize_int8_(model: nn.Module, skip=("lm_head",)) -> nn.Module:
    """Replace every ``nn.Linear`` (except names ending in ``skip``) by Int8Linear, in place."""
    for name, mod in list(model.named_modules()):
        for cname, child in list(mod.named_children()):
            full = f"{name}.{cname}" if name else cname
            if isinstance(child, nn.Linear) and not any(full.endswith(s) for s in skip):
                setattr(mod, cname, Int8Linear.from_linear(child))
    return model
