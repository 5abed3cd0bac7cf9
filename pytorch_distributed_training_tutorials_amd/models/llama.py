"""Llama models for the big-model placement path (reference NB03:52-56).

The reference loads ``baffo32/decapoda-research-llama-7B-hf`` in int8 with
``device_map="auto"``. There is no network here, so models are built from a
``LlamaConfig`` with random weights (HF transformers' architecture, same
parameter names/shapes): ``preset="7b"`` is the reference's shape (32 layers,
hidden 4096, intermediate 11008, vocab 32000) and can be instantiated on the
``meta`` device to plan placement without allocating; ``"tiny"`` is for tests.
"""
from __future__ import annotations

import torch

PRESETS = {
    "7b": dict(vocab_size=32000, hidden_size=4096, intermediate_size=11008, num_hidden_layers=32,
               num_attention_heads=32, num_key_value_heads=32, max_position_embeddings=2048, rms_norm_eps=1e-6),
    "tiny": dict(vocab_size=512, hidden_size=128, intermediate_size=352, num_hidden_layers=4,
                 num_attention_heads=4, num_key_value_heads=4, max_position_embeddings=256, rms_norm_eps=1e-6),
}


def llama_config(preset: str = "tiny", **overrides):
    from transformers import LlamaConfig

    kw = dict(PRESETS[preset])
    kw.update(overrides)
    return LlamaConfig(**kw)


def build_llama(preset: str = "tiny", dtype=torch.bfloat16, device="cpu", seed: int = 0, **overrides):
    """Random-init ``LlamaForCausalLM`` (``device="meta"`` allocates nothing)."""
    from transformers import LlamaForCausalLM

    cfg = llama_config(preset, **overrides)
    torch.manual_seed(seed)
    with torch.device(device):
        model = LlamaForCausalLM(cfg)
    return model.to(dtype)
