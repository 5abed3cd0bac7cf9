"""device_map-style placement + int8 weight-only quantisation."""
import pytest
import torch

from pytorch_distributed_training_tutorials_amd.models.llama import build_llama
from pytorch_distributed_training_tutorials_amd.ops.quant import Int8Linear, quantize_int8_, quantize_rowwise
from pytorch_distributed_training_tutorials_amd.parallel.placement import (dispatch_model, infer_device_map,
                                                                          placement_report, placement_units)


def test_llama7b_meta_placement_over_4_devices_is_ordered_and_balanced():
    m = build_llama("7b", dtype=torch.float16, device="meta")
    assert sum(p.numel() for p in m.parameters()) == 6_738_415_616
    dmap = infer_device_map(m, ["cuda:0", "cuda:1", "cuda:2", "cuda:3"])
    names = list(dmap)
    assert names[0] == "model.embed_tokens" and names[-1] == "lm_head"
    devs = [int(d[-1]) for d in dmap.values()]
    assert devs == sorted(devs) and set(devs) == {0, 1, 2, 3}  # layer order preserved, all GPUs used
    layers = [n for n in names if n.startswith("model.layers.")]
    assert len(layers) == 32  # decoder layers are never split
    per = {d: sum(1 for n in layers if dmap[n] == f"cuda:{d}") for d in range(4)}
    assert all(6 <= v <= 10 for v in per.values()), per


def _param_index_ranges(model, dmap):
    def dev_of(pname):
        return dmap[max((k for k in dmap if pname == k or pname.startswith(k + ".")), key=len)]

    out = {}
    for i, (n, _) in enumerate(model.named_parameters()):
        out.setdefault(dev_of(n), [i, i])[1] = i
    return out


def test_llama7b_int8_auto_map_matches_reference_recording():
    """The reference's recorded device_map="auto" split of int8 Llama-7B over 4 GPUs
    (03.model_parallel.ipynb:114-404): embed + layers 0-5 on cuda:0 (parameter idx 0-54), 6-13 on
    cuda:1 (55-126), 14-21 on cuda:2 (127-198), 22-31 + norm + lm_head on cuda:3 (199-290)."""
    m = build_llama("7b", dtype=torch.float16, device="meta")
    names = [n for n, _ in m.named_parameters()]
    assert len(names) == 291
    devs = ["cuda:0", "cuda:1", "cuda:2", "cuda:3"]
    for cap in (None, 24 * 2 ** 30, 80 * 2 ** 30):  # independent of the (unrecorded) GPU capacity
        mm = None if cap is None else {d: cap for d in devs}
        dmap = infer_device_map(m, devs, max_memory=mm, linear_weight_bytes=1)
        assert _param_index_ranges(m, dmap) == {"cuda:0": [0, 54], "cuda:1": [55, 126], "cuda:2": [127, 198],
                                                "cuda:3": [199, 290]}
        layers = {d: sum(1 for n, v in dmap.items() if n.startswith("model.layers.") and v == d) for d in devs}
        assert layers == {"cuda:0": 6, "cuda:1": 8, "cuda:2": 8, "cuda:3": 10}
        assert dmap["model.embed_tokens"] == "cuda:0" and dmap["model.norm"] == dmap["lm_head"] == "cuda:3"
    # what is int8 and what stays fp16 after quantising (NB03:67-92): the 7 projections per layer
    from pytorch_distributed_training_tutorials_amd.parallel.placement import _bytes
    q = _bytes(m.model.layers[0], 1)
    assert q == (4 * 4096 * 4096 + 3 * 4096 * 11008) + 2 * 4096 * 2


def test_llama7b_auto_map_agrees_with_accelerate():
    """Cross-check against accelerate's own balanced planner (importable here, not used by the
    package): same budgets x 0.9 (the int8 loader's reserve), same map."""
    accel = pytest.importorskip("accelerate.utils")
    m = build_llama("7b", dtype=torch.float16, device="meta")
    special = {}
    for n, mod in m.named_modules():
        for pn, _ in mod.named_parameters(recurse=False):
            if not (isinstance(mod, torch.nn.Linear) and n != "lm_head"):
                special[f"{n}.{pn}" if n else pn] = torch.float16
    mm = {i: 64 * 2 ** 30 for i in range(4)}
    mm["cpu"] = 2 ** 40
    import warnings

    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        bal = accel.get_balanced_memory(m, max_memory=dict(mm), no_split_module_classes=["LlamaDecoderLayer"],
                                        dtype=torch.int8, special_dtypes=special)
        bal = {k: v * 0.9 for k, v in bal.items()}
        ref = accel.infer_auto_device_map(m, max_memory=bal, no_split_module_classes=["LlamaDecoderLayer"],
                                          dtype=torch.int8, special_dtypes=special)
    ours = infer_device_map(m, [f"cuda:{i}" for i in range(4)], max_memory={f"cuda:{i}": mm[i] for i in range(4)},
                            linear_weight_bytes=1)
    ref_ranges = _param_index_ranges(m, {k: f"cuda:{v}" for k, v in ref.items()})
    assert _param_index_ranges(m, ours) == ref_ranges


def test_placement_units_no_split():
    m = build_llama("tiny", dtype=torch.float32)
    units = [n for n, _ in placement_units(m)]
    assert "model.layers.0" in units and not any(n.startswith("model.layers.0.") for n in units)


def test_quantize_rowwise_cpu():
    w = torch.randn(64, 96)
    q, s = quantize_rowwise(w)
    assert q.dtype == torch.int8 and s.shape == (64,)
    assert (q.float() * s[:, None] - w).abs().max() <= s.max() * 0.5 + 1e-6


def test_tiny_llama_int8_dispatch_cpu_matches_fp32_closely():
    m = build_llama("tiny", dtype=torch.float32)
    x = torch.randint(0, 512, (2, 12))
    with torch.no_grad():
        ref = m(x).logits
    quantize_int8_(m)
    assert sum(isinstance(mod, Int8Linear) for mod in m.modules()) == 4 * 7
    dmap = infer_device_map(m, ["cpu", "cpu"])
    dispatch_model(m, dmap)
    with torch.no_grad():
        out = m(x).logits
    assert (out - ref).abs().max() / ref.abs().max() < 0.05
    rep = placement_report(m)
    assert rep[0][1] == "model.embed_tokens.weight"


@pytest.mark.gpu
def test_tiny_llama_int8_on_gpu_native_kernel():
    m = build_llama("tiny", dtype=torch.bfloat16)
    x = torch.randint(0, 512, (2, 12))
    with torch.no_grad():
        ref = m.float()(x).logits
    m = m.to(torch.bfloat16)
    quantize_int8_(m)
    dispatch_model(m, infer_device_map(m, ["cuda:0", "cuda:0"]))
    with torch.no_grad():
        out = m(x.cuda()).logits.float().cpu()
    assert (out - ref).abs().max() / ref.abs().max() < 0.08
