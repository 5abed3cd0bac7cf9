"""LLM.int8 (bitsandbytes' load_in_8bit matmul; reference NB03:52-56):
outlier features in 16/32-bit, the rest int8 x int8 -> int32 on MFMA."""
import pytest
import torch


def _lin(K=64, N=48, seed=0):
    torch.manual_seed(seed)
    return torch.nn.Linear(K, N)


def test_llm_int8_reference_cpu_tracks_fp32_and_handles_outliers():
    from pytorch_distributed_training_tutorials_amd.ops.quant import Int8Linear

    lin = _lin()
    m = Int8Linear.from_linear(lin, llm_int8=True, threshold=6.0)
    x = torch.randn(9, 64)
    x[:, 5] *= 40.0  # an outlier feature: kept out of the int8 product
    y, ref = m(x), lin(x)
    assert (y - ref).abs().max() <= 0.02 * ref.abs().max()
    # without the decomposition the outlier column would dominate every row's absmax
    m_plain = Int8Linear.from_linear(lin, llm_int8=True, threshold=1e9)
    assert (m_plain(x) - ref).abs().max() > 2 * (y - ref).abs().max()


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(70, 50, 128), (64, 64, 64), (5, 130, 48), (129, 17, 256),
                                   (256, 384, 512), (130, 260, 384), (1, 300, 1024), (300, 7, 128)])
def test_int8_mm_exact_integer_products(dev, M, N, K):
    """v_mfma_i32_16x16x64_i8 operand map: exact int32 products (scales 1, f32 out); K % 128 == 0
    runs the LDS-staged tiled kernel (edge tiles included), the rest the direct one."""
    from pytorch_distributed_training_tutorials_amd._ext import native

    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randint(-127, 128, (M, K), generator=g, dtype=torch.int8)
    B = torch.randint(-127, 128, (N, K), generator=g, dtype=torch.int8)
    ref = (A.long() @ B.long().t()).float()
    y = native().int8_mm(A.to(dev), torch.ones(M, device=dev), B.to(dev), torch.ones(N, device=dev))
    assert torch.equal(y.cpu(), ref)


@pytest.mark.gpu
@pytest.mark.parametrize("out", ["float32", "bfloat16", "float16"])
def test_int8_mm_epilogue_dtypes(dev, out):
    """Scales, the outlier addend and a bias of the output dtype, rounded once into out."""
    from pytorch_distributed_training_tutorials_amd._ext import native

    M, N, K = 96, 200, 256
    g = torch.Generator().manual_seed(7)
    A = torch.randint(-127, 128, (M, K), generator=g, dtype=torch.int8)
    B = torch.randint(-127, 128, (N, K), generator=g, dtype=torch.int8)
    sa, sb = torch.rand(M, generator=g) * 0.01, torch.rand(N, generator=g) * 0.01
    add = torch.randn(M, N, generator=g)
    dt = getattr(torch, out)
    bias = torch.randn(N, generator=g).to(dt)
    ref = (A.double() @ B.double().t()) * sa.double()[:, None] * sb.double()[None, :] + add.double() + bias.double()
    y = native().int8_mm(A.to(dev), sa.to(dev), B.to(dev), sb.to(dev), add.to(dev), bias.to(dev), out)
    assert y.dtype == dt
    tol = {"float32": 1e-5, "bfloat16": 1e-2, "float16": 2e-3}[out]
    torch.testing.assert_close(y.cpu().double(), ref.to(dt).double(), rtol=tol, atol=tol)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("outliers", [0, 3])
def test_llm_int8_linear_matches_reference(dev, dtype, outliers):
    from pytorch_distributed_training_tutorials_amd.ops.quant import Int8Linear, llm_int8_reference

    lin = _lin(K=256, N=96, seed=outliers).to(dev).to(dtype)
    m = Int8Linear.from_linear(lin, llm_int8=True)
    x = torch.randn(4, 33, 256, device=dev, dtype=dtype)
    for j in range(outliers):
        x[..., 7 + 50 * j] *= 30.0
    y = m(x)
    ref = llm_int8_reference(x.reshape(-1, 256), m.weight_q, m.weight_scale, m.bias, m.threshold).reshape(y.shape)
    tol = dict(rtol=1e-5, atol=1e-5) if dtype == torch.float32 else dict(rtol=1e-2, atol=1e-2)
    assert y.dtype == dtype
    torch.testing.assert_close(y, ref, **tol)
    full = lin(x).float()
    assert (y.float() - full).abs().max() <= 0.03 * full.abs().max()


@pytest.mark.gpu
def test_llm_int8_unsupported_k_falls_back(dev):
    """in_features = 40 (no 16-deep K instance) converts and runs on the reference path (ADVICE r3:
    quantize_int8_ converts every Linear, so such a layer must not fail in forward)."""
    from pytorch_distributed_training_tutorials_amd.ops.quant import Int8Linear, llm_int8_reference, quantize_int8_

    model = torch.nn.Sequential(torch.nn.Linear(40, 24), torch.nn.ReLU(), torch.nn.Linear(24, 8)).to(dev)
    x = torch.randn(5, 40, device=dev)
    full = model(x)
    quantize_int8_(model, llm_int8=True)
    assert isinstance(model[0], Int8Linear) and isinstance(model[2], Int8Linear)
    y = model(x)
    assert y.shape == (5, 8) and torch.isfinite(y).all()
    m = model[0]
    ref = llm_int8_reference(x, m.weight_q, m.weight_scale, m.bias, m.threshold)
    torch.testing.assert_close(m(x), ref)
    assert (y - full).abs().max() <= 0.05 * full.abs().max() + 1e-3


@pytest.mark.gpu
def test_int8_weight_only_fp16(dev):
    """Weight-only int8 on fp16 activations (run in fp32, output fp16) tracks the fp16 Linear."""
    from pytorch_distributed_training_tutorials_amd.ops.quant import Int8Linear

    lin = _lin(K=256, N=96, seed=2).to(dev).half()
    m = Int8Linear.from_linear(lin)
    x = torch.randn(17, 256, device=dev, dtype=torch.float16)
    y = m(x)
    assert y.dtype == torch.float16
    full = lin(x).float()
    assert (y.float() - full).abs().max() <= 0.02 * full.abs().max()


@pytest.mark.gpu
def test_tiny_llama_llm_int8_logits_track_bf16(dev):
    """load_in_8bit-style model: every projection LLM.int8 (lm_head kept 16-bit)."""
    from pytorch_distributed_training_tutorials_amd.models.llama import build_llama
    from pytorch_distributed_training_tutorials_amd.ops.quant import Int8Linear, quantize_int8_

    ref = build_llama("tiny", dtype=torch.float32).to(dev).eval()
    q = build_llama("tiny", dtype=torch.float32).to(dev).eval()
    quantize_int8_(q, llm_int8=True)
    n8 = sum(isinstance(m, Int8Linear) for m in q.modules())
    assert n8 == 7 * 4 and q.lm_head.weight.dtype == torch.float32
    ids = torch.randint(0, 512, (2, 24), device=dev)
    with torch.no_grad():
        a, b = ref(ids).logits, q(ids).logits
    assert (a - b).norm() <= 0.05 * a.norm()


@pytest.mark.gpu
@pytest.mark.parametrize("M", [1, 7, 16, 17, 32])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("outliers", [0, 3])
def test_llm_int8_decode_path_matches_reference(dev, M, dtype, outliers):
    """Decode shapes (<= 32 tokens): csrc/kernels/int8_decode.hip (outliers + quantisation + int8 GEMV
    with the outlier columns fused, no host read) against the plain-PyTorch LLM.int8 product; N not a
    multiple of 16, K = 320 (5 K-steps: uneven split over the 4 waves)."""
    from pytorch_distributed_training_tutorials_amd import native
    from pytorch_distributed_training_tutorials_amd.ops.quant import Int8Linear, llm_int8_reference

    lin = _lin(K=320, N=101, seed=M + outliers).to(dev).to(dtype)
    m = Int8Linear.from_linear(lin, llm_int8=True)
    x = torch.randn(M, 320, device=dev, dtype=dtype)
    for j in range(outliers):
        x[min(j, M - 1), 7 + 100 * j] = 40.0
    assert native().int8_decode_supported(M, 101, 320)
    y = m(x)
    ref = llm_int8_reference(x, m.weight_q, m.weight_scale, m.bias, m.threshold)
    tol = dict(rtol=1e-5, atol=1e-5) if dtype == torch.float32 else dict(rtol=1e-2, atol=1e-2)
    assert y.dtype == dtype and y.shape == (M, 101)
    torch.testing.assert_close(y, ref, **tol)
    if outliers:  # the outlier columns are decomposed, not quantised: close to the unquantised product
        full = lin(x).float()
        assert (y.float() - full).abs().max() <= 0.03 * full.abs().max()


@pytest.mark.gpu
def test_llm_int8_decode_llama_shape(dev):
    """The reference's Llama-7B MLP up-projection at one decode token batch (M = 16, 4096 -> 11008,
    fp16, two outlier features)."""
    from pytorch_distributed_training_tutorials_amd.ops.quant import Int8Linear, llm_int8_reference

    torch.manual_seed(0)
    lin = torch.nn.Linear(4096, 11008, bias=False, device=dev, dtype=torch.float16)
    m = Int8Linear.from_linear(lin, llm_int8=True)
    x = torch.randn(16, 4096, device=dev, dtype=torch.float16)
    x[:, 1234] *= 20.0
    x[3, 77] = -30.0
    y = m(x)
    ref = llm_int8_reference(x, m.weight_q, m.weight_scale, None, m.threshold)
    torch.testing.assert_close(y, ref, rtol=1e-2, atol=1e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("M", [5, 32])
def test_llm_int8_decode_many_outliers_across_workgroups(dev, M):
    """fp32 decode with 40 outlier columns spread over the four 512-column statistics workgroups of
    K = 2048 (several per workgroup, one in the last chunk): the per-workgroup lists concatenate in
    column order and the product matches the reference to fp32 rounding."""
    from pytorch_distributed_training_tutorials_amd.ops.quant import Int8Linear, llm_int8_reference

    torch.manual_seed(M)
    lin = torch.nn.Linear(2048, 200, device=dev)
    m = Int8Linear.from_linear(lin, llm_int8=True)
    x = torch.randn(M, 2048, device=dev)
    cols = torch.randperm(2047, generator=torch.Generator().manual_seed(M))[:39].tolist() + [2047]
    for j, col in enumerate(cols):
        x[j % M, col] = 10.0 + j
    y = m(x)
    ref = llm_int8_reference(x, m.weight_q, m.weight_scale, m.bias, m.threshold)
    torch.testing.assert_close(y, ref, rtol=1e-5, atol=1e-4)


@pytest.mark.gpu
def test_llm_int8_decode_packed_weights(dev):
    """The decode GEMV's pre-shuffled weight copy (int8_decode_pack): its layout (tile, K step, lane)
    against a PyTorch re-arrangement, the packed and row-major GEMVs bit-identical (same int32
    products in the same order), and the cache rebuilt after an in-place weight update."""
    from pytorch_distributed_training_tutorials_amd import native
    from pytorch_distributed_training_tutorials_amd.ops.quant import Int8Linear, llm_int8_reference

    C = native()
    torch.manual_seed(11)
    N, K = 37, 192
    q = torch.randint(-127, 128, (N, K), device=dev, dtype=torch.int8)
    p = C.int8_decode_pack(q)
    tiles = (N + 15) // 16
    rows = torch.clamp(torch.arange(tiles * 16, device=dev), max=N - 1)
    qq = q[rows].view(tiles, 16, K // 64, 4, 16)  # [tile, c, step, g, byte]
    want = qq.permute(0, 2, 3, 1, 4).reshape(-1)  # [tile, step, lane = 16 g + c, byte]
    assert torch.equal(p, want)
    lin = torch.nn.Linear(K, N, device=dev, dtype=torch.bfloat16)
    m = Int8Linear.from_linear(lin, llm_int8=True)
    x = torch.randn(9, K, device=dev, dtype=torch.bfloat16)
    x[2, 70] = 30.0
    a = C.int8_decode(x, m.weight_q, m.weight_scale, m.bias, m.threshold, "bfloat16", C.int8_decode_pack(m.weight_q))
    b = C.int8_decode(x, m.weight_q, m.weight_scale, m.bias, m.threshold, "bfloat16", None)
    assert torch.equal(a, b)
    m(x)
    m.weight_q.mul_(-1)
    y = m(x)
    torch.testing.assert_close(y, llm_int8_reference(x, m.weight_q, m.weight_scale, m.bias, m.threshold),
                               rtol=1e-2, atol=1e-2)


def test_decode_packed_cache_tracks_weight_identity_and_version():
    """The pre-shuffled weight cache (Int8Linear._decode_packed) is rebuilt after an in-place weight
    update and after the buffer is replaced by another tensor, and reused otherwise (CPU: a stub
    packer stands in for the native one)."""
    from pytorch_distributed_training_tutorials_amd.ops.quant import Int8Linear

    calls = []

    class Packer:
        def int8_decode_pack(self, w):
            calls.append(1)
            return w.clone()

    m, C = Int8Linear(64, 16), Packer()
    p = m._decode_packed(C)
    assert m._decode_packed(C) is p and len(calls) == 1
    m.weight_q.add_(1)
    m._decode_packed(C)
    assert len(calls) == 2
    m.weight_q = torch.zeros(16, 64, dtype=torch.int8)
    m._decode_packed(C)
    assert len(calls) == 3
    # a write through .data bypasses the version counter: the explicit hook drops the copy
    m.weight_q.data.copy_(torch.ones(16, 64, dtype=torch.int8))
    m.invalidate_packed()
    assert torch.equal(m._decode_packed(C), m.weight_q) and len(calls) == 4
    # load_state_dict invalidates by itself
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    sd["weight_q"].fill_(3)
    m.load_state_dict(sd)
    assert torch.equal(m._decode_packed(C), sd["weight_q"]) and len(calls) == 5
