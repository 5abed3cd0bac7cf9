"""Numerics of every gfx950 kernel against plain PyTorch fp32 references (GPU)."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _ref_step(X, Y, idx, params, H, loss_kind, relu=True):
    """Torch fp32 reference of one Linear[-ReLU-Linear] step: (loss, grads)."""
    ps = [p.detach().clone().requires_grad_(True) for p in params]
    x = X[idx.long()]
    if H > 0:
        W1, b1, W2, b2 = ps
        z = F.linear(F.relu(F.linear(x, W1, b1)), W2, b2)
    else:
        W, b = ps
        z = F.linear(x, W, b)
    y = Y[idx.long()]
    if loss_kind == "ce_soft":
        loss = F.cross_entropy(z, y)
    elif loss_kind == "ce_index":
        loss = F.cross_entropy(z, y)
    else:
        loss = F.mse_loss(z, y)
    loss.backward()
    return loss.detach(), [p.grad for p in ps]


@pytest.mark.parametrize("H,Dout,loss_kind", [(0, 1, "ce_soft"), (0, 4, "ce_soft"), (16, 10, "ce_index"),
                                              (64, 10, "ce_index"), (32, 3, "mse"), (0, 5, "mse")])
def test_fused_mlp_step_matches_torch(native, dev, H, Dout, loss_kind):
    torch.manual_seed(0)
    N, Din, B = 256, 20, 32
    X = torch.rand(N, Din, device=dev)
    if loss_kind == "ce_index":
        Y = torch.randint(0, Dout, (N,), device=dev)
    elif loss_kind == "ce_soft":
        Y = torch.rand(N, Dout, device=dev)
    else:
        Y = torch.randn(N, Dout, device=dev)
    shapes = ([(H, Din), (H,), (Dout, H), (Dout,)] if H else [(Dout, Din), (Dout,)])
    params = [torch.randn(s, device=dev) * 0.3 for s in shapes]
    P = torch.cat([p.reshape(-1) for p in params])
    G = torch.zeros_like(P)
    idx = torch.randperm(N, device=dev)[:B].to(torch.int32)
    loss = torch.zeros(1, device=dev)
    kind = {"ce_soft": 0, "ce_index": 1, "mse": 2}[loss_kind]
    native.fused_mlp_step(X, None if kind == 1 else Y, Y if kind == 1 else None, idx, P, G, None, None, loss,
                          B, Din, H, Dout, kind, -100, True, 1.0, False, 0, 0.0, 0.0, 0.0, 0.0, False)
    rl, rg = _ref_step(X, Y, idx, params, H, loss_kind)
    torch.testing.assert_close(loss[0], rl, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(G, torch.cat([g.reshape(-1) for g in rg]), rtol=1e-4, atol=1e-6)


def test_fused_reference_toy_is_exactly_zero(native, dev):
    """Quirk Q1: Linear(20,1) + soft CE on [B,1] -> loss == 0 and grads == 0 exactly."""
    X = torch.rand(64, 20, device=dev)
    Y = torch.rand(64, 1, device=dev)
    P = torch.randn(21, device=dev)
    G = torch.full_like(P, 7.0)
    loss = torch.full((1,), 3.0, device=dev)
    native.fused_mlp_step(X, Y, None, None, P, G, None, None, loss, 32, 20, 0, 1, 0, -100, True, 1.0, False,
                          0, 0.0, 0.0, 0.0, 0.0, False)
    assert loss.abs().item() == 0.0
    assert (G == 0).all()


@pytest.mark.parametrize("momentum", [0.0, 0.9])
def test_fused_deferred_update_equals_sgd(native, dev, momentum):
    torch.manual_seed(1)
    N, Din, H, Dout, B = 128, 20, 16, 10, 32
    X = torch.randn(N, Din, device=dev)
    Y = torch.randint(0, Dout, (N,), device=dev)
    shapes = [(H, Din), (H,), (Dout, H), (Dout,)]
    params = [torch.randn(s, device=dev) * 0.3 for s in shapes]
    # torch reference: 3 SGD steps
    ref = [p.clone().requires_grad_(True) for p in params]
    opt = torch.optim.SGD(ref, lr=0.1, momentum=momentum)
    idxs = [torch.randperm(N, device=dev)[:B].to(torch.int32) for _ in range(3)]
    for idx in idxs:
        opt.zero_grad()
        x = X[idx.long()]
        z = F.linear(F.relu(F.linear(x, ref[0], ref[1])), ref[2], ref[3])
        F.cross_entropy(z, Y[idx.long()]).backward()
        opt.step()
    P = torch.cat([p.reshape(-1) for p in params])
    G = torch.zeros_like(P)
    mom = torch.zeros_like(P) if momentum else None
    step = torch.zeros(1, dtype=torch.int32, device=dev)
    loss = torch.zeros(1, device=dev)
    for i, idx in enumerate(idxs):
        mode = 1 if i > 0 else 0  # deferred ("pre") update of the previous step
        native.fused_mlp_step(X, None, Y, idx, P, G, mom, step, loss, B, Din, H, Dout, 1, -100, True, 1.0, False,
                              mode, 0.1, momentum, 0.0, 0.0, False)
    native.sgd_flat_(P, G, mom, step, 0.1, momentum, 0.0, 0.0, False, 1.0)
    torch.testing.assert_close(P, torch.cat([p.detach().reshape(-1) for p in ref]), rtol=1e-4, atol=1e-5)


# ----------------------------------------------------------------------------- GEMM
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,N,K", [(32, 1, 20), (8, 2, 32), (20, 10, 10000), (120, 1000, 2048), (67, 45, 33),
                                   (256, 256, 256)])
@pytest.mark.parametrize("layout", ["NT", "NN", "TN"])
def test_gemm_layouts(native, dev, dtype, M, N, K, layout):
    torch.manual_seed(M + N + K)
    a = torch.randn(M, K, device=dev).to(dtype)
    b = torch.randn(K, N, device=dev).to(dtype)
    A = a if layout != "TN" else a.t().contiguous().t()
    B = b if layout != "NT" else b.t().contiguous().t()
    from pytorch_distributed_training_tutorials_amd.ops.linear import gemm

    C = gemm(A, B, out_dtype=torch.float32)
    ref = a.float() @ b.float()
    tol = 2e-5 * math.sqrt(K) if dtype == torch.float32 else 2e-2
    torch.testing.assert_close(C, ref, rtol=tol, atol=tol * 4)


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (512, 768, 1024), (300, 200, 128), (120, 1000, 2048),
                                   (1, 257, 64), (1000, 17, 192)])
@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("sched", [0, 1, 2, 3, 4, 5, 6])
def test_gemm_big_matches_fp32(native, dev, M, N, K, out_dtype, sched):
    """256x256 LDS-DMA kernel: C = A.Bt^T (+bias, ReLU, alpha/beta) vs fp32 on the same bf16 operands;
    asymmetric operands catch a transposed C write, edge shapes the clamped rows."""
    torch.manual_seed(M * 7 + N + K)
    A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    Bt = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
    assert native.gemm_big_ok(A, Bt)
    ref = A.float() @ Bt.float().t()
    C = torch.empty(M, N, device=dev, dtype=out_dtype)
    native.gemm_big_(A, Bt, C, sched=sched)
    tol = 1e-4 * math.sqrt(K) if out_dtype == torch.float32 else 1e-2 * math.sqrt(K) / 8
    torch.testing.assert_close(C.float(), ref, rtol=tol, atol=tol)
    bias = torch.randn(N, device=dev)
    C0 = torch.randn(M, N, device=dev).to(out_dtype)
    C1 = C0.clone()
    native.gemm_big_(A, Bt, C1, bias, True, 0.5, 2.0, sched)
    torch.testing.assert_close(C1.float(), F.relu(0.5 * ref + 2.0 * C0.float() + bias), rtol=tol, atol=tol)


@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (512, 768, 1024), (300, 200, 128), (120, 1000, 2048),
                                   (1, 257, 64), (1000, 17, 192)])
@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
def test_gemm_big_tile128_matches_fp32(native, dev, M, N, K, out_dtype):
    """128x128-tile variant (4 waves): same contract as the 256 tile, edges clamped."""
    torch.manual_seed(M * 5 + N + K)
    A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    Bt = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
    ref = A.float() @ Bt.float().t()
    tol = 1e-4 * math.sqrt(K) if out_dtype == torch.float32 else 1e-2 * math.sqrt(K) / 8
    bias = torch.randn(N, device=dev)
    C0 = torch.randn(M, N, device=dev).to(out_dtype)
    C1 = C0.clone()
    native.gemm_big_(A, Bt, C1, bias, True, 0.5, 2.0, tile=128)
    torch.testing.assert_close(C1.float(), F.relu(0.5 * ref + 2.0 * C0.float() + bias), rtol=tol, atol=tol)


@pytest.mark.parametrize("tile", [128, 256])
@pytest.mark.parametrize("split", [2, 3, 7, 32])
def test_gemm_big_split_k(native, dev, tile, split):
    """split-K slices atomically accumulate into a zeroed f32 C; bias added once (slice 0);
    uneven slices (K-tiles not divisible by the split) and more slices than K-tiles clamp."""
    M, N, K = 200, 300, 64 * 13
    torch.manual_seed(split + tile)
    A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    Bt = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
    bias = torch.randn(N, device=dev)
    C = torch.zeros(M, N, device=dev)
    native.gemm_big_(A, Bt, C, bias, False, 0.5, tile=tile, split_k=split)
    ref = 0.5 * (A.float() @ Bt.float().t()) + bias
    torch.testing.assert_close(C, ref, rtol=1e-3, atol=1e-3)
    with pytest.raises(RuntimeError):  # atomics need an f32 accumulator
        native.gemm_big_(A, Bt, torch.zeros(M, N, device=dev, dtype=torch.bfloat16), tile=tile, split_k=split)


@pytest.mark.parametrize("M,N,K", [(4096, 4096, 256), (2048, 2048, 2048), (120, 1000, 2048), (256, 512, 4096)])
def test_gemm_nt_big_planner(dev, M, N, K):
    """ops.linear.gemm_nt_big picks (tile, split) by shape; every plan gives the fp32 result."""
    from pytorch_distributed_training_tutorials_amd.ops.linear import gemm_nt_big, plan_big

    torch.manual_seed(1)
    A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    Bt = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
    bias = torch.randn(N, device=dev).to(torch.bfloat16)
    ref = F.relu(A.float() @ Bt.float().t() + bias.float())
    tile, split = plan_big(M, N, K)
    assert tile in (128, 256) and split >= 1
    out = gemm_nt_big(A, Bt, torch.bfloat16, bias=bias, relu=True)
    tol = 1e-2 * math.sqrt(K) / 8
    torch.testing.assert_close(out.float(), ref, rtol=tol, atol=tol)


@pytest.mark.parametrize("tile,sched", [(128, -1), (256, 1), (256, 2), (256, 3)])
@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
def test_gemm_big_strided_output(native, dev, sched, tile, out_dtype):
    """The coalesced epilogue (LDS-staged rows, 16-B stores) on output views: a row stride that is
    not a multiple of 8 elements takes the per-element path, an aligned column slice the vector
    one; the columns around the view stay untouched."""
    M, N, K = 300, 200, 192
    torch.manual_seed(tile + sched)
    A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    Bt = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
    bias = torch.randn(N, device=dev)
    ref = F.relu(A.float() @ Bt.float().t() + bias)
    tol = 1e-4 * math.sqrt(K) if out_dtype == torch.float32 else 1e-2 * math.sqrt(K) / 8
    for pad, off in ((3, 1), (16, 8)):
        big = torch.full((M, N + pad), 7.0, device=dev, dtype=out_dtype)
        view = big[:, off:off + N]
        native.gemm_big_(A, Bt, view, bias, True, 1.0, 0.0, sched, tile=tile)
        torch.testing.assert_close(view.float(), ref, rtol=tol, atol=tol)
        assert bool((big[:, :off] == 7).all()) and bool((big[:, off + N:] == 7).all())


def test_gemm_big_identity_and_strides(native, dev):
    """A = I picks rows of Bt exactly; strided (sliced) operands use their row stride."""
    K = 128
    eye = torch.eye(K, device=dev, dtype=torch.bfloat16)
    Bt = torch.arange(300 * K, device=dev, dtype=torch.float32).reshape(300, K).remainder(97).to(torch.bfloat16)
    C = torch.empty(K, 300, device=dev)
    native.gemm_big_(eye, Bt, C)
    torch.testing.assert_close(C, Bt.float().t(), rtol=0, atol=0)
    big = (torch.rand(200, 3 * K, device=dev) * 2 - 1).to(torch.bfloat16)
    A = big[:, K:2 * K]  # row stride 3K
    C2 = torch.empty(200, 300, device=dev)
    native.gemm_big_(A, Bt, C2)
    torch.testing.assert_close(C2, A.float() @ Bt.float().t(), rtol=1e-3, atol=1e-2)
    assert not native.gemm_big_ok(A[:, :100], Bt[:, :100])  # K % 64 != 0 -> strided kernel


def test_gemm_epilogues(native, dev):
    torch.manual_seed(0)
    M, N, K = 70, 50, 90
    A = torch.randn(M, K, device=dev)
    B = torch.randn(K, N, device=dev)
    bias = torch.randn(N, device=dev)
    mask = (torch.randn(M, K, device=dev) > 0).float()
    C = torch.empty(M, N, device=dev)
    cs = torch.zeros(M, device=dev)
    native.gemm_(A, B, C, bias, mask, True, 1.0, 0.0, cs, 1)
    Am = A * mask
    torch.testing.assert_close(C, F.relu(Am @ B + bias), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(cs, Am.sum(1), rtol=1e-4, atol=1e-4)
    # accumulate (beta)
    C2 = torch.randn(M, N, device=dev)
    ref = 0.5 * (A @ B) + 2.0 * C2
    native.gemm_(A, B, C2, None, None, False, 0.5, 2.0, None, 1)
    torch.testing.assert_close(C2, ref, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("relu", [False, True])
def test_linear_autograd(native, dev, dtype, relu):
    from pytorch_distributed_training_tutorials_amd.ops.linear import linear

    torch.manual_seed(3)
    x = torch.randn(37, 53, device=dev, dtype=dtype, requires_grad=True)
    w = torch.randn(29, 53, device=dev, dtype=dtype, requires_grad=True)
    b = torch.randn(29, device=dev, dtype=dtype, requires_grad=True)
    y = linear(x, w, b, relu)
    g = torch.randn_like(y)
    y.backward(g)
    xr, wr, br = (t.detach().float().requires_grad_(True) for t in (x, w, b))
    yr = F.linear(xr, wr, br)
    if relu:
        yr = F.relu(yr)
    yr.backward(g.float())
    tol = 1e-4 if dtype == torch.float32 else 5e-2
    torch.testing.assert_close(y.float(), yr, rtol=tol, atol=tol)
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=tol, atol=tol)
    torch.testing.assert_close(w.grad.float(), wr.grad, rtol=tol, atol=tol)
    torch.testing.assert_close(b.grad.float(), br.grad, rtol=tol, atol=tol * 4)


@pytest.mark.parametrize("engine", ["native", "auto"])
@pytest.mark.parametrize("relu", [False, True])
def test_linear_big_bf16_path(native, dev, relu, engine, monkeypatch):
    """bf16 Linear large enough for the 256x256 kernel (forward, dx, dW, db) vs fp32 autograd;
    ``native``: every GEMM on gemm_big.hip, ``auto``: plain GEMMs on hipBLASLt, fused ones native."""
    import importlib

    monkeypatch.setenv("PTDT_LINEAR_GEMM", engine)
    L = importlib.import_module("pytorch_distributed_training_tutorials_amd.ops.linear")  # module, not the op
    from pytorch_distributed_training_tutorials_amd.utils import tuning

    for d in (tuning._LOCAL, tuning._AGREED, tuning._DECIDED):
        d["linear"].clear()
    assert L._library(relu) == (engine == "auto" and not relu)
    torch.manual_seed(5)
    M, K, N = 512, 384, 320
    assert L._big(M, N, K, torch.bfloat16) and L._big(N, K, M, torch.bfloat16)
    x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16).requires_grad_(True)
    w = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16).requires_grad_(True)
    b = torch.randn(N, device=dev, dtype=torch.bfloat16, requires_grad=True)
    y = L.linear(x, w, b, relu)
    g = (torch.rand_like(y.float()) * 2 - 1).to(torch.bfloat16)
    y.backward(g)
    xr, wr, br = (t.detach().float().requires_grad_(True) for t in (x, w, b))
    yr = F.linear(xr, wr, br)
    if relu:
        yr = F.relu(yr)
    yr.backward(g.float())
    for got, ref, k in ((y, yr, K), (x.grad, xr.grad, N), (w.grad, wr.grad, M), (b.grad, br.grad, M)):
        tol = 2e-2 * math.sqrt(k) / 4
        torch.testing.assert_close(got.float(), ref, rtol=tol, atol=tol)
    if engine == "auto":  # every plain GEMM of the layer was timed on both engines and the winner cached
        keys = [k.split(",") for k in tuning._LOCAL["linear"]]
        forms = {k[0] for k in keys if tuple(map(int, k[1:])) in ((M, N, K), (M, K, N), (N, K, M))}
        assert forms == ({"nn", "tn"} if relu else {"nt", "nn", "tn"})


def test_linear_under_autocast(native, dev):
    """bf16 autocast over fp32 master weights (ResNet-50 DDP bench path): bf16 MFMA
    compute, fp32 grads for the fp32 parameters."""
    from pytorch_distributed_training_tutorials_amd.ops.linear import Linear

    torch.manual_seed(4)
    m = Linear(64, 48).to(dev)
    x = torch.randn(40, 64, device=dev)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(x)
    assert y.dtype == torch.bfloat16
    y.float().sum().backward()
    assert m.weight.grad.dtype == torch.float32 and m.bias.grad.dtype == torch.float32
    ref = F.linear(x, m.weight.detach(), m.bias.detach())
    torch.testing.assert_close(y.float(), ref, rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(m.weight.grad, x.sum(0).expand(48, 64), rtol=3e-2, atol=3e-1)


def test_linear_long_k_split(native, dev):
    """ToyModel's net1: Linear(10000, 10) + ReLU on [20, 10000] (split-K path)."""
    from pytorch_distributed_training_tutorials_amd.ops.linear import linear

    x = torch.randn(20, 10000, device=dev, requires_grad=True)
    w = (torch.randn(10, 10000, device=dev) * 0.01).requires_grad_(True)
    b = torch.randn(10, device=dev, requires_grad=True)
    y = linear(x, w, b, True)
    y.sum().backward()
    xr, wr, br = (t.detach().clone().requires_grad_(True) for t in (x, w, b))
    F.relu(F.linear(xr, wr, br)).sum().backward()
    torch.testing.assert_close(y, F.relu(F.linear(xr, wr, br)), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(w.grad, wr.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(x.grad, xr.grad, rtol=1e-4, atol=1e-4)


# ----------------------------------------------------------------------------- losses
@pytest.mark.parametrize("B,C", [(32, 1), (32, 10), (120, 1000), (7, 3)])
def test_cross_entropy_soft_and_index(native, dev, B, C):
    from pytorch_distributed_training_tutorials_amd.ops.loss import cross_entropy

    torch.manual_seed(B * C)
    z = torch.randn(B, C, device=dev, requires_grad=True)
    t_soft = torch.rand(B, C, device=dev)
    t_idx = torch.randint(0, C, (B,), device=dev)
    if B > 3:
        t_idx[2] = -100
    for t, ls in ((t_soft, 0.0), (t_idx, 0.0), (t_idx, 0.1), (t_soft, 0.2)):
        z.grad = None
        l = cross_entropy(z, t, label_smoothing=ls)
        l.backward()
        zr = z.detach().clone().requires_grad_(True)
        lr_ = F.cross_entropy(zr, t, label_smoothing=ls)
        lr_.backward()
        torch.testing.assert_close(l, lr_, rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(z.grad, zr.grad, rtol=1e-5, atol=1e-6)


def test_mse(native, dev):
    from pytorch_distributed_training_tutorials_amd.ops.loss import mse_loss

    x = torch.randn(120, 1000, device=dev, requires_grad=True)
    y = torch.randn(120, 1000, device=dev)
    l = mse_loss(x, y)
    l.backward()
    xr = x.detach().clone().requires_grad_(True)
    lr_ = F.mse_loss(xr, y)
    lr_.backward()
    torch.testing.assert_close(l, lr_, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(x.grad, xr.grad, rtol=1e-5, atol=1e-8)


# ----------------------------------------------------------------------------- optimizers
@pytest.mark.parametrize("kw", [dict(lr=0.1), dict(lr=0.05, momentum=0.9), dict(lr=0.05, momentum=0.9, nesterov=True,
                                                                               weight_decay=1e-3),
                                dict(lr=0.05, momentum=0.5, dampening=0.1)])
def test_fused_sgd_matches_torch(native, dev, kw):
    from pytorch_distributed_training_tutorials_amd.ops.flat import FlatParameters
    from pytorch_distributed_training_tutorials_amd.ops.optim import FusedSGD

    torch.manual_seed(0)
    shapes = [(33, 7), (7,), (1000,), (5, 5, 3)]
    ps = [torch.randn(s, device=dev, requires_grad=True) for s in shapes]
    rs = [p.detach().clone().requires_grad_(True) for p in ps]
    for flat in (False, True):
        qs = [p.detach().clone().requires_grad_(True) for p in ps]
        if flat:
            FlatParameters(qs, with_grads=True)
        opt, ropt = FusedSGD(qs, **kw), torch.optim.SGD([r.detach().clone().requires_grad_(True) for r in rs], **kw)
        rps = ropt.param_groups[0]["params"]
        for it in range(3):
            gs = [torch.randn_like(p) for p in ps]
            for q, r, g in zip(qs, rps, gs):
                if q.grad is None:
                    q.grad = g.clone()
                else:
                    q.grad.copy_(g)
                r.grad = g.clone()
            opt.step()
            ropt.step()
        for q, r in zip(qs, rps):
            torch.testing.assert_close(q.detach(), r.detach(), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("momentum", [0.0, 0.9])
def test_fused_sgd_bf16_shadow_multi_chunk(native, dev, momentum):
    """Multi-tensor SGD with bf16 weight shadows over tensors spanning several 4096-element chunks,
    with 4-element tails and a misaligned view (the vector and scalar paths): parameters match
    torch.optim.SGD and every shadow is the bf16 rounding of its updated parameter."""
    from pytorch_distributed_training_tutorials_amd.ops.optim import FusedSGD

    torch.manual_seed(1)
    base = torch.randn(20001, device=dev)
    ps = [torch.randn(9003, device=dev), torch.randn(64, 3, 7, 7, device=dev), base[1:8194].clone(), base[3:10]]
    ps = [p.detach().clone().requires_grad_(True) for p in ps]
    rs = [p.detach().clone().requires_grad_(True) for p in ps]
    kw = dict(lr=0.05, momentum=momentum, weight_decay=1e-4)
    opt, ropt = FusedSGD(ps, bf16_shadow=True, **kw), torch.optim.SGD(rs, **kw)
    for _ in range(3):
        for q, r in zip(ps, rs):
            g = torch.randn_like(q)
            q.grad, r.grad = g.clone(), g.clone()
        opt.step()
        ropt.step()
    for q, r in zip(ps, rs):
        torch.testing.assert_close(q.detach(), r.detach(), rtol=1e-5, atol=1e-6)
        assert torch.equal(q._ptdt_bf16, q.detach().to(torch.bfloat16))


@pytest.mark.parametrize("decoupled", [False, True])
def test_fused_adam_matches_torch(native, dev, decoupled):
    from pytorch_distributed_training_tutorials_amd.ops.optim import FusedAdam

    torch.manual_seed(0)
    ps = [torch.randn(s, device=dev, requires_grad=True) for s in [(66,), (2, 32), (4097,)]]
    qs = [p.detach().clone().requires_grad_(True) for p in ps]
    rs = [p.detach().clone().requires_grad_(True) for p in ps]
    opt = FusedAdam(qs, lr=1e-2, weight_decay=1e-2, decoupled_weight_decay=decoupled)
    ropt = (torch.optim.AdamW if decoupled else torch.optim.Adam)(rs, lr=1e-2, weight_decay=1e-2)
    for _ in range(4):
        for q, r in zip(qs, rs):
            g = torch.randn_like(q)
            q.grad, r.grad = g.clone(), g.clone()
        opt.step()
        ropt.step()
    for q, r in zip(qs, rs):
        torch.testing.assert_close(q, r, rtol=1e-5, atol=1e-6)


def test_bucket_pack_unpack(native, dev):
    ts = [torch.randn(s, device=dev) for s in [(3, 4), (100,), (7,)]]
    flat = torch.zeros(sum(t.numel() for t in ts), device=dev)
    native.bucket_copy(ts, flat, 0.25, False)
    torch.testing.assert_close(flat, torch.cat([t.reshape(-1) for t in ts]) * 0.25)
    outs = [torch.zeros_like(t) for t in ts]
    native.bucket_copy(outs, flat, 4.0, True)
    for o, t in zip(outs, ts):
        torch.testing.assert_close(o, t)


# ----------------------------------------------------------------------------- data kernels
def test_philox_uniform_and_normal(native, dev):
    u = torch.empty(1 << 20, device=dev)
    native.philox_(u, 123, 0, 0)
    assert 0.0 <= u.min().item() and u.max().item() < 1.0
    assert abs(u.mean().item() - 0.5) < 5e-3 and abs(u.var().item() - 1 / 12) < 5e-3
    n = torch.empty(1 << 20, device=dev)
    native.philox_(n, 123, 0, 1)
    assert abs(n.mean().item()) < 5e-3 and abs(n.std().item() - 1.0) < 5e-3
    u2 = torch.empty(1 << 20, device=dev)
    native.philox_(u2, 123, 0, 0)
    assert torch.equal(u, u2)


def test_one_hot_and_gather(native, dev):
    idx = torch.randint(0, 1000, (120,), device=dev)
    oh = native.one_hot(idx, 1000)
    torch.testing.assert_close(oh, F.one_hot(idx, 1000).float())
    src = torch.randn(500, 33, device=dev)
    sel = torch.randint(0, 500, (77,), device=dev, dtype=torch.int32)
    out = torch.empty(77, 33, device=dev)
    native.gather_rows_(src, sel, out)
    torch.testing.assert_close(out, src[sel.long()])


@pytest.mark.parametrize("N,W", [(2048, 1), (2048, 8), (1000, 3), (5, 8), (2049, 4)])
def test_device_sampler_matches_host_model(native, dev, N, W):
    from pytorch_distributed_training_tutorials_amd.data.device_sampler import (DeviceDistributedSampler,
                                                                                 reference_indices)

    allidx = []
    for r in range(W):
        s = DeviceDistributedSampler(N, W, r, seed=7, device=dev)
        s.set_epoch(3)
        out = torch.zeros(s.num_samples, dtype=torch.int32, device=dev)
        s.generate(out)
        assert s.current_epoch() == 3
        ref = reference_indices(N, W, r, 3, seed=7)
        assert out.cpu().numpy().tolist() == ref.tolist()
        allidx.append(ref)
    flat = sorted(set(int(i) for a in allidx for i in a))
    assert flat == list(range(N))


# ----------------------------------------------------------------------------- int8
def test_int8_quant_and_gemm(native, dev):
    torch.manual_seed(0)
    w = torch.randn(300, 256, device=dev)
    q, s = native.quantize_int8(w)
    deq = q.float() * s[:, None]
    assert (deq - w).abs().max().item() <= s.max().item() * 0.51
    for dt in (torch.float32, torch.bfloat16):
        x = torch.randn(40, 256, device=dev).to(dt)
        b = torch.randn(300, device=dev).to(dt)
        y = native.int8_linear(x, q, s, b)
        # activations are multiplied in bf16 on the MFMA (fp32 accumulate): reference rounds x the same way
        ref = x.bfloat16().float() @ deq.t() + b.float()
        tol = 1e-3 if dt == torch.float32 else 2e-2
        torch.testing.assert_close(y.float(), ref, rtol=tol, atol=tol)


def test_bn_relu(native, dev):
    x = torch.randn(4, 6, 5, 5, device=dev)
    sc, sh = torch.randn(6, device=dev), torch.randn(6, device=dev)
    y = native.bn_relu(x, sc, sh, True)
    torch.testing.assert_close(y, F.relu(x * sc[None, :, None, None] + sh[None, :, None, None]))


def test_fused_optimizers_channels_last(native, dev):
    """channels_last conv weights: grads/state keep the parameter's memory order and
    the native SGD/Adam match torch.optim (ResNet-50 DDP bench path)."""
    from pytorch_distributed_training_tutorials_amd.ops.optim import FusedAdam, FusedSGD

    for opt_cls, ref_cls, kw in ((FusedSGD, torch.optim.SGD, dict(lr=0.1, momentum=0.9, weight_decay=1e-4)),
                                 (FusedAdam, torch.optim.Adam, dict(lr=1e-2))):
        torch.manual_seed(0)
        conv = torch.nn.Conv2d(8, 16, 3).to(dev).to(memory_format=torch.channels_last)
        ref = torch.nn.Conv2d(8, 16, 3).to(dev).to(memory_format=torch.channels_last)
        ref.load_state_dict(conv.state_dict())
        o1, o2 = opt_cls(conv.parameters(), **kw), ref_cls(ref.parameters(), **kw)
        x = torch.randn(4, 8, 10, 10, device=dev).to(memory_format=torch.channels_last)
        for _ in range(3):
            for m, o in ((conv, o1), (ref, o2)):
                o.zero_grad()
                m(x).square().mean().backward()
                o.step()
        assert not conv.weight.is_contiguous()  # stayed channels_last
        torch.testing.assert_close(conv.weight, ref.weight, rtol=1e-5, atol=1e-6)


def test_fused_adam_resume_keeps_flat_state(native, dev):
    """FusedAdam.load_state_dict re-homes the moments in ONE flat buffer (the step keeps
    the single-launch adam_flat_ path) and the resumed run matches torch.optim.Adam."""
    from pytorch_distributed_training_tutorials_amd.ops.flat import contiguous_span
    from pytorch_distributed_training_tutorials_amd.ops.optim import FusedAdam

    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 4)).to(dev)
    ref = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 4)).to(dev)
    ref.load_state_dict(m.state_dict())
    x = torch.randn(8, 16, device=dev)
    o_ref = torch.optim.Adam(ref.parameters(), lr=1e-2)
    o = FusedAdam(m.parameters(), lr=1e-2)
    for it in range(5):
        if it == 2:  # resume mid-run from the fused optimizer's own state_dict
            sd = o.state_dict()
            o = FusedAdam(m.parameters(), lr=1e-2)
            o.load_state_dict(sd)
            ps = list(m.parameters())
            assert contiguous_span([o.state[p]["exp_avg"] for p in ps]) is not None
            assert contiguous_span([o.state[p]["exp_avg_sq"] for p in ps]) is not None
        for mod, opt in ((m, o), (ref, o_ref)):
            opt.zero_grad()
            mod(x).square().mean().backward()
            opt.step()
    for a, b in zip(m.parameters(), ref.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
