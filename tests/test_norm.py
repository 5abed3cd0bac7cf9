"""BatchNorm with fused residual/ReLU (ops/norm.py, csrc/kernels/batchnorm.hip) vs
PyTorch's fp32 batch_norm composite. CPU tests cover the fallback and module
contract; GPU tests the native NHWC kernels."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from pytorch_distributed_training_tutorials_amd.ops.norm import BatchNorm2d, batch_norm_act


def _reference(x, bn_ref, residual, relu):
    y = bn_ref(x)
    if residual is not None:
        y = y + residual
    return F.relu(y) if relu else y


def test_module_contract_matches_nn_batchnorm():
    a, b = BatchNorm2d(64), nn.BatchNorm2d(64)
    assert list(a.state_dict().keys()) == list(b.state_dict().keys())
    assert isinstance(a, nn.BatchNorm2d)
    b.load_state_dict(a.state_dict())


@pytest.mark.parametrize("relu,res", [(False, False), (True, False), (True, True)])
def test_cpu_fallback_matches_composite(relu, res):
    torch.manual_seed(0)
    x = torch.randn(4, 16, 5, 5, requires_grad=True)
    r = torch.randn(4, 16, 5, 5, requires_grad=True) if res else None
    ours, ref = BatchNorm2d(16), nn.BatchNorm2d(16)
    with torch.no_grad():
        ours.weight.uniform_(0.5, 1.5)
        ours.bias.uniform_(-0.5, 0.5)
    ref.load_state_dict(ours.state_dict())
    x2 = x.detach().clone().requires_grad_()
    r2 = r.detach().clone().requires_grad_() if res else None
    y = ours(x, r, relu)
    y2 = _reference(x2, ref, r2, relu)
    torch.testing.assert_close(y, y2)
    y.square().sum().backward()
    y2.square().sum().backward()
    torch.testing.assert_close(x.grad, x2.grad)
    torch.testing.assert_close(ours.weight.grad, ref.weight.grad)
    for k in ("running_mean", "running_var", "num_batches_tracked"):
        torch.testing.assert_close(getattr(ours, k), getattr(ref, k))
    ours.eval(), ref.eval()
    torch.testing.assert_close(ours(x, r, relu), _reference(x2, ref, r2, relu))


def test_resnet_uses_fused_bn_and_keeps_param_count():
    from pytorch_distributed_training_tutorials_amd.models.resnet import resnet50

    m = resnet50()
    assert sum(p.numel() for p in m.parameters()) == 25_557_032
    assert all(type(b) is BatchNorm2d for b in m.modules() if isinstance(b, nn.BatchNorm2d))


# ------------------------------------------------------------------------ GPU
SHAPES = [(4, 64, 14, 14), (2, 256, 7, 7), (3, 2048, 2, 2), (5, 24, 3, 3), (128, 64, 28, 28)]


@pytest.mark.gpu
@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("relu,res", [(False, False), (True, False), (True, True), (False, True)])
def test_native_bn_train_fwd_bwd(shape, dtype, relu, res):
    dev = torch.device("cuda", 0)
    C = shape[1]
    if C % (4 if dtype == torch.float32 else 8):
        pytest.skip("channel count not a multiple of the vector width (fallback path)")
    torch.manual_seed(sum(shape))
    x0 = (torch.randn(shape, device=dev) * 2 + 3).to(dtype).contiguous(memory_format=torch.channels_last)
    r0 = torch.randn(shape, device=dev).to(dtype).contiguous(memory_format=torch.channels_last) if res else None
    g0 = torch.randn(shape, device=dev).to(dtype).contiguous(memory_format=torch.channels_last)
    ours = BatchNorm2d(C).to(dev)
    with torch.no_grad():
        ours.weight.uniform_(0.5, 1.5)
        ours.bias.uniform_(-0.5, 0.5)
        ours.running_mean.uniform_(-1, 1)
    ref = nn.BatchNorm2d(C).to(dev)
    ref.load_state_dict(ours.state_dict())
    x = x0.clone().requires_grad_()
    r = r0.clone().requires_grad_() if res else None
    y = ours(x, r, relu)
    assert y.dtype == dtype and y.is_contiguous(memory_format=torch.channels_last)
    # fp32 reference on the same (rounded) inputs
    xr = x0.float().clone().requires_grad_()
    rr = r0.float().clone().requires_grad_() if res else None
    yr = _reference(xr, ref, rr, relu)
    tol = 2e-5 if dtype == torch.float32 else 2e-2
    torch.testing.assert_close(y.float(), yr, rtol=tol, atol=tol)
    y.backward(g0)
    yr.backward(g0.float())
    gtol = 1e-4 if dtype == torch.float32 else 5e-2
    # elements whose pre-ReLU value rounds to the other side of 0 flip their mask: skip them
    keep = (yr.detach().abs() > 1e-3) | (not relu)
    torch.testing.assert_close(x.grad.float()[keep], xr.grad[keep], rtol=gtol, atol=gtol)
    if res:
        torch.testing.assert_close(r.grad.float()[keep], rr.grad[keep], rtol=gtol, atol=gtol)
    wtol = 1e-3 * (x0.numel() / C) ** 0.5 if dtype == torch.bfloat16 else 1e-3
    torch.testing.assert_close(ours.weight.grad, ref.weight.grad, rtol=1e-3, atol=wtol)
    torch.testing.assert_close(ours.bias.grad, ref.bias.grad, rtol=1e-3, atol=wtol)
    torch.testing.assert_close(ours.running_mean, ref.running_mean, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(ours.running_var, ref.running_var, rtol=1e-4, atol=1e-5)
    assert int(ours.num_batches_tracked) == int(ref.num_batches_tracked) == 1
    # eval: running statistics, one launch, same epilogue
    ours.eval(), ref.eval()
    with torch.no_grad():
        torch.testing.assert_close(ours(x0, r0, relu).float(), _reference(x0.float(), ref, r0.float() if res else None,
                                                                          relu), rtol=tol, atol=tol)


@pytest.mark.gpu
def test_native_bn_large_mean_is_stable():
    """Shifted sums: |mean| = 1e3 * std must not cancel the variance."""
    dev = torch.device("cuda", 0)
    x = (torch.randn(64, 32, 8, 8, device=dev) + 1000.0).contiguous(memory_format=torch.channels_last)
    bn = BatchNorm2d(32).to(dev)
    y = bn(x)
    var = x.float().var(dim=(0, 2, 3), unbiased=False)
    ref = (x - x.mean(dim=(0, 2, 3), keepdim=True)) / torch.sqrt(var.view(1, -1, 1, 1) + bn.eps)
    torch.testing.assert_close(y, ref, rtol=1e-3, atol=1e-3)


@pytest.mark.gpu
def test_native_bn_2d_and_graph_replay_deterministic():
    """[M, C] input; two launches on the same stream give bit-identical stats (fixed-order combine)
    and the in-kernel ticket re-arm survives hipGraph replay."""
    dev = torch.device("cuda", 0)
    x = torch.randn(50000, 128, device=dev, dtype=torch.bfloat16)
    bn = BatchNorm2d(128).to(dev)
    bn.track_running_stats = False
    bn.running_mean = bn.running_var = bn.num_batches_tracked = None
    y1 = batch_norm_act(x, bn, relu=True)
    y2 = batch_norm_act(x, bn, relu=True)
    assert torch.equal(y1, y2)
    ref = F.relu(F.batch_norm(x.float(), None, None, bn.weight, bn.bias, True, 0.1, bn.eps))
    torch.testing.assert_close(y1.float(), ref, rtol=2e-2, atol=2e-2)
    out = torch.empty_like(y1)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        batch_norm_act(x, bn, relu=True)  # side-stream warmup before capture (torch.cuda.graph recipe)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out.copy_(batch_norm_act(x, bn, relu=True))
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, y1)


@pytest.mark.gpu
def test_resnet50_fused_bn_matches_plain_bn():
    """ResNet-50 (channels_last, fp32) with the fused BN path vs the same weights with
    nn.BatchNorm2d (MIOpen), both against a float64 CPU reference: the fused model's
    error must be at the level of the plain GPU model's (53 BNs, the deepest
    normalising 16 rows, amplify fp32 rounding on the way back to conv1)."""
    from pytorch_distributed_training_tutorials_amd.models.resnet import resnet50

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    ours = resnet50(num_classes=10).to(dev).to(memory_format=torch.channels_last)
    plain = resnet50(num_classes=10, norm_layer=nn.BatchNorm2d).to(dev).to(memory_format=torch.channels_last)
    plain.load_state_dict(ours.state_dict())
    ref = resnet50(num_classes=10, norm_layer=nn.BatchNorm2d).double()
    ref.load_state_dict(ours.state_dict())
    x = torch.randn(4, 3, 64, 64, device=dev).contiguous(memory_format=torch.channels_last)
    outs = [m(x.to(dtype=next(m.parameters()).dtype, device=next(m.parameters()).device))
            for m in (ours, plain, ref)]
    torch.testing.assert_close(outs[0], outs[1], rtol=2e-3, atol=2e-3)
    for o in outs:
        o.square().mean().backward()
    # ReLU masks flip where a pre-activation rounds across 0 (differently in each fp32 model), so
    # single small tensors scatter; the whole-model gradient error must match the plain model's
    d_ours = d_plain = ref_sq = 0.0
    for (n, p1), p2, p3 in zip(ours.named_parameters(), plain.parameters(), ref.parameters()):
        g = p3.grad
        e1 = (p1.grad.double().cpu() - g).norm().item() ** 2
        d_ours += e1
        d_plain += (p2.grad.double().cpu() - g).norm().item() ** 2
        ref_sq += g.norm().item() ** 2
        assert e1 ** 0.5 <= 0.1 * g.norm().item() + 1e-6, f"{n}: fused gradient off by {e1 ** 0.5:.3g}"
    e_ours, e_plain = (d_ours / ref_sq) ** 0.5, (d_plain / ref_sq) ** 0.5
    assert e_ours <= 3 * e_plain + 1e-3, f"whole-model gradient error: fused {e_ours:.3g} vs plain {e_plain:.3g}"


@pytest.mark.gpu
@pytest.mark.parametrize("shape,k,s,p", [((4, 64, 112, 112), 3, 2, 1), ((2, 32, 9, 7), 3, 2, 1),
                                         ((3, 16, 8, 8), 2, 2, 0), ((2, 24, 7, 5), 3, 1, 1)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_native_maxpool_nhwc_matches_torch(shape, k, s, p, dtype):
    from pytorch_distributed_training_tutorials_amd.ops.norm import MaxPool2d

    dev = torch.device("cuda", 0)
    torch.manual_seed(sum(shape))
    x0 = torch.randn(shape, device=dev).to(dtype).contiguous(memory_format=torch.channels_last)
    x = x0.clone().requires_grad_()
    xr = x0.float().clone().requires_grad_()
    y = MaxPool2d(k, s, p)(x)
    yr = F.max_pool2d(xr, k, s, p)
    assert y.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(y.float(), yr, rtol=0, atol=0)  # a max is exact
    g = torch.randn(yr.shape, device=dev).to(dtype)
    y.backward(g.contiguous(memory_format=torch.channels_last))
    yr.backward(g.float())
    tol = 1e-6 if dtype == torch.float32 else 2e-2  # overlapping windows: summation order
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=tol, atol=tol)


def test_maxpool_cpu_falls_back():
    from pytorch_distributed_training_tutorials_amd.ops.norm import MaxPool2d

    x = torch.randn(2, 8, 9, 9)
    torch.testing.assert_close(MaxPool2d(3, 2, 1)(x), F.max_pool2d(x, 3, 2, 1))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_residual_link_matches_autograd_add(dtype):
    """Identity shortcut between two fused BNs: the residual gradient handed to the
    producer's backward kernels (dy + dy2 in-kernel) equals autograd's add (fp32), and
    in bf16 is at least as close to the fp32 result as autograd's bf16 add."""
    from pytorch_distributed_training_tutorials_amd.ops.norm import BatchNorm2d

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    x0 = torch.randn(4, 64, 9, 7, device=dev).contiguous(memory_format=torch.channels_last)
    w0 = torch.randn(64, 64, 1, 1, device=dev).contiguous(memory_format=torch.channels_last) * 0.2

    def grads(dt, link):
        torch.manual_seed(1)
        bn_a, bn_b = BatchNorm2d(64).to(dev), BatchNorm2d(64).to(dev)
        x = x0.to(dt).clone().requires_grad_(True)
        y1 = bn_a(x, relu=True)                              # producer
        h = torch.nn.functional.conv2d(y1, w0.to(dt))        # the block's conv path
        y2 = bn_b(h, residual=y1, relu=True, link=link)      # consumer: identity shortcut
        (y2.float() * torch.linspace(-1, 1, y2.numel(), device=dev).view_as(y2)).sum().backward()
        return [t.grad.float().clone() for t in (x, bn_a.weight, bn_a.bias, bn_b.weight, bn_b.bias)]

    if dtype == torch.float32:
        for g0, g1 in zip(grads(dtype, False), grads(dtype, True)):
            torch.testing.assert_close(g1, g0, rtol=1e-4, atol=1e-5)
    else:
        truth = grads(torch.float32, False)
        for gt, g0, g1 in zip(truth, grads(dtype, False), grads(dtype, True)):
            e0, e1 = (g0 - gt).norm().item(), (g1 - gt).norm().item()
            assert e1 <= 1.5 * e0 + 1e-3 * gt.norm().item(), (e1, e0)


@pytest.mark.gpu
@pytest.mark.parametrize("taker", ["first", "third"])
def test_residual_link_two_deliverers_on_two_streams(taker):
    """Two consumers deliver a residual gradient on two streams and the producer takes it on the
    first deliverer's stream or on a third one: the taker must see the finished
    sum every time. The producers are slow elementwise chains, so a missing or wrong wait races."""
    from pytorch_distributed_training_tutorials_amd.ops.norm import ResidualLink

    dev = torch.device("cuda", 0)
    s1, s2, s3 = (torch.cuda.Stream(dev) for _ in range(3))
    base = torch.randn(1 << 22, device=dev)
    for rep in range(25):
        link = ResidualLink()
        torch.cuda.synchronize()
        with torch.cuda.stream(s1):
            a = base.clone()
            for _ in range(8):
                a = a * 1.0001 + 0.5
            link.put(a)
        with torch.cuda.stream(s2):
            b = base.clone()
            for _ in range(24):
                b = b * 0.9999 - 0.25
            link.put(b)  # waits for s1's delivery, adds on s2
        with torch.cuda.stream(s1 if taker == "first" else s3):
            got = link.take(dev).clone()
        torch.cuda.synchronize()
        assert torch.equal(got, a + b), f"repetition {rep}: the taker read an unfinished sum"


@pytest.mark.gpu
def test_residual_link_retain_graph_double_backward():
    """A retained graph run backward twice: every pass re-delivers the linked residual
    gradient, so the accumulated gradients equal 2x the un-linked autograd add."""
    from pytorch_distributed_training_tutorials_amd.ops.norm import BatchNorm2d

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    x0 = torch.randn(4, 64, 9, 7, device=dev).contiguous(memory_format=torch.channels_last)
    w0 = torch.randn(64, 64, 1, 1, device=dev).contiguous(memory_format=torch.channels_last) * 0.2

    def grads(link, passes):
        torch.manual_seed(1)
        bn_a, bn_b = BatchNorm2d(64).to(dev), BatchNorm2d(64).to(dev)
        x = x0.clone().requires_grad_(True)
        y1 = bn_a(x, relu=True)
        y2 = bn_b(torch.nn.functional.conv2d(y1, w0), residual=y1, relu=True, link=link)
        loss = (y2 * torch.linspace(-1, 1, y2.numel(), device=dev).view_as(y2)).sum()
        for k in range(passes):
            loss.backward(retain_graph=k + 1 < passes)
        return [t.grad.clone() for t in (x, bn_a.weight, bn_a.bias, bn_b.weight, bn_b.bias)]

    for g2, g1 in zip(grads(True, 2), grads(False, 1)):
        torch.testing.assert_close(g2, 2 * g1, rtol=1e-4, atol=1e-5)


def test_grad_link_delivers_branch_gradient_to_the_link():
    """ops.norm.grad_link: the linked branch's gradient goes to the producer's ResidualLink
    (summed later inside its backward kernels) instead of into autograd's sum."""
    from pytorch_distributed_training_tutorials_amd.ops.norm import ResidualLink, grad_link

    x = torch.randn(3, 4, requires_grad=True)
    h = x * 1.0  # a non-leaf "producer output"
    assert grad_link(h) is h  # no link: pass-through
    h._ptdt_res_link = ResidualLink()
    (h * 2.0).sum().backward(retain_graph=True)  # unlinked use only
    torch.testing.assert_close(x.grad, torch.full((3, 4), 2.0))
    x.grad = None
    hl = grad_link(h)
    ((h * 2.0).sum() + (hl * 3.0).sum()).backward()
    torch.testing.assert_close(x.grad, torch.full((3, 4), 2.0))  # the linked branch is not in autograd's sum
    torch.testing.assert_close(h._ptdt_res_link.dres, torch.full((3, 4), 3.0))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_grad_link_downsample_branch_matches_autograd_add(dtype):
    """A fused BN's output consumed by two convolutions (a ResNet downsample block's conv1 and
    downsample conv): with grad_link on one branch the two input gradients are summed inside
    the producer BN's backward; gradients equal autograd's add (fp32) / are as close (bf16)."""
    from pytorch_distributed_training_tutorials_amd.ops.norm import BatchNorm2d, grad_link

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    x0 = torch.randn(4, 64, 9, 7, device=dev).contiguous(memory_format=torch.channels_last)
    r0 = torch.randn(4, 64, 9, 7, device=dev).contiguous(memory_format=torch.channels_last)
    wa = torch.randn(32, 64, 1, 1, device=dev).contiguous(memory_format=torch.channels_last) * 0.2
    wb = torch.randn(32, 64, 1, 1, device=dev).contiguous(memory_format=torch.channels_last) * 0.2

    def grads(dt, link):
        torch.manual_seed(1)
        bn = BatchNorm2d(64).to(dev)
        x = x0.to(dt).clone().requires_grad_(True)
        y = bn(x, residual=r0.to(dt), relu=True)  # producer: a bn3 with residual (bit-mask path)
        yb = grad_link(y) if link else y
        out = torch.nn.functional.conv2d(y, wa.to(dt)) + 0.5 * torch.nn.functional.conv2d(yb, wb.to(dt))
        (out.float() * torch.linspace(-1, 1, out.numel(), device=dev).view_as(out)).sum().backward()
        return [t.grad.float().clone() for t in (x, bn.weight, bn.bias)]

    if dtype == torch.float32:
        for g0, g1 in zip(grads(dtype, False), grads(dtype, True)):
            torch.testing.assert_close(g1, g0, rtol=1e-4, atol=1e-5)
    else:
        truth = grads(torch.float32, False)
        for gt, g0, g1 in zip(truth, grads(dtype, False), grads(dtype, True)):
            e0, e1 = (g0 - gt).norm().item(), (g1 - gt).norm().item()
            assert e1 <= 1.5 * e0 + 1e-3 * gt.norm().item(), (e1, e0)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(8, 64, 56, 56), (3, 32, 17, 15)])
def test_bn_relu_maxpool_matches_composed(shape):
    """The ResNet stem fusion (BN apply + ReLU inside the pool's loads) vs BN-then-pool on the same
    native kernels: output bit-identical, gradients and running statistics equal."""
    import copy

    from pytorch_distributed_training_tutorials_amd.ops.norm import MaxPool2d, bn_relu_maxpool

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    bn1 = BatchNorm2d(shape[1]).to(dev)
    with torch.no_grad():
        bn1.weight.uniform_(-1.5, 1.5)  # negative scales too: the max is taken after the affine
        bn1.bias.uniform_(-0.5, 0.5)
    bn2 = copy.deepcopy(bn1)
    pool = MaxPool2d(kernel_size=3, stride=2, padding=1)
    x = torch.randn(*shape, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x1, x2 = x.clone().requires_grad_(), x.clone().requires_grad_()
    y1 = bn_relu_maxpool(x1, bn1, pool)
    y2 = pool(bn2(x2, relu=True))
    assert torch.equal(y1, y2)
    g = torch.randn_like(y1)
    y1.backward(g)
    y2.backward(g)
    assert torch.equal(x1.grad, x2.grad)
    torch.testing.assert_close(bn1.weight.grad, bn2.weight.grad)
    torch.testing.assert_close(bn1.bias.grad, bn2.bias.grad)
    for k in ("running_mean", "running_var", "num_batches_tracked"):
        torch.testing.assert_close(getattr(bn1, k), getattr(bn2, k))


_FENCE_PROBE = r"""
import sys, torch
from pytorch_distributed_training_tutorials_amd import native
C = native()
out = []
g = torch.Generator(device="cpu").manual_seed(11)
for M, Cn in ((128 * 56 * 56, 64), (128 * 28 * 28, 256), (128 * 7 * 7, 2048)):
    x = (torch.randn(M, Cn, generator=g) * 3 + 1).to("cuda", torch.bfloat16)
    y, st, _ = C.bn_fwd_train(x, None, None, None, None, None, None, True, 0.1, 1e-5, None, False)
    dy = torch.randn(M, Cn, generator=g).to("cuda", torch.bfloat16)
    dx, dw, db, _ = C.bn_bwd(dy, x, None, torch.ones(Cn, device="cuda"), st, True, False, True, None, None, None,
                             None, None)
    out.append(torch.cat([st.flatten(), dw.flatten(), db.flatten(), dx.float().flatten()[:65536]]).cpu())
torch.save(out, sys.argv[1])
"""


@pytest.mark.gpu
def test_bn_sc1_handoff_bit_identical_to_fence_handoff(tmp_path):
    """The last-block partial hand-off (relaxed ticket + sc1 stores/loads) gives the same
    bits as the fence-based form (PTDT_BN_FENCE=1, read once per process: two child processes) on
    many-block shapes: ResNet's 56x56x64, 28x28x256 and 7x7x2048 activations at batch 128."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = []
    for fence in ("0", "1"):
        path = str(tmp_path / f"f{fence}.pt")
        env = dict(os.environ, PTDT_BN_FENCE=fence, PYTHONPATH=root)
        p = subprocess.run([sys.executable, "-c", _FENCE_PROBE, path], env=env, capture_output=True, text=True,
                           timeout=240)
        assert p.returncode == 0, p.stderr[-3000:]
        res.append(torch.load(path, weights_only=True))
    for a, b in zip(*res):
        assert torch.equal(a, b)
