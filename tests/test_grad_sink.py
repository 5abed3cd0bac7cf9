"""Grad sinks (ops/conv.py): the weight cast's backward lands the gradient in the DDP
bucket slot and autograd adopts that view as .grad (no accumulate kernel)."""
import pytest
import torch
import torch.nn as nn

from pytorch_distributed_training_tutorials_amd.ops.conv import Conv2d, SinkCast


def test_sink_cast_backward_writes_into_sink_and_is_adopted():
    w = nn.Parameter(torch.randn(4, 3))
    buf = torch.full((12,), float("nan"))
    w._ptdt_grad_sink = lambda: buf.view(4, 3)
    y = SinkCast.apply(w, torch.bfloat16)
    assert y.dtype == torch.bfloat16
    (y.float() * torch.arange(12.0).view(4, 3)).sum().backward()
    torch.testing.assert_close(buf.view(4, 3), torch.arange(12.0).view(4, 3))
    assert w.grad.data_ptr() == buf.data_ptr()  # adopted, not cloned
    # .grad defined (accumulation): ordinary cast, autograd adds
    y = SinkCast.apply(w, torch.bfloat16)
    (y.float() * 2).sum().backward()
    torch.testing.assert_close(w.grad, torch.arange(12.0).view(4, 3) + 2)


def test_sink_claimed_once_per_forward_sums_tied_uses():
    """A weight cast twice in one forward (tied weights): the first backward claims the
    slot, the second returns an ordinary gradient and autograd sums both (ADVICE r1:
    writing both into the slot made the first contribution vanish)."""
    w = nn.Parameter(torch.randn(4, 3))
    buf = torch.full((12,), float("nan"))
    claimed = []

    def sink():  # the one-shot semantics of parallel.ddp's sinks
        if claimed:
            return None
        claimed.append(1)
        return buf.view(4, 3)

    w._ptdt_grad_sink = sink
    y1 = SinkCast.apply(w, torch.bfloat16)
    y2 = SinkCast.apply(w, torch.bfloat16)
    (y1.float().sum() * 1.0 + y2.float().sum() * 3.0).backward()
    torch.testing.assert_close(w.grad, torch.full((4, 3), 4.0))


def _deferring_sink(buf):
    """parallel.ddp's sink + deferred-cast protocol on one slot: claimed once, the cast recorded
    by index (no reference to the view autograd adopts) and landed by flush() or by defer(None, None)."""
    claimed, pending = [], []

    def sink():
        if claimed:
            return None
        claimed.append(1)
        return buf.view(4, 3)

    def flush():
        for g in pending:
            buf.view(4, 3).copy_(g)
        pending.clear()

    def defer(dst, src):
        if dst is None:
            flush()
        else:
            pending.append(src)
        return True
    return sink, defer, flush, pending


def test_deferred_cast_is_adopted_and_landed_by_flush():
    w = nn.Parameter(torch.randn(4, 3))
    buf = torch.zeros(12)
    sink, defer, flush, pending = _deferring_sink(buf)
    w._ptdt_grad_sink, w._ptdt_grad_defer = sink, defer
    (SinkCast.apply(w, torch.bfloat16).float() * torch.arange(12.0).view(4, 3)).sum().backward()
    assert len(pending) == 1 and w.grad.data_ptr() == buf.data_ptr()  # adopted, not copied
    flush()  # the bucket-completion flush
    torch.testing.assert_close(w.grad, torch.arange(12.0).view(4, 3))


def test_deferred_cast_tied_weight_lands_before_the_sum():
    """Two uses of one weight: the second backward finds the slot claimed and lands the first's
    deferred cast before autograd adds the two contributions into the slot."""
    w = nn.Parameter(torch.randn(4, 3))
    buf = torch.zeros(12)
    sink, defer, flush, pending = _deferring_sink(buf)
    w._ptdt_grad_sink, w._ptdt_grad_defer = sink, defer
    y1 = SinkCast.apply(w, torch.bfloat16)
    y2 = SinkCast.apply(w, torch.bfloat16)
    (y1.float().sum() * 1.0 + y2.float().sum() * 3.0).backward()
    flush()
    assert not pending
    torch.testing.assert_close(w.grad, torch.full((4, 3), 4.0))


def test_conv2d_is_a_drop_in_conv():
    a, b = Conv2d(3, 8, 3, padding=1), nn.Conv2d(3, 8, 3, padding=1)
    b.load_state_dict(a.state_dict())
    x = torch.randn(2, 3, 5, 5)
    torch.testing.assert_close(a(x), b(x))
    assert isinstance(a, nn.Conv2d)


def _small_net():
    from pytorch_distributed_training_tutorials_amd.ops.linear import Linear

    from pytorch_distributed_training_tutorials_amd.ops.norm import BatchNorm2d

    return nn.Sequential(Conv2d(3, 16, 3, padding=1), BatchNorm2d(16), nn.ReLU(), Conv2d(16, 32, 3, stride=2, padding=1),
                         nn.ReLU(), nn.AdaptiveAvgPool2d(1), nn.Flatten(), Linear(32, 10))


@pytest.mark.gpu
@pytest.mark.parametrize("defer", ["1", "0"])
def test_ddp_autocast_grads_land_in_buckets(defer, monkeypatch):
    """World-1 native DDP under bf16 autocast: every conv/linear weight grad is adopted as its
    bucket view (no accumulate kernel) and equals the plain model's grad, across zero_grad
    iterations and a no_sync accumulation; with deferred casts (default) the bf16 grads are
    converted per bucket by one multi-tensor launch and nothing is left pending after backward.
    (A small net: ResNet-50 in bf16 at toy batch sizes is chaotic -- two identical models
    already differ after a few BN layers.)"""
    from pytorch_distributed_training_tutorials_amd.parallel import env
    from pytorch_distributed_training_tutorials_amd.parallel.ddp import DistributedDataParallel

    monkeypatch.setenv("PTDT_DEFER_GRAD_CAST", defer)
    dev = torch.device("cuda", 0)
    if not torch.distributed.is_initialized():
        env.init_process_group("nccl")
    torch.manual_seed(0)
    m = _small_net().to(dev).to(memory_format=torch.channels_last)
    ref = _small_net().to(dev).to(memory_format=torch.channels_last)
    ref.load_state_dict(m.state_dict())
    ddp = DistributedDataParallel(m, device_ids=[0])
    assert len(ddp._sink_params) == 5  # 2 conv + BN weight/bias + linear weight
    assert ddp._defer == (defer == "1")
    flushes = []
    if ddp._defer:
        orig = ddp._flush_casts
        ddp._flush_casts = lambda b=None: (flushes.append((b, len(ddp._pending.get(b, ())) if b is not None
                                                            else sum(map(len, ddp._pending.values())))), orig(b))
    xs = [torch.randn(16, 3, 32, 32, device=dev).contiguous(memory_format=torch.channels_last) for _ in range(3)]

    def loss(model, x):
        with torch.autocast("cuda", torch.bfloat16):
            return model(x).float().square().mean()

    for it in range(2):
        ddp.zero_grad()
        ref.zero_grad(set_to_none=True)
        loss(ddp, xs[it]).backward()
        loss(ref, xs[it]).backward()
        torch.cuda.synchronize()
        if ddp._defer:  # 3 weights through SinkCast (2 conv + linear), cast in per-bucket batches
            assert not ddp._pending and sum(n for _, n in flushes) == 3 * (it + 1)
        spans = [(f.data_ptr(), f.data_ptr() + f.numel() * f.element_size()) for f in ddp.reducer.bucket_tensors()]
        for p in ddp._sink_params:
            assert any(lo <= p.grad.data_ptr() < hi for lo, hi in spans)
        for (n, p1), p2 in zip(m.named_parameters(), ref.parameters()):
            rel = ((p1.grad - p2.grad).norm() / (p2.grad.norm() + 1e-12)).item()
            assert rel < 2e-2, f"iteration {it}, {n}: {rel}"
    # accumulation: grads defined -> the ordinary cast + autograd add
    with ddp.no_sync():
        loss(ddp, xs[2]).backward()
    loss(ref, xs[2]).backward()
    for (n, p1), p2 in zip(m.named_parameters(), ref.parameters()):
        rel = ((p1.grad - p2.grad).norm() / (p2.grad.norm() + 1e-12)).item()
        assert rel < 2e-2, f"no_sync accumulation, {n}: {rel}"


def test_ddp_remove_grad_sinks_cpu_is_noop_and_gpu_detaches():
    """remove_grad_sinks() clears every installed sink (CPU wrappers install none)."""
    import torch.distributed as dist

    from pytorch_distributed_training_tutorials_amd.parallel import comm as comm_mod
    from pytorch_distributed_training_tutorials_amd.parallel.ddp import DistributedDataParallel

    from pytorch_distributed_training_tutorials_amd.parallel.env import free_port

    own = not dist.is_initialized()
    if own:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{free_port()}", rank=0, world_size=1)
    try:
        m = nn.Sequential(Conv2d(3, 4, 3))
        ddp = DistributedDataParallel(m, comm=comm_mod.get_default(None))
        assert ddp._sink_params == []
        m[0].weight._ptdt_grad_sink = lambda: None
        ddp._sink_params = [m[0].weight]
        ddp.remove_grad_sinks()
        assert getattr(m[0].weight, "_ptdt_grad_sink", None) is None
    finally:
        if own:
            dist.destroy_process_group()


@pytest.mark.gpu
def test_ddp_autocast_tied_weight_grads_are_summed():
    """A Linear applied twice per forward under bf16 autocast with native DDP: its weight
    gradient is the sum of both uses (the plain model's), not the last one."""
    from pytorch_distributed_training_tutorials_amd.ops.linear import Linear
    from pytorch_distributed_training_tutorials_amd.parallel import env
    from pytorch_distributed_training_tutorials_amd.parallel.ddp import DistributedDataParallel

    class Twice(nn.Module):
        def __init__(self):
            super().__init__()
            self.lin = Linear(16, 16)

        def forward(self, x):
            return self.lin(torch.relu(self.lin(x)))

    env.init_process_group("nccl")
    try:
        dev = torch.device("cuda", 0)
        torch.manual_seed(0)
        m = Twice().to(dev)
        ref = Twice().to(dev)
        ref.load_state_dict(m.state_dict())
        ddp = DistributedDataParallel(m, device_ids=[0])
        x = torch.randn(8, 16, device=dev)
        for _ in range(2):
            ddp.zero_grad()
            ref.zero_grad()
            with torch.autocast("cuda", torch.bfloat16):
                ddp(x).float().sum().backward()
                ref(x).float().sum().backward()
            torch.testing.assert_close(m.lin.weight.grad, ref.lin.weight.grad, rtol=2e-2, atol=2e-2)
        ddp.remove_grad_sinks()
    finally:
        env.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("defer", ["1", "0"])
def test_ddp_tied_weight_with_fp32_embedding_use(defer, monkeypatch):
    """A Linear head whose weight is also read by an fp32 F.embedding (tied embedding / lm_head):
    one use goes through SinkCast (deferred cast into a slot zero_grad did not clear), the other
    does not. Both gradients must survive every step (the pending cast overwrote the
    sum from the second step on, when the slot holds the previous step's gradient)."""
    import torch.nn.functional as F

    from pytorch_distributed_training_tutorials_amd.ops.linear import Linear
    from pytorch_distributed_training_tutorials_amd.parallel import env
    from pytorch_distributed_training_tutorials_amd.parallel.ddp import DistributedDataParallel

    monkeypatch.setenv("PTDT_DEFER_GRAD_CAST", defer)

    class Tied(nn.Module):
        def __init__(self):
            super().__init__()
            self.head = Linear(16, 40)  # weight [40, 16] doubles as a 40-token embedding table

        def forward(self, idx):
            return self.head(F.embedding(idx, self.head.weight))

    env.init_process_group("nccl")
    try:
        dev = torch.device("cuda", 0)
        torch.manual_seed(0)
        m = Tied().to(dev)
        ref = Tied().to(dev)
        ref.load_state_dict(m.state_dict())
        ddp = DistributedDataParallel(m, device_ids=[0])
        for step in range(4):
            idx = torch.randint(0, 40, (8,), device=dev)
            ddp.zero_grad()
            ref.zero_grad()
            with torch.autocast("cuda", torch.bfloat16):
                (ddp(idx).float() ** 2).sum().backward()
                (ref(idx).float() ** 2).sum().backward()
            torch.testing.assert_close(m.head.weight.grad, ref.head.weight.grad, rtol=2e-2, atol=2e-2,
                                       msg=lambda s, step=step: f"step {step}: {s}")
            torch.testing.assert_close(m.head.bias.grad, ref.head.bias.grad, rtol=2e-2, atol=2e-2)
        ddp.remove_grad_sinks()
    finally:
        env.destroy_process_group()


@pytest.mark.gpu
def test_fused_sgd_bf16_shadow_replaces_autocast_cast():
    """FusedSGD(bf16_shadow=True) writes bf16(p) in the update kernel; conv under bf16
    autocast then uses it (no per-forward cast) and the training trajectory is the
    same as with the cast; a weight changed outside the optimizer invalidates it."""
    from pytorch_distributed_training_tutorials_amd.ops.conv import Conv2d, cast_weight
    from pytorch_distributed_training_tutorials_amd.ops.optim import FusedSGD

    dev = torch.device("cuda", 0)
    x = torch.randn(4, 8, 10, 10, device=dev).contiguous(memory_format=torch.channels_last)
    outs = []
    for shadow in (False, True):
        torch.manual_seed(0)
        conv = Conv2d(8, 16, 3, padding=1).to(dev).to(memory_format=torch.channels_last)
        opt = FusedSGD(conv.parameters(), lr=0.1, momentum=0.9, bf16_shadow=shadow)
        for _ in range(3):
            opt.zero_grad()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = conv(x)
            y.float().square().mean().backward()
            opt.step()
        outs.append([p.detach().clone() for p in conv.parameters()])
        if shadow:
            w = conv.weight
            assert torch.equal(w._ptdt_bf16, w.detach().to(torch.bfloat16))
            with torch.autocast("cuda", dtype=torch.bfloat16):
                assert cast_weight(w).data_ptr() == w._ptdt_bf16.data_ptr()
                with torch.no_grad():
                    w.mul_(0.5)  # outside the optimizer: the shadow is stale now
                assert cast_weight(w).data_ptr() != w._ptdt_bf16.data_ptr()
    for a, b in zip(*outs):  # (MIOpen's weight-gradient solvers may sum in any order: not bitwise)
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


def test_same_dense_layout_ignores_unit_dims():
    """A 1x1-conv weight gradient from MIOpen may carry channels_last strides on its size-1 dims;
    it is still the slot's layout (the deferred cast must not fall back to a per-tensor copy)."""
    from pytorch_distributed_training_tutorials_amd.parallel.ddp import _same_dense_layout

    base = torch.empty(64 * 256)
    a = base.as_strided((64, 256, 1, 1), (256, 1, 1, 1))
    b = base.as_strided((64, 256, 1, 1), (256, 1, 256, 256))
    assert _same_dense_layout(a, b)
    c = torch.empty(64, 256, 3, 3).contiguous(memory_format=torch.channels_last)
    assert not _same_dense_layout(c, torch.empty(64, 256, 3, 3))
    assert _same_dense_layout(c, torch.empty_like(c))


@pytest.mark.gpu
def test_rgb_stem_conv_padded_under_autocast():
    """Conv2d with 3 input channels under bf16 autocast runs as a 4-channel convolution (zero input
    channel, zero weight slice): same output and weight gradient as the plain bf16 convolution."""
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    conv = Conv2d(3, 64, 7, stride=2, padding=3, bias=False).to(dev).to(memory_format=torch.channels_last)
    ref = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False).to(dev).to(memory_format=torch.channels_last)
    ref.load_state_dict(conv.state_dict())
    x = torch.randn(4, 3, 64, 64, device=dev).contiguous(memory_format=torch.channels_last)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y, yr = conv(x), ref(x)
    assert y.shape == yr.shape == (4, 64, 32, 32)
    torch.testing.assert_close(y.float(), yr.float(), rtol=2e-2, atol=2e-2)
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g)
    assert conv.weight.grad.shape == (64, 3, 7, 7)
    torch.testing.assert_close(conv.weight.grad, ref.weight.grad, rtol=2e-2, atol=5e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_rgb4_pack_matches_torch(dtype):
    from pytorch_distributed_training_tutorials_amd import native

    dev = torch.device("cuda", 0)
    x = torch.randn(3, 3, 17, 9, device=dev, dtype=dtype).contiguous(memory_format=torch.channels_last)
    y = native().rgb4_pack(x)
    assert y.shape == (3, 4, 17, 9) and y.dtype == torch.bfloat16
    assert y.is_contiguous(memory_format=torch.channels_last)
    ref = torch.cat([x.to(torch.bfloat16), torch.zeros(3, 1, 17, 9, device=dev, dtype=torch.bfloat16)], 1)
    assert torch.equal(y, ref)
