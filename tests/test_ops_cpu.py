"""CPU paths: op fallbacks, optimizers, flat parameters, bucket planning, checkpoints."""
import pytest
import torch
import torch.nn.functional as F

from pytorch_distributed_training_tutorials_amd import native
from pytorch_distributed_training_tutorials_amd.models.toy import SampleModel, ToyMLP, ToyModel, ddp_toy_model, model_size
from pytorch_distributed_training_tutorials_amd.ops import FusedAdam, FusedSGD, cross_entropy, linear, mse_loss
from pytorch_distributed_training_tutorials_amd.ops.flat import FlatParameters, contiguous_span
from pytorch_distributed_training_tutorials_amd.parallel import bucketing
from pytorch_distributed_training_tutorials_amd.utils.checkpoint import load_checkpoint, save_checkpoint


def test_reference_zero_loss_quirk_cpu():
    """Q1: CE on [B,1] logits with float [B,1] targets is identically zero (and so are grads)."""
    m = ddp_toy_model()
    x, y = torch.rand(32, 20), torch.rand(32, 1)
    loss = cross_entropy(m(x), y)
    loss.backward()
    assert loss.item() == 0.0
    assert (m.weight.grad == 0).all() and (m.bias.grad == 0).all()


def test_linear_and_losses_cpu_match_torch():
    x = torch.randn(5, 7)
    w, b = torch.randn(3, 7), torch.randn(3)
    torch.testing.assert_close(linear(x, w, b, True), F.relu(F.linear(x, w, b)))
    t = torch.randint(0, 3, (5,))
    torch.testing.assert_close(cross_entropy(x[:, :3], t), F.cross_entropy(x[:, :3], t))
    torch.testing.assert_close(mse_loss(x, x * 2), F.mse_loss(x, x * 2))


def test_model_param_counts():
    assert model_size(ddp_toy_model()) == 21
    assert model_size(SampleModel(32, 2)) == 66
    assert model_size(ToyModel("cpu", "cpu")) == 100_065
    assert list(ToyModel("cpu", "cpu").state_dict()) == ["net1.weight", "net1.bias", "net2.weight", "net2.bias"]


@pytest.mark.parametrize("kw", [dict(lr=0.1), dict(lr=0.1, momentum=0.9, weight_decay=1e-2),
                                dict(lr=0.1, momentum=0.9, nesterov=True)])
def test_fused_sgd_cpu(kw):
    torch.manual_seed(0)
    a = ToyMLP(4, 8, 3)
    b = ToyMLP(4, 8, 3)
    b.load_state_dict(a.state_dict())
    oa, ob = FusedSGD(a.parameters(), **kw), torch.optim.SGD(b.parameters(), **kw)
    for _ in range(3):
        x = torch.randn(6, 4)
        for m, o in ((a, oa), (b, ob)):
            o.zero_grad()
            m(x).pow(2).mean().backward()
            o.step()
    for p, q in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(p, q)


def test_fused_adam_cpu():
    torch.manual_seed(0)
    a = ToyMLP(4, 8, 3)
    b = ToyMLP(4, 8, 3)
    b.load_state_dict(a.state_dict())
    oa, ob = FusedAdam(a.parameters(), lr=1e-2), torch.optim.Adam(b.parameters(), lr=1e-2)
    for _ in range(3):
        x = torch.randn(6, 4)
        for m, o in ((a, oa), (b, ob)):
            o.zero_grad()
            m(x).pow(2).mean().backward()
            o.step()
    for p, q in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(p, q)


def test_flat_parameters_views():
    m = ToyMLP(4, 8, 3)
    ref = {k: v.clone() for k, v in m.state_dict().items()}
    fp = FlatParameters(list(m.parameters()), with_grads=True)
    flat = fp.flat()
    assert flat.numel() == sum(p.numel() for p in m.parameters())
    for k, v in m.state_dict().items():
        torch.testing.assert_close(v, ref[k])
    span = contiguous_span([p.data for p in m.parameters()])
    assert span is not None and span.data_ptr() == flat.data_ptr()
    flat.fill_(1.0)
    assert all((p == 1).all() for p in m.parameters())
    assert contiguous_span([torch.zeros(3), torch.zeros(3)]) is None


def test_bucket_plan_reverse_order_and_caps():
    ps = [torch.zeros(n) for n in (10, 20, 30, 40)]
    plan = bucketing.plan(ps, first_cap_bytes=100, cap_bytes=200)
    assert plan[0] == [3]  # 160 B >= first cap -> first bucket closes after the last layer
    assert sorted(i for b in plan for i in b) == [0, 1, 2, 3]
    first, cap = bucketing.xgmi_bucket_caps(8)
    assert first == 1 << 20 and 16 << 20 <= cap <= 64 << 20
    mixed = [torch.zeros(4), torch.zeros(4, dtype=torch.float64), torch.zeros(4)]
    for b in bucketing.plan(mixed, first_cap_bytes=1 << 30, cap_bytes=1 << 30):
        assert len({mixed[i].dtype for i in b}) == 1


def test_resnet_like_bucket_counts():
    """ResNet-50-sized grads under torch defaults -> 5 fp32 buckets."""
    from pytorch_distributed_training_tutorials_amd.models.resnet import resnet50

    m = resnet50()
    ps = [p for p in m.parameters()]
    assert sum(p.numel() for p in ps) == 25_557_032
    plan = bucketing.plan(ps, first_cap_bytes=1 << 20, cap_bytes=25 << 20)
    assert 4 <= len(plan) <= 6


def test_checkpoint_roundtrip_with_module_prefix(tmp_path):
    from pytorch_distributed_training_tutorials_amd.utils.trainer import _ModuleView

    m = _ModuleView(ToyMLP(4, 8, 3))
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9)
    m(torch.randn(2, 4)).sum().backward()
    opt.step()
    path = str(tmp_path / "ck.pt")
    save_checkpoint(path, m, opt, epoch=4)
    m2 = ToyMLP(4, 8, 3)  # bare module accepts the DDP-prefixed checkpoint
    st = load_checkpoint(path, m2)
    assert st["epoch"] == 4
    for p, q in zip(m.module.parameters(), m2.parameters()):
        torch.testing.assert_close(p, q)


def test_native_extension_importable_on_cpu():
    C = native()
    assert C.ARCH == "gfx950"


def test_persistent_engine_selection():
    """Host-side dispatch: Linear(Din, Dout) with B <= 64 and an instantiated
    (features per lane, Dout) pair runs the single-wave engine; anything else the
    workgroup engine."""
    C = native()
    ce_soft, ce_index = 0, 1
    # flagship toy: layout F (4 feature groups x 16 row slots), 2 rows per slot, 5 features per lane
    assert C.persistent_engine(32, 20, 0, 1, ce_soft, 2048, 1) == "wave:L0R2K5"
    assert C.persistent_engine(32, 20, 0, 1, ce_soft, 2048, 1, 3) == "wave:L4R2K5"  # row-group layouts only
    assert C.persistent_engine(32, 20, 0, 1, ce_soft, 256, 8).startswith("wave")  # 8 ranks
    assert C.persistent_engine(64, 16, 0, 1, ce_soft, 1000, 1).startswith("wave")
    # hidden layer: the 4-wave MFMA step body when the shape fits it, the LDS dot-product body otherwise
    assert C.persistent_engine(32, 20, 64, 10, ce_index, 2048, 1) == "tp:4waves"  # tensor-parallel MFMA engine
    # b1 rides in W1 as input column Din: Din + bias <= 32
    assert C.persistent_engine(32, 32, 64, 10, ce_index, 2048, 1, 0, False) == "tp:4waves"
    assert C.persistent_engine(32, 32, 64, 10, ce_index, 2048, 1, 0, True) == "workgroup:mfma"
    assert C.persistent_engine(32, 20, 64, 10, ce_index, 2048, 1, 5) == "workgroup:mfma"  # forced
    assert C.persistent_engine(32, 20, 64, 10, ce_index, 2048, 1, 1) == "workgroup"  # forced
    assert C.persistent_engine(64, 20, 64, 10, ce_index, 2048, 1) == "workgroup"  # B > 32
    assert C.persistent_engine(32, 20, 100, 10, ce_index, 2048, 1) == "workgroup"  # H not a multiple of 16
    assert C.persistent_engine(128, 20, 0, 1, ce_soft, 2048, 1) == "workgroup"  # B > 64
    assert C.persistent_engine(32, 20, 0, 10, ce_index, 2048, 1) == "workgroup"  # Dout 10 not instantiated
    assert C.persistent_engine(32, 20, 0, 1, ce_soft, 2048, 1, 1) == "workgroup"  # forced


def test_fused_adam_state_dict_resume_and_torch_interchange():
    """FusedAdam's bias-correction step travels in the state_dict (torch layout): 3 steps +
    save/load + 2 steps == 5 uninterrupted torch.optim.Adam steps, and the state loads into
    torch.optim.Adam too (the step counter used to be dropped)."""
    from pytorch_distributed_training_tutorials_amd.ops.optim import FusedAdam

    def run(cls, steps, params, sd=None):
        opt = cls(params, lr=1e-2)
        if sd is not None:
            opt.load_state_dict(sd)
        for _ in range(steps):
            for p in params:
                p.grad = torch.sin(p.detach() * 3) + 0.1
            opt.step()
        return opt

    torch.manual_seed(0)
    p0 = [torch.nn.Parameter(torch.randn(5, 3)), torch.nn.Parameter(torch.randn(4))]
    clone = lambda ps: [torch.nn.Parameter(t.detach().clone()) for t in ps]  # noqa: E731
    ref = clone(p0)
    run(torch.optim.Adam, 5, ref)
    a = clone(p0)
    sd = run(FusedAdam, 3, a).state_dict()
    assert all(float(v["step"]) == 3.0 for v in sd["state"].values())
    for cls in (FusedAdam, torch.optim.Adam):
        b = clone(a)
        run(cls, 2, b, sd)
        for x, y in zip(b, ref):
            torch.testing.assert_close(x, y, rtol=1e-5, atol=1e-6)


def test_conv_bn_act_falls_back_off_gpu():
    """ops.convbn.conv_bn_act on CPU tensors is exactly the unfused bn_act(bn, conv(x))."""
    import copy

    from pytorch_distributed_training_tutorials_amd.models.resnet import bn_act, conv1x1
    from pytorch_distributed_training_tutorials_amd.ops.convbn import _fusable, conv_bn_act
    from pytorch_distributed_training_tutorials_amd.ops.norm import BatchNorm2d

    torch.manual_seed(0)
    conv, bn = conv1x1(64, 32), BatchNorm2d(32)
    conv2, bn2 = copy.deepcopy(conv), copy.deepcopy(bn)
    x = torch.randn(2, 64, 5, 5)
    assert not _fusable(conv, bn, x, None)
    y = conv_bn_act(conv, bn, x, relu=True)
    torch.testing.assert_close(y, bn_act(bn2, conv2(x), relu=True))
    torch.testing.assert_close(bn.running_var, bn2.running_var)


def test_residual_link_put_take_cpu():
    """ops.norm.ResidualLink: the first consumer stores, a second one adds, the producer takes and
    clears (CPU tensors: no stream bookkeeping); None when no consumer delivered."""
    import torch

    from pytorch_distributed_training_tutorials_amd.ops.norm import ResidualLink

    link = ResidualLink()
    assert link.take(torch.device("cpu")) is None
    a, b = torch.ones(3), torch.full((3,), 2.0)
    link.put(a)
    link.put(b)
    got = link.take(torch.device("cpu"))
    assert torch.equal(got, torch.full((3,), 3.0))
    assert link.dres is None and link.stream is None
