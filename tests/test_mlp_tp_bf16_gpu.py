"""bf16 tensor-parallel toy-MLP engine (csrc/kernels/mlp_tp_impl.h, BF; BASELINE.json config 2
"toy MLP bf16") against plain PyTorch references of the same DDP steps:
(a) fp32 PyTorch with bf16 rounding at torch.autocast(bfloat16)'s rounding points (tight),
(b) torch.autocast(bfloat16) itself (hipBLASLt bf16 GEMMs; tight up to accumulation order),
(c) plain fp32 (bf16 tolerance); 40 steps across launches and epoch boundaries."""
import os

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from pytorch_distributed_training_tutorials_amd.parallel.env import free_port
from pytorch_distributed_training_tutorials_amd.parallel.launcher import spawn

from . import _workers
from ._tp_ref import ddp_reference
from .test_mlp_tp_gpu import _data, _epoch_orders

pytestmark = pytest.mark.gpu


def _autocast_reference(model, X, Y, order, B, loss, steps, lr, mom):
    opt = torch.optim.SGD(model.parameters(), lr=lr, momentum=mom)
    S = -(-order[0].numel() // B)
    for k in range(steps):
        e, j = divmod(k, S)
        idx = order[e][j * B:(j + 1) * B].long()
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = model(X[idx])
            l = F.mse_loss(out, Y[idx]) if loss == "mse" else F.cross_entropy(out, Y[idx])
        l.backward()
        opt.step()


def _flat(ps):
    return torch.cat([p.detach().reshape(-1).float() for p in ps])


@pytest.mark.parametrize("B,Din,H,Dout,loss,bias", [
    (32, 20, 64, 10, "ce_index", True),   # the BASELINE toy MLP
    (32, 20, 64, 10, "ce_soft", True),
    (16, 7, 32, 3, "ce_soft", True),      # one input tile (dW1: MT = 1), odd Din (scalar staging)
    (32, 31, 16, 16, "mse", True),        # Din + bias = 32: the whole K = 32 input step
    (32, 32, 16, 16, "mse", False),
    (24, 20, 48, 1, "ce_soft", True),     # the reference's one-class zero-loss shape
    (32, 17, 64, 10, "ce_index", False),
    (8, 4, 16, 2, "mse", True),
    (32, 12, 64, 10, "ce_index", True),   # one tile, float4 staging
])
def test_tp_bf16_engine_matches_references(dev, B, Din, H, Dout, loss, bias):
    from pytorch_distributed_training_tutorials_amd.data.device_sampler import DeviceDistributedSampler
    from pytorch_distributed_training_tutorials_amd.ops.fused_step import FusedMLPStep

    N = 7 * B + 5  # a partial batch at every epoch end
    X, Y = _data(dev, N, Din, Dout, loss, B + Din + H)
    steps, lr, mom = 40, 0.05, 0.9
    torch.manual_seed(3)
    mk = lambda: nn.Sequential(nn.Linear(Din, H, bias=bias), nn.ReLU(), nn.Linear(H, Dout, bias=bias)).to(dev)  # noqa: E731
    m_tp, m_ac, m_32 = mk(), mk(), mk()
    m_ac.load_state_dict(m_tp.state_dict())
    m_32.load_state_dict(m_tp.state_dict())
    init = [m_tp[0].weight, m_tp[0].bias, m_tp[2].weight, m_tp[2].bias]
    init = [None if p is None else p.detach().clone() for p in init]
    eng = FusedMLPStep(m_tp, loss=loss, lr=lr, momentum=mom, dtype="bf16")
    sampler = DeviceDistributedSampler(N, 1, 0, seed=2, device=dev)
    assert eng.persistent_engine(B, sampler) == f"tp_bf16:{H // 16}waves"
    order = _epoch_orders(sampler, 6, dev)
    cursor = torch.zeros(2, dtype=torch.int32, device=dev)
    losses = torch.zeros(steps, device=dev)
    plan = eng.persistent_plan(X, Y, B, sampler, cursor, losses)
    for n in (1, 12, 20, 7):  # launches start mid-epoch and cross epoch boundaries
        plan.launch(n)
    torch.cuda.synchronize()
    S = -(-N // B)
    assert cursor.tolist() == [steps // S, steps % S]
    got = _flat(m_tp.parameters())
    assert torch.isfinite(got).all()
    # (a) bf16 rounding emulated in fp32 PyTorch: the same arithmetic up to fp32 summation order
    em_p, em_g, em_l = ddp_reference(init, X, Y, [order], B, loss, steps, lr, mom, "emulate")
    torch.testing.assert_close(got, _flat(em_p), rtol=2e-3, atol=2e-4)
    torch.testing.assert_close(losses[:7].cpu(), torch.tensor(em_l[-7:]), rtol=5e-3, atol=5e-4)
    torch.testing.assert_close(eng.G, _flat(em_g), rtol=2e-2, atol=2e-4)  # DDP bucket: last step's bf16 grads
    # (b) torch.autocast(bfloat16) on the same batches
    _autocast_reference(m_ac, X, Y, order, B, loss, steps, lr, mom)
    torch.testing.assert_close(got, _flat(m_ac.parameters()), rtol=5e-3, atol=5e-4)
    # (c) plain fp32 at bf16 tolerance: 40 momentum-SGD steps amplify single-element bf16 differences
    # (ReLU masks flip), so the trajectory is compared in norm and the losses per step
    f32_p, _, f32_l = ddp_reference(init, X, Y, [order], B, loss, steps, lr, mom, "fp32")
    want = _flat(f32_p)
    assert float((got - want).norm() / want.norm()) < 5e-2  # (bf16 inputs: 8 x 4 batches measured 3.4 %)
    torch.testing.assert_close(got, want, rtol=0.0, atol=6e-2)
    torch.testing.assert_close(losses[:7].cpu(), torch.tensor(f32_l[-7:]), rtol=5e-2, atol=1e-2)


def test_tp_bf16_plan_splits_equal_one_launch(dev):
    """Launch splits, the list cache and epoch boundaries change nothing (bitwise)."""
    from pytorch_distributed_training_tutorials_amd.data.device_sampler import DeviceDistributedSampler
    from pytorch_distributed_training_tutorials_amd.models.toy import ToyMLP
    from pytorch_distributed_training_tutorials_amd.ops.fused_step import FusedMLPStep

    N = 300
    X, Y = _data(dev, N, 20, 10, "ce_index", 11)
    out = []
    for splits in ((37,), (1, 2, 3, 5, 26)):
        torch.manual_seed(1)
        eng = FusedMLPStep(ToyMLP(20, 64, 10).to(dev), loss="ce_index", lr=0.05, momentum=0.9, dtype="bf16")
        sampler = DeviceDistributedSampler(N, 1, 0, seed=4, device=dev)
        cursor = torch.zeros(2, dtype=torch.int32, device=dev)
        losses = torch.zeros(37, device=dev)
        plan = eng.persistent_plan(X, Y, 16, sampler, cursor, losses)
        for n in splits:
            plan.launch(n)
        torch.cuda.synchronize()
        out.append(eng.P.clone())
    assert torch.equal(out[0], out[1])


def test_tp_bf16_rejects_other_engines(dev):
    from pytorch_distributed_training_tutorials_amd.data.device_sampler import DeviceDistributedSampler
    from pytorch_distributed_training_tutorials_amd.models.toy import ToyMLP, ddp_toy_model
    from pytorch_distributed_training_tutorials_amd.ops.fused_step import FusedMLPStep

    eng = FusedMLPStep(ToyMLP(20, 64, 10).to(dev), loss="ce_index", dtype="bf16")
    s = DeviceDistributedSampler(64, 1, 0, device=dev)
    with pytest.raises(ValueError):
        eng.persistent_engine(32, s, "wave")
    with pytest.raises(NotImplementedError):
        eng.step(torch.zeros(32, 20, device=dev), torch.zeros(32, dtype=torch.long, device=dev), None, 32)
    with pytest.raises(ValueError):
        FusedMLPStep(ddp_toy_model().to(dev), dtype="bf16")


@pytest.mark.parametrize("world", [2, 4, 8])
def test_tp_bf16_ranks_one_gpu(tmp_path, world):
    """W ranks sharing cuda:0 (in-kernel xGMI exchange over IPC buffers): bit-identical replicas,
    equal to one process averaging the ranks' bf16 gradients in rank order."""
    spawn(_workers.tp_bf16_ranks_one_gpu, args=(world, free_port(), str(tmp_path)), nprocs=world)
    res = [torch.load(os.path.join(tmp_path, f"r{r}.pt"), weights_only=True) for r in range(world)]
    assert all(r["engine"] == "tp_bf16:4waves" for r in res)
    for r in res[1:]:
        assert torch.equal(r["params"], res[0]["params"])
    X, Y = res[0]["X"], res[0]["Y"]
    orders = [r["orders"] for r in res]
    em_p, _, _ = ddp_reference(res[0]["init"], X, Y, orders, 16, "ce_index", 23, 0.05, 0.9, "emulate")
    torch.testing.assert_close(res[0]["params"], _flat(em_p), rtol=2e-3, atol=2e-4)
