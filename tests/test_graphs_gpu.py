"""Whole-step hipGraph capture (utils/graphs.py): a DDP ResNet-50 training step
(native conv weight casts with grad sinks, fused BN, DDP reducer, FusedSGD with
bf16 shadows) replayed from one captured graph follows the same trajectory as the
same steps launched eagerly."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pg():
    from pytorch_distributed_training_tutorials_amd.parallel import env

    env.init_process_group("nccl")
    yield
    env.destroy_process_group()


def _run(dev, graphed: bool, steps: int, init_state):
    from pytorch_distributed_training_tutorials_amd.models.resnet import resnet50
    from pytorch_distributed_training_tutorials_amd.ops.loss import cross_entropy
    from pytorch_distributed_training_tutorials_amd.ops.optim import FusedSGD
    from pytorch_distributed_training_tutorials_amd.parallel import comm as comm_mod
    from pytorch_distributed_training_tutorials_amd.parallel.ddp import DistributedDataParallel
    from pytorch_distributed_training_tutorials_amd.utils.graphs import GraphedStep

    comm = comm_mod.get_default(dev)
    model = resnet50(num_classes=10).to(dev).to(memory_format=torch.channels_last)
    model.load_state_dict(init_state)
    ddp = DistributedDataParallel(model, device_ids=[dev.index], comm=comm)
    opt = FusedSGD(model.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4, bf16_shadow=True)
    g = torch.Generator(device="cpu").manual_seed(7)
    x = torch.randn(4, 3, 64, 64, generator=g).to(dev).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (4,), generator=g).to(dev)

    def step():
        ddp.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=not graphed):
            out = ddp(x)
        loss = cross_entropy(out.float(), y)
        loss.backward()
        opt.step()
        return loss

    losses = []
    if graphed:
        warm = 2
        # the warm-up steps are training steps; record their losses through a wrapper
        def rec():
            loss = step()
            losses.append(loss.detach().clone())
            return loss

        gs = GraphedStep(rec, dev, comm=comm, warmup=warm)
        losses.pop()  # the capture call's (never executed) loss tensor
        for _ in range(steps - warm):
            losses.append(gs().detach().clone())
        assert gs.n_collectives == 0  # world 1: the reducer issues no collective
    else:
        for _ in range(steps):
            losses.append(step().detach().clone())
    torch.cuda.synchronize(dev)
    return [float(v) for v in losses], {k: v.detach().float().cpu() for k, v in model.state_dict().items()}


def test_graphed_resnet_ddp_step_matches_eager(pg, dev):
    from pytorch_distributed_training_tutorials_amd.models.resnet import resnet50

    torch.manual_seed(0)
    init = {k: v.clone() for k, v in resnet50(num_classes=10).state_dict().items()}
    old = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    try:
        la, sa = _run(dev, False, 6, init)
        lb, sb = _run(dev, True, 6, init)
    finally:
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = old
    assert len(la) == len(lb) == 6
    assert all(torch.isfinite(torch.tensor(la)))
    # replays must keep training: the loss moves, and equals the eager trajectory
    assert la[-1] != la[0]
    torch.testing.assert_close(torch.tensor(lb), torch.tensor(la), rtol=2e-3, atol=2e-3)
    for k in sa:
        torch.testing.assert_close(sb[k], sa[k], rtol=2e-3, atol=2e-4, msg=lambda m, k=k: f"{k}: {m}")
