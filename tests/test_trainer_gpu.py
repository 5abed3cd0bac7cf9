"""Trainer product path on one GPU: torch-identical device sampler orders, one
persistent launch per snapshot interval, engine snapshots/resume, and the
xGMI-failure fallback."""
import os

import pytest
import torch

from pytorch_distributed_training_tutorials_amd.parallel.env import free_port
from pytorch_distributed_training_tutorials_amd.parallel.launcher import spawn

from . import _workers

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [2, 3, 500, 2048, 20000])
def test_device_epoch_indices_match_torch_distributed_sampler(dev, n):
    """torch_perm kernel == torch.utils.data.DistributedSampler, every rank, several
    epochs (20000 rows: the global-scratch variant)."""
    from torch.utils.data.distributed import DistributedSampler as TorchSampler

    from pytorch_distributed_training_tutorials_amd.data import DeviceDataLoader, DeviceTensorDataset, DistributedSampler

    ds = DeviceTensorDataset(torch.zeros(n, 1, device=dev))
    for W in (1, 2, 3, 8):
        for drop_last in (False, True):
            if drop_last and n < W:
                continue
            for rank in sorted({0, W - 1}):
                smp = DistributedSampler(ds, W, rank, seed=7, drop_last=drop_last)
                dl = DeviceDataLoader(ds, batch_size=4, sampler=smp)
                got = dl.device_epoch_indices([0, 1, 5]).cpu()
                for k, e in enumerate((0, 1, 5)):
                    ref = TorchSampler(range(n), num_replicas=W, rank=rank, seed=7, drop_last=drop_last)
                    ref.set_epoch(e)
                    assert got[k].tolist() == list(ref), (n, W, rank, e, drop_last)


def test_device_epoch_indices_no_shuffle_and_plain_loader(dev):
    from pytorch_distributed_training_tutorials_amd.data import DeviceDataLoader, DeviceTensorDataset, DistributedSampler

    ds = DeviceTensorDataset(torch.zeros(37, 1, device=dev))
    dl = DeviceDataLoader(ds, batch_size=4, sampler=DistributedSampler(ds, 4, 3, shuffle=False))
    assert dl.device_epoch_indices([0, 2]).cpu().tolist() == [list(DistributedSampler(ds, 4, 3, shuffle=False))] * 2
    dl = DeviceDataLoader(ds, batch_size=4, shuffle=True, seed=9)
    dl.set_epoch(4)
    assert dl.device_epoch_indices([4])[0].cpu().tolist() == dl.host_indices().tolist()


@pytest.mark.parametrize("engine", ["persistent", "fused"])
def test_trainer_snapshot_resume_is_bitwise(dev, tmp_path, engine):
    """2 epochs + snapshot + resume for 1 == 3 uninterrupted epochs, momentum 0.9
    (momentum buffer and first-step flag travel in torch.optim.SGD layout)."""
    from pytorch_distributed_training_tutorials_amd.data import DeviceDataLoader, DeviceTensorDataset, DistributedSampler
    from pytorch_distributed_training_tutorials_amd.models.toy import ToyMLP
    from pytorch_distributed_training_tutorials_amd.ops.optim import FusedSGD
    from pytorch_distributed_training_tutorials_amd.parallel import env
    from pytorch_distributed_training_tutorials_amd.utils.trainer import Trainer

    env.init_process_group("nccl")
    try:
        ds = DeviceTensorDataset.synthetic_classification(300, 20, 4, device=dev, seed=2)

        def make(snapshot=None, save_every=0):
            torch.manual_seed(4)
            model = ToyMLP(20, 32, 4)
            loader = DeviceDataLoader(ds, batch_size=32, sampler=DistributedSampler(ds, 1, 0, seed=5))
            opt = FusedSGD(model.parameters(), lr=0.05, momentum=0.9)
            return model, Trainer(model, loader, opt, 0, engine=engine, snapshot_path=snapshot,
                                  save_every=save_every, verbose=False)

        m_ref, t_ref = make()
        t_ref.train(3)
        torch.cuda.synchronize()
        ref = torch.cat([p.detach().reshape(-1) for p in m_ref.parameters()])
        snap = str(tmp_path / "snap.pt")
        _, t1 = make(snap, save_every=2)
        t1.train(2)
        st = torch.load(snap, weights_only=True)
        assert st["epoch"] == 1 and all("momentum_buffer" in v for v in st["optimizer"]["state"].values())
        m2, t2 = make(snap, save_every=2)
        assert t2.epochs_run == 2
        t2.train(3)
        torch.cuda.synchronize()
        got = torch.cat([p.detach().reshape(-1) for p in m2.parameters()])
        assert torch.equal(got, ref)
    finally:
        env.destroy_process_group()


def test_trainer_persistent_one_launch_for_all_epochs(dev, capsys):
    """Status lines of every epoch, a single persistent launch (global step count),
    loss per step recorded for all epochs."""
    from pytorch_distributed_training_tutorials_amd.data import DeviceDataLoader, DeviceTensorDataset, DistributedSampler
    from pytorch_distributed_training_tutorials_amd.models.toy import ToyMLP
    from pytorch_distributed_training_tutorials_amd.ops.optim import FusedSGD
    from pytorch_distributed_training_tutorials_amd.parallel import env
    from pytorch_distributed_training_tutorials_amd.utils.trainer import Trainer

    env.init_process_group("nccl")
    try:
        ds = DeviceTensorDataset.synthetic_classification(256, 20, 4, device=dev, seed=2)
        model = ToyMLP(20, 32, 4)
        loader = DeviceDataLoader(ds, batch_size=32, sampler=DistributedSampler(ds, 1, 0))
        t = Trainer(model, loader, FusedSGD(model.parameters(), lr=0.05), 0)
        assert t.engine_name == "persistent"
        t.train(10)
        out = capsys.readouterr().out
        for e in range(10):
            assert f"[GPU: 0 Epoch: {e}, Batch size: 32 | Steps 8]" in out
        assert t.global_step == 80
        losses = t.last_losses()[:80]
        assert torch.isfinite(losses).all() and float(losses[-8:].mean()) < float(losses[:8].mean())
    finally:
        env.destroy_process_group()


@pytest.mark.parametrize("inject", [False, True])
def test_trainer_xgmi_timeout_falls_back_to_rccl_path(tmp_path, inject):
    world = 2
    spawn(_workers.trainer_xgmi_fallback_one_gpu, args=(world, free_port(), str(tmp_path), inject), nprocs=world)
    res = [torch.load(os.path.join(tmp_path, f"r{r}.pt"), weights_only=True) for r in range(world)]
    for r in res:
        assert r["persistent_engine"] == "persistent"
        assert r["persistent_fallbacks"] == (1 if inject else 0)
        assert r["persistent_final_engine"] == ("fused" if inject else "persistent")
    assert torch.equal(res[0]["persistent"], res[1]["persistent"])  # replicas back in sync
    assert torch.equal(res[0]["fused"], res[1]["fused"])
    tol = 1e-6 if inject else 1e-5  # the fallback re-runs on the fused engine itself
    torch.testing.assert_close(res[0]["persistent"], res[0]["fused"], rtol=tol, atol=tol)


def test_trainer_persistent_launch_budget_chunks_epochs(dev, monkeypatch):
    """A device-memory budget for the per-launch epoch lists splits max_epoch into several
    persistent launches; the parameters are bitwise those of one launch."""
    from pytorch_distributed_training_tutorials_amd.data import DeviceDataLoader, DeviceTensorDataset, DistributedSampler
    from pytorch_distributed_training_tutorials_amd.models.toy import ToyMLP
    from pytorch_distributed_training_tutorials_amd.ops.optim import FusedSGD
    from pytorch_distributed_training_tutorials_amd.parallel import env
    from pytorch_distributed_training_tutorials_amd.utils.trainer import Trainer

    env.init_process_group("nccl")
    try:
        out = {}
        for budget in (None, 3 * (4 * 256 + 4 * 8)):  # None: all 10 epochs in one launch; else 3 per launch
            if budget is None:
                monkeypatch.delenv("PTDT_PERSIST_EPOCH_BYTES", raising=False)
            else:
                monkeypatch.setenv("PTDT_PERSIST_EPOCH_BYTES", str(budget))
            ds = DeviceTensorDataset.synthetic_classification(256, 20, 4, device=dev, seed=2)
            torch.manual_seed(0)
            model = ToyMLP(20, 32, 4)
            loader = DeviceDataLoader(ds, batch_size=32, sampler=DistributedSampler(ds, 1, 0))
            t = Trainer(model, loader, FusedSGD(model.parameters(), lr=0.05), 0)
            assert t.engine_name == "persistent"
            assert t._max_epochs_per_launch() == (3 if budget else t._max_epochs_per_launch())
            t.train(10)
            torch.cuda.synchronize()
            assert t.global_step == 80
            out[budget] = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
        a, b = out.values()
        assert torch.equal(a, b)
    finally:
        env.destroy_process_group()
