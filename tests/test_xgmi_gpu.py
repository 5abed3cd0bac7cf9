"""xGMI one-shot all-reduce protocol on one GPU (two processes sharing cuda:0 via IPC)."""
import os

import pytest
import torch
import torch.nn.functional as F

from pytorch_distributed_training_tutorials_amd.parallel.env import free_port
from pytorch_distributed_training_tutorials_amd.parallel.launcher import spawn

from . import _workers

pytestmark = pytest.mark.gpu


def test_xgmi_allreduce_and_fused_step_two_ranks(tmp_path):
    world = 2
    spawn(_workers.xgmi_two_procs_one_gpu, args=(world, free_port(), str(tmp_path)), nprocs=world)
    res = [torch.load(os.path.join(tmp_path, f"r{r}.pt"), weights_only=True) for r in range(world)]
    assert all(r["ok"] for r in res)
    assert max(r["max_err"] for r in res) < 1e-6
    # replicas bit-identical (rank-ordered sums)
    assert torch.equal(res[0]["params"], res[1]["params"])
    assert torch.equal(res[0]["grads"], res[1]["grads"])
    # and equal to one process training on the full 16-row batches
    from pytorch_distributed_training_tutorials_amd.models.toy import ToyMLP

    torch.manual_seed(5)
    m = ToyMLP(20, 16, 4)
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9)
    X = torch.randn(64, 20, generator=torch.Generator().manual_seed(9))
    Y = torch.randint(0, 4, (64,), generator=torch.Generator().manual_seed(10))
    for s in range(6):
        sl = slice(16 * (s % 4), 16 * (s % 4) + 16)
        opt.zero_grad()
        F.cross_entropy(m(X[sl]), Y[sl]).backward()
        opt.step()
    ref = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
    torch.testing.assert_close(res[0]["params"], ref, rtol=1e-4, atol=1e-5)


def test_xgmi_single_rank_in_kernel_path(dev):
    """world == 1: the in-kernel all-reduce degenerates to a local copy; results equal the RCCL path."""
    import torch.distributed as dist

    from pytorch_distributed_training_tutorials_amd.models.toy import ToyMLP
    from pytorch_distributed_training_tutorials_amd.ops.fused_step import FusedMLPStep
    from pytorch_distributed_training_tutorials_amd.parallel import env
    from pytorch_distributed_training_tutorials_amd.parallel import comm as comm_mod
    from pytorch_distributed_training_tutorials_amd.parallel.xgmi import XgmiAllReduce

    env.init_process_group("nccl")
    c = comm_mod.get_default(dev)
    xg = XgmiAllReduce(c, dev)
    assert xg.ok
    X = torch.randn(128, 20, device=dev)
    Y = torch.randint(0, 10, (128,), device=dev)
    outs = []
    for use in (False, True):
        torch.manual_seed(3)
        eng = FusedMLPStep(ToyMLP(20, 32, 10).to(dev), loss="ce_index", lr=0.05, momentum=0.9, comm=c,
                           xgmi=xg if use else None)
        for s in range(5):
            idx = torch.arange(32, dtype=torch.int32, device=dev) + 32 * (s % 4)
            eng.step(X, Y, idx, 32)
        eng.flush()
        torch.cuda.synchronize()
        outs.append(eng.P.clone())
    torch.testing.assert_close(outs[0], outs[1], rtol=1e-6, atol=1e-7)
    env.destroy_process_group()


def test_persistent_engine_world1_equals_per_step(dev):
    from pytorch_distributed_training_tutorials_amd.data.device_sampler import DeviceDistributedSampler
    from pytorch_distributed_training_tutorials_amd.models.toy import ToyMLP, ddp_toy_model
    from pytorch_distributed_training_tutorials_amd.ops.fused_step import FusedMLPStep

    from ._workers import _per_step_reference

    for kind in ("mlp", "toy"):
        if kind == "mlp":
            X = torch.randn(500, 20, device=dev)
            Y = torch.randint(0, 10, (500,), device=dev)
            mk, loss, mom = (lambda: ToyMLP(20, 64, 10)), "ce_index", 0.9
        else:
            X = torch.rand(2048, 20, device=dev)
            Y = torch.rand(2048, 1, device=dev)
            mk, loss, mom = (lambda: ddp_toy_model()), "ce_soft", 0.0
        res = []
        for mode in ("persistent", "per_step"):
            torch.manual_seed(7)
            eng = FusedMLPStep(mk().to(dev), loss=loss, lr=0.05, momentum=mom)
            sampler = DeviceDistributedSampler(X.shape[0], 1, 0, seed=1, device=dev)
            if mode == "persistent":
                cursor = torch.zeros(2, dtype=torch.int32, device=dev)
                losses = torch.zeros(40, device=dev)
                # the LDS workgroup body: same summation order as the per-step kernel (bitwise-close)
                eng.run_persistent(X, Y, 150, 32, sampler, cursor, losses, max_steps_per_launch=40,
                                   variant="workgroup" if kind == "mlp" else None)
                torch.cuda.synchronize()
                S = -(-X.shape[0] // 32)
                assert cursor.tolist() == [150 // S, 150 % S]
            else:
                _per_step_reference(eng, X, Y, sampler, 150, 32, dev)
            torch.cuda.synchronize()
            res.append(eng.P.clone())
        torch.testing.assert_close(res[0], res[1], rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("kind,splits", [
    ("linear_mse", (1, 5, 37, 3, 20, 43, 41)), ("mlp_workgroup", (1, 5, 37, 3, 20, 43, 41)),
    ("mlp_mfma", (1, 5, 37, 3, 20, 43, 41)),
    # launches starting 1-3 positions before an epoch end (S = 20): the single-wave engine's
    # early start computes fewer own positions there and takes barrier 0 together with the
    # epoch crossing; 1- and 2-step launches end before the trainer ever reads the LDS list
    ("linear_mse", (19, 1, 18, 3, 17, 4, 2, 1, 1, 84)),
])
def test_persistent_plan_with_list_cache_equals_per_step(dev, kind, splits):
    """PersistentPlan (launch resolved once, epoch lists cached across launches):
    irregular launch splits crossing epoch boundaries (starts mid-epoch on a
    cached list, epochs built by the helper waves) follow the per-step trajectory."""
    from pytorch_distributed_training_tutorials_amd.data.device_sampler import DeviceDistributedSampler
    from pytorch_distributed_training_tutorials_amd.models.toy import ToyMLP, ddp_toy_model
    from pytorch_distributed_training_tutorials_amd.ops.fused_step import FusedMLPStep

    from ._workers import _per_step_reference

    if kind == "linear_mse":
        X, Y = torch.rand(640, 20, device=dev), torch.rand(640, 1, device=dev)
        mk, loss, mom, variant = (lambda: ddp_toy_model()), "mse", 0.9, None
    else:
        X, Y = torch.randn(500, 20, device=dev), torch.randint(0, 10, (500,), device=dev)
        mk, loss, mom = (lambda: ToyMLP(20, 64, 10)), "ce_index", 0.9
        variant = "workgroup" if kind == "mlp_workgroup" else "mfma"
    total = sum(splits)  # 150 steps, epochs of 20 (linear) / 16 (mlp) steps
    res = []
    for mode in ("plan", "per_step"):
        torch.manual_seed(7)
        eng = FusedMLPStep(mk().to(dev), loss=loss, lr=0.05, momentum=mom)
        sampler = DeviceDistributedSampler(X.shape[0], 1, 0, seed=1, device=dev)
        if mode == "plan":
            cursor = torch.zeros(2, dtype=torch.int32, device=dev)
            losses = torch.zeros(max(splits), device=dev)
            plan = eng.persistent_plan(X, Y, 32, sampler, cursor, losses, variant=variant)
            for n in splits:
                plan.launch(n)
            torch.cuda.synchronize()
            S = -(-X.shape[0] // 32)
            assert cursor.tolist() == [total // S, total % S]
        else:
            _per_step_reference(eng, X, Y, sampler, total, 32, dev)
        torch.cuda.synchronize()
        res.append(eng.P.clone())
    assert torch.isfinite(res[0]).all()
    tol = 1e-6 if kind != "mlp_mfma" else 1e-4
    torch.testing.assert_close(res[0], res[1], rtol=tol, atol=tol)


@pytest.mark.parametrize("kind", ["linear_mse", "mlp_tp"])
def test_persistent_plan_launch_at_equals_device_cursor(dev, kind):
    """PersistentPlan.launch_at(n, pos) (start position from the host's step count, no
    cursor load at kernel entry) runs bitwise the same trajectory as launch(n) from the
    device cursor, and leaves the cursor where launch(n) does."""
    from pytorch_distributed_training_tutorials_amd.data.device_sampler import DeviceDistributedSampler
    from pytorch_distributed_training_tutorials_amd.models.toy import ToyMLP, ddp_toy_model
    from pytorch_distributed_training_tutorials_amd.ops.fused_step import FusedMLPStep

    if kind == "linear_mse":
        X, Y = torch.rand(640, 20, device=dev), torch.rand(640, 1, device=dev)
        mk, loss = (lambda: ddp_toy_model()), "mse"
    else:
        X, Y = torch.randn(500, 20, device=dev), torch.randint(0, 10, (500,), device=dev)
        mk, loss = (lambda: ToyMLP(20, 64, 10)), "ce_index"
    splits = [1, 5, 37, 3, 20, 43, 41]
    res, curs, engines = [], [], []
    for mode in ("cursor", "at"):
        torch.manual_seed(7)
        eng = FusedMLPStep(mk().to(dev), loss=loss, lr=0.05, momentum=0.9)
        sampler = DeviceDistributedSampler(X.shape[0], 1, 0, seed=1, device=dev)
        cursor = torch.zeros(2, dtype=torch.int32, device=dev)
        losses = torch.zeros(max(splits), device=dev)
        plan = eng.persistent_plan(X, Y, 32, sampler, cursor, losses)
        pos = 0
        for n in splits:
            plan.launch(n) if mode == "cursor" else plan.launch_at(n, pos)
            pos += n
        torch.cuda.synchronize()
        res.append(eng.P.clone())
        curs.append(cursor.tolist())
        engines.append(eng.persistent_engine(32, sampler))
    assert engines[0].startswith("tp" if kind == "mlp_tp" else "wave"), engines[0]
    assert curs[0] == curs[1]
    assert torch.equal(res[0], res[1])


@pytest.mark.parametrize("kind", ["mlp", "linear", "linear_nopair", "linear_rows"])
def test_persistent_engine_two_ranks_one_gpu(tmp_path, kind):
    world = 2
    spawn(_workers.persistent_two_procs_one_gpu, args=(world, free_port(), str(tmp_path), kind), nprocs=world)
    res = [torch.load(os.path.join(tmp_path, f"r{r}.pt"), weights_only=True) for r in range(world)]
    assert res[0]["engine"].startswith("tp" if kind == "mlp" else "wave")
    assert torch.equal(res[0]["persistent"], res[1]["persistent"])  # replicas in sync
    torch.testing.assert_close(res[0]["persistent"], res[0]["per_step"], rtol=1e-5, atol=1e-5)
    assert res[0]["cursor"].tolist() == [23 // 10, 23 % 10]  # 150 samples/rank / 16 -> 10 steps per epoch


@pytest.mark.parametrize("cfg", [
    # (Din, Dout, loss, momentum, dataset rows, batch): flagship toy, partial last batch + momentum,
    # MSE, CE with ignore_index rows, B=64 (one lane per row), B=8 (8 lanes per row)
    (20, 1, "ce_soft", 0.0, 2048, 32),
    (20, 2, "ce_index", 0.9, 500, 32),
    (13, 1, "mse", 0.9, 300, 32),
    (20, 2, "ce_index_ignore", 0.0, 400, 32),
    (16, 1, "ce_soft", 0.9, 1000, 64),
    (30, 4, "mse", 0.5, 200, 8),
])
def test_wave_engine_matches_workgroup_engine(dev, cfg):
    """The single-wave register engine (linear_wave.hip) against the LDS workgroup
    engine and the per-step kernel on the same sampler stream (fp32, summation
    order differs only)."""
    from pytorch_distributed_training_tutorials_amd.data.device_sampler import DeviceDistributedSampler
    from pytorch_distributed_training_tutorials_amd.ops.fused_step import FusedMLPStep

    from ._workers import _per_step_reference

    Din, Dout, loss, mom, N, B = cfg
    g = torch.Generator().manual_seed(11)
    X = torch.randn(N, Din, generator=g).to(dev)
    kw = {}
    if loss.startswith("ce_index"):
        Y = torch.randint(0, Dout, (N,), generator=g)
        if loss.endswith("ignore"):
            Y[::5] = -100
            kw["ignore_index"] = -100
        Y = Y.to(dev)
        loss = "ce_index"
    else:
        Y = torch.rand(N, Dout, generator=g).to(dev)
    n_steps = 3 * -(-N // B) + 5  # several epoch transitions, mid-epoch stop
    res = {}
    for mode in ("wave_f", "wave_rows", "workgroup", "per_step"):
        torch.manual_seed(7)
        eng = FusedMLPStep(torch.nn.Linear(Din, Dout).to(dev), loss=loss, lr=0.05, momentum=mom, **kw)
        sampler = DeviceDistributedSampler(N, 1, 0, seed=2, device=dev)
        if mode == "per_step":
            _per_step_reference(eng, X, Y, sampler, n_steps, B, dev)
        else:
            eng_name = eng.persistent_engine(B, sampler, mode)
            if mode.startswith("wave") and eng_name == "workgroup":
                continue  # this layout family has no instantiation for the shape
            assert eng_name.startswith("workgroup" if mode == "workgroup" else "wave")
            assert (mode != "wave_f") or eng_name.startswith("wave:L0")
            cursor = torch.zeros(2, dtype=torch.int32, device=dev)
            losses = torch.zeros(n_steps, device=dev)
            # two launches: the second resumes from the cursor mid-epoch
            eng.run_persistent(X, Y, n_steps - 7, B, sampler, cursor, losses, variant=mode)
            eng.run_persistent(X, Y, 7, B, sampler, cursor, losses[n_steps - 7:], variant=mode)
            torch.cuda.synchronize()
            S = -(-N // B)
            assert cursor.tolist() == [n_steps // S, n_steps % S]
            res[mode + "_loss"] = losses.clone()
            res[mode + "_G"] = eng.G.clone()
        torch.cuda.synchronize()
        res[mode] = eng.P.clone()
    waves = [w for w in ("wave_f", "wave_rows") if w in res]
    assert waves
    for w in waves:
        torch.testing.assert_close(res[w], res["workgroup"], rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(res[w], res["per_step"], rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(res[w + "_loss"], res["workgroup_loss"], rtol=1e-4, atol=1e-5, equal_nan=True)
        torch.testing.assert_close(res[w + "_G"], res["workgroup_G"], rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("B,Din,H,Dout,loss", [(32, 20, 64, 10, "ce_index"), (16, 7, 32, 3, "ce_soft"),
                                               (32, 32, 16, 16, "mse"), (24, 20, 48, 1, "ce_soft"),
                                               (32, 20, 64, 10, "ce_soft")])
def test_mfma_mlp_engine_matches_workgroup_engine(dev, B, Din, H, Dout, loss):
    """The 4-wave MFMA step body (toy MLP) vs the LDS dot-product body: same training trajectory
    (fp32 MFMA: only the summation order differs), partial last batches included."""
    from pytorch_distributed_training_tutorials_amd.data.device_sampler import DeviceDistributedSampler
    from pytorch_distributed_training_tutorials_amd.models.toy import ToyMLP
    from pytorch_distributed_training_tutorials_amd.ops.fused_step import FusedMLPStep

    N = 7 * B + 5  # a partial batch at every epoch end
    g = torch.Generator(device=dev).manual_seed(B + Din + H)
    X = torch.randn(N, Din, device=dev, generator=g)
    if loss == "ce_index":
        Y = torch.randint(0, Dout, (N,), device=dev, generator=g)
    elif loss == "ce_soft":
        Y = torch.rand(N, Dout, device=dev, generator=g)
    else:
        Y = torch.randn(N, Dout, device=dev, generator=g)
    out = {}
    for variant in ("mfma", "workgroup"):
        torch.manual_seed(3)
        eng = FusedMLPStep(ToyMLP(Din, H, Dout).to(dev), loss=loss, lr=0.05, momentum=0.9)
        sampler = DeviceDistributedSampler(N, 1, 0, seed=2, device=dev)
        assert eng.persistent_engine(B, sampler, variant) == ("workgroup:mfma" if variant == "mfma" else "workgroup")
        cursor = torch.zeros(2, dtype=torch.int32, device=dev)
        losses = torch.zeros(64, device=dev)
        eng.run_persistent(X, Y, 40, B, sampler, cursor, losses, max_steps_per_launch=64, variant=variant)
        torch.cuda.synchronize()
        out[variant] = (eng.P.clone(), losses[:40].clone())
    torch.testing.assert_close(out["mfma"][1], out["workgroup"][1], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(out["mfma"][0], out["workgroup"][0], rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_wave_engine_pair_exchange_equals_chunked(tmp_path, world):
    """W ranks sharing the GPU: at W = 2 the single-wave engine's packed pair exchange (one store + one
    poll per step) and the chunked per-row-slot exchange (PTDT_XGMI_PAIR=0) train to the same bits
    (x0 + x1 either way); at W = 4 / 8 both runs take the chunked exchange. Replicas in sync and close
    to the per-step reference at every W."""
    got = {}
    for kind in ("linear", "linear_nopair"):
        d = tmp_path / kind
        d.mkdir()
        spawn(_workers.persistent_two_procs_one_gpu, args=(world, free_port(), str(d), kind), nprocs=world)
        res = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(world)]
        assert all(torch.equal(r["persistent"], res[0]["persistent"]) for r in res)
        torch.testing.assert_close(res[0]["persistent"], res[0]["per_step"], rtol=1e-5, atol=1e-5)
        got[kind] = res[0]["persistent"]
    assert torch.equal(got["linear"], got["linear_nopair"])
