"""Native communicator, reducer, fused engine and hipGraph replay on one GPU."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pg():
    from pytorch_distributed_training_tutorials_amd.parallel import env

    env.init_process_group("nccl")
    yield
    env.destroy_process_group()


def test_rccl_single_rank_collectives(pg, dev):
    from pytorch_distributed_training_tutorials_amd.parallel import comm as comm_mod

    c = comm_mod.get_default(dev)
    assert c.native and c.world == 1
    t = torch.arange(10, dtype=torch.float32, device=dev)
    c.all_reduce(t, "sum")
    torch.testing.assert_close(t, torch.arange(10, dtype=torch.float32, device=dev))
    c.all_reduce(t, "avg")
    c.broadcast(t, 0)
    out = torch.empty(10, device=dev)
    c.all_gather(out, t)
    torch.testing.assert_close(out, t)
    c.barrier()
    assert c.handle.seq >= 4


def test_native_ddp_single_rank_grads_are_bucket_views(pg, dev):
    from pytorch_distributed_training_tutorials_amd.models.toy import ToyMLP
    from pytorch_distributed_training_tutorials_amd.ops.loss import cross_entropy
    from pytorch_distributed_training_tutorials_amd.parallel.ddp import DistributedDataParallel

    torch.manual_seed(0)
    m = ToyMLP(20, 64, 10).to(dev)
    ref = ToyMLP(20, 64, 10).to(dev)
    ref.load_state_dict(m.state_dict())
    ddp = DistributedDataParallel(m, device_ids=[0], bucket_cap_mb=0.001, first_bucket_mb=0.0001)
    assert len(ddp.bucket_sizes_bytes()) >= 2
    x = torch.randn(32, 20, device=dev)
    y = torch.randint(0, 10, (32,), device=dev)
    for _ in range(3):  # includes the post-iteration-0 rebuild path
        ddp.zero_grad()
        cross_entropy(ddp(x), y).backward()
    ref.zero_grad()
    F.cross_entropy(ref(x), y).backward()
    for p, q in zip(m.parameters(), ref.parameters()):
        torch.testing.assert_close(p.grad, q.grad, rtol=1e-4, atol=1e-5)
    flat_ptrs = {t.data_ptr(): t.numel() * t.element_size() for t in ddp.reducer.bucket_tensors()}
    for p in m.parameters():
        assert any(b <= p.grad.data_ptr() < b + n for b, n in flat_ptrs.items())
    assert list(ddp.state_dict().keys())[0].startswith("module.")


def test_fused_engine_graph_equals_eager(pg, dev):
    from pytorch_distributed_training_tutorials_amd.data.device_sampler import DeviceDistributedSampler
    from pytorch_distributed_training_tutorials_amd.models.toy import ToyMLP
    from pytorch_distributed_training_tutorials_amd.ops.fused_step import FusedMLPStep
    from pytorch_distributed_training_tutorials_amd.parallel import comm as comm_mod

    c = comm_mod.get_default(dev)
    torch.manual_seed(0)
    X = torch.randn(256, 20, device=dev)
    Y = torch.randint(0, 10, (256,), device=dev)
    results = []
    for use_graph in (False, True):
        torch.manual_seed(1)
        model = ToyMLP(20, 32, 10).to(dev)
        eng = FusedMLPStep(model, loss="ce_index", lr=0.05, momentum=0.9, comm=c)
        s = DeviceDistributedSampler(256, 1, 0, seed=3, device=dev)
        idx = torch.zeros(256, dtype=torch.int32, device=dev)
        batches = [(i * 32, 32) for i in range(8)]

        def fn():
            s.generate(idx)
            eng.run(X, Y, idx, batches)

        s.set_epoch(0)
        if use_graph:
            g = eng.graph(fn, extra_state=(s._epoch,))
            for _ in range(3):
                g.replay()
        else:
            for _ in range(3):
                fn()
        torch.cuda.synchronize()
        assert s.current_epoch() == 2
        results.append(eng.P.clone())
    torch.testing.assert_close(results[0], results[1], rtol=0, atol=0)


def test_trainer_fused_engine_prints_reference_lines(pg, dev, capsys):
    from pytorch_distributed_training_tutorials_amd.data import DeviceDataLoader, DeviceTensorDataset, DistributedSampler
    from pytorch_distributed_training_tutorials_amd.models.toy import ddp_toy_model
    from pytorch_distributed_training_tutorials_amd.ops.optim import FusedSGD
    from pytorch_distributed_training_tutorials_amd.utils.trainer import Trainer

    ds = DeviceTensorDataset.synthetic_regression(2048, device=dev)
    loader = DeviceDataLoader(ds, batch_size=32, sampler=DistributedSampler(ds, 1, 0))
    model = ddp_toy_model()
    t = Trainer(model, loader, FusedSGD(model.parameters(), lr=1e-2), 0)
    assert t.engine_name == "persistent"  # one launch per epoch
    t.train(2)
    out = capsys.readouterr().out
    assert "[GPU: 0 Epoch: 0, Batch size: 32 | Steps 64]" in out
    assert "[GPU: 0 Epoch: 1, Batch size: 32 | Steps 64]" in out
    assert float(t.last_losses().abs().max()) == 0.0  # quirk Q1: zero loss
    assert list(t.model.state_dict()) == ["module.weight", "module.bias"]


@pytest.mark.parametrize("model_kind", ["linear", "mlp"])
def test_trainer_persistent_engine_equals_fused_engine(pg, dev, model_kind):
    """The per-epoch persistent launch (fed the loader's torch-identical sampler order)
    reaches the same parameters as the per-step fused kernel over the same batches."""
    from pytorch_distributed_training_tutorials_amd.data import DeviceDataLoader, DeviceTensorDataset, DistributedSampler
    from pytorch_distributed_training_tutorials_amd.models.toy import ToyMLP
    from pytorch_distributed_training_tutorials_amd.ops.optim import FusedSGD
    from pytorch_distributed_training_tutorials_amd.utils.trainer import Trainer

    torch.manual_seed(3)
    ds = DeviceTensorDataset.synthetic_classification(500, 20, 4, device=dev)  # 16 steps, last one short
    params = []
    for engine in ("persistent", "fused"):
        torch.manual_seed(4)
        model = torch.nn.Linear(20, 4) if model_kind == "linear" else ToyMLP(20, 32, 4)
        loader = DeviceDataLoader(ds, batch_size=32, sampler=DistributedSampler(ds, 1, 0, shuffle=True, seed=5))
        t = Trainer(model, loader, FusedSGD(model.parameters(), lr=0.05, momentum=0.9), 0, engine=engine,
                    verbose=False)
        assert t.engine_name == engine
        t.train(3)
        torch.cuda.synchronize()
        params.append(torch.cat([p.detach().reshape(-1) for p in model.parameters()]))
    torch.testing.assert_close(params[0], params[1], rtol=1e-5, atol=1e-6)


def test_trainer_autograd_engine_mlp_learns(pg, dev):
    from pytorch_distributed_training_tutorials_amd.data import DeviceDataLoader, DeviceTensorDataset, DistributedSampler
    from pytorch_distributed_training_tutorials_amd.models.toy import ToyMLP
    from pytorch_distributed_training_tutorials_amd.ops.loss import cross_entropy
    from pytorch_distributed_training_tutorials_amd.ops.optim import FusedSGD
    from pytorch_distributed_training_tutorials_amd.utils.trainer import Trainer

    torch.manual_seed(0)
    ds = DeviceTensorDataset.synthetic_classification(512, 20, 4, device=dev)
    loader = DeviceDataLoader(ds, batch_size=32, sampler=DistributedSampler(ds, 1, 0))
    model = ToyMLP(20, 64, 4)
    t = Trainer(model, loader, FusedSGD(model.parameters(), lr=0.1), 0, engine="autograd", verbose=False)
    x, y = ds.tensors
    l0 = float(cross_entropy(model.to(dev)(x), y))
    t.train(5)
    l1 = float(cross_entropy(model(x), y))
    assert l1 < l0


def test_ddp_channels_last_grads_keep_param_layout(pg, dev):
    """Native DDP reducer: bucket views of channels_last weights use the parameter's
    strides (no layout-contract copies) and FusedSGD steps them in place."""
    from pytorch_distributed_training_tutorials_amd.ops.optim import FusedSGD
    from pytorch_distributed_training_tutorials_amd.parallel import comm as comm_mod
    from pytorch_distributed_training_tutorials_amd.parallel.ddp import DistributedDataParallel

    torch.manual_seed(1)
    model = torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3), torch.nn.ReLU(), torch.nn.Conv2d(8, 4, 3))
    model = model.to(dev).to(memory_format=torch.channels_last)
    ddp = DistributedDataParallel(model, device_ids=[dev.index], comm=comm_mod.get_default(dev))
    opt = FusedSGD(model.parameters(), lr=0.1, momentum=0.9)
    x = torch.randn(2, 3, 12, 12, device=dev).to(memory_format=torch.channels_last)
    ddp.zero_grad()
    ddp(x).sum().backward()
    w = model[0].weight
    assert w.grad.stride() == w.stride()
    before = w.detach().clone()
    opt.step()
    torch.testing.assert_close(w.detach(), before - 0.1 * w.grad, rtol=1e-6, atol=1e-7)


def test_rccl_watchdog_event_pool_recycles(pg, dev):
    """Eager collectives under the watchdog reuse completion events (no create/destroy per call)."""
    import time

    from pytorch_distributed_training_tutorials_amd.parallel import comm as comm_mod

    c = comm_mod.new_communicator(dev, name="evpool")  # watchdog on (PTDT_COMM_TIMEOUT, 600 s)
    t = torch.ones(1024, device=dev)
    for r in range(30):
        for _ in range(10):
            c.all_reduce(t, "sum")
        torch.cuda.synchronize()
        time.sleep(0.12 if r % 10 == 9 else 0.0)  # let the watchdog drain and recycle
    time.sleep(0.3)
    h = c.handle
    assert h.seq == 300
    assert h.events_created <= 120, h.events_created  # bounded by what was in flight, not by 300 calls
    assert h.event_pool_size == h.events_created  # all completed and returned to the pool
    torch.testing.assert_close(t, torch.ones(1024, device=dev))


def test_graph_captured_collectives_complete_on_device_counter(pg, dev):
    import time

    from pytorch_distributed_training_tutorials_amd.parallel import comm as comm_mod

    C = comm_mod.native()
    rc = C.RcclComm(0, 1, C.RcclComm.new_unique_id(), dev.index or 0, 1.0, False)
    t = torch.arange(64, dtype=torch.float32, device=dev)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        for _ in range(3):
            rc.all_reduce(t, 0, s.cuda_stream)  # warm-up outside capture
    torch.cuda.synchronize()
    before = rc.captured
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
        for _ in range(3):
            t.mul_(1.0)
            rc.all_reduce(t, 0, s.cuda_stream)
    k = rc.captured - before
    assert k == 3
    for _ in range(4):
        g.replay()
        rc.expect_captured(k)
    torch.cuda.synchronize()
    assert rc.completed_captured == 12
    time.sleep(1.3)  # past the timeout: every expectation was met, so no abort
    assert not rc.aborted, rc.error()
    rc.expect_captured(1)  # a completion that never comes: the watchdog aborts
    deadline = time.time() + 5
    while not rc.aborted and time.time() < deadline:
        time.sleep(0.1)
    assert rc.aborted and "graph-captured" in rc.error()
    torch.testing.assert_close(t, torch.arange(64, dtype=torch.float32, device=dev))


def test_force_collective_issues_bucket_allreduce_at_world_1(pg, dev, monkeypatch):
    from pytorch_distributed_training_tutorials_amd.models.toy import ToyMLP
    from pytorch_distributed_training_tutorials_amd.ops.loss import cross_entropy
    from pytorch_distributed_training_tutorials_amd.parallel.ddp import DistributedDataParallel

    x = torch.randn(32, 20, device=dev)
    y = torch.randint(0, 10, (32,), device=dev)
    grads = []
    for force in ("0", "1"):
        monkeypatch.setenv("PTDT_FORCE_COLLECTIVE", force)
        torch.manual_seed(0)
        ddp = DistributedDataParallel(ToyMLP(20, 64, 10).to(dev), device_ids=[0], bucket_cap_mb=0.001,
                                      first_bucket_mb=0.0001)
        nb = len(ddp.bucket_sizes_bytes())
        s0 = ddp.comm.handle.seq
        ddp.zero_grad()
        cross_entropy(ddp(x), y).backward()
        torch.cuda.synchronize()
        issued = ddp.comm.handle.seq - s0
        assert issued == (nb if force == "1" else 0), (force, issued, nb)
        grads.append(torch.cat([p.grad.reshape(-1) for p in ddp.module.parameters()]))
    torch.testing.assert_close(grads[0], grads[1], rtol=0, atol=0)


def test_rccl_clique_single_device_collectives(dev):
    """The single-process DataParallel transport (ncclCommInitAll clique, grouped
    broadcast/reduce/all-reduce) on a one-GPU clique: the same calls DataParallel makes
    over distinct GPUs (tests/test_multi_gpu.py covers 2-8 devices)."""
    from pytorch_distributed_training_tutorials_amd._ext import native

    cl = native().RcclClique([dev.index or 0])
    assert cl.size == 1
    t = torch.arange(1000, dtype=torch.float32, device=dev)
    want = t.clone()
    cl.broadcast([t], 0)
    cl.reduce([t], 0)
    cl.all_reduce([t])
    torch.cuda.synchronize()
    torch.testing.assert_close(t, want)
