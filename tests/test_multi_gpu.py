"""Multi-GPU suite: active only when >= 2 GPUs are visible (skips on 1-GPU boxes).

One process per GPU over RCCL/xGMI for the DDP, xGMI and pipeline cases; one
process driving several GPUs for DataParallel (RcclClique broadcast/reduce) and
the in-process model-parallel splits. Each case checks semantic equivalence
with a single-device / single-process run:
  * native DDP at W = 2/4/8 == one process on the W*B batch; replicas bitwise equal
    (ddp_gpus.py:32-39);
  * xGMI one-shot all-reduce across devices == RCCL ncclAvg at 21 / 1994 / 65536
    floats, and the persistent engines (all-reduce inside the kernel) == the
    fused engine + RCCL at W = N;
  * the Trainer on W GPUs: status lines with 2048/(32 W) steps, replicas in sync;
  * DataParallel on up to 4 distinct GPUs: the [8, 32] replica split, grads ==
    single device (01.data_parallel.ipynb:300-308);
  * ToyModel / ModelParallelResNet50 across cuda:0 / cuda:1 == unsplit
    (03.model_parallel.ipynb:515-516);
  * the 2-rank RCCL send/recv PipelineStage == single process.
"""
import os

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from pytorch_distributed_training_tutorials_amd.parallel.env import free_port
from pytorch_distributed_training_tutorials_amd.parallel.launcher import spawn

from . import _mgpu_workers

pytestmark = pytest.mark.gpu

N_GPU = torch.cuda.device_count() if torch.cuda.is_available() else 0


def needs(n):
    return pytest.mark.skipif(N_GPU < n, reason=f"needs {n} GPUs, {N_GPU} visible")


def _ranks(tmp_path, world):
    return [torch.load(os.path.join(tmp_path, f"r{r}.pt"), weights_only=True) for r in range(world)]


@pytest.mark.parametrize("world", [2, 4, 8])
def test_native_ddp_multi_gpu_equals_single_process(tmp_path, world):
    if N_GPU < world:
        pytest.skip(f"needs {world} GPUs, {N_GPU} visible")
    spawn(_mgpu_workers.ddp_gpu, args=(world, free_port(), str(tmp_path)), nprocs=world)
    res = _ranks(tmp_path, world)
    assert all(r["in_sync"] for r in res)
    assert all(torch.equal(r["params"], res[0]["params"]) for r in res)
    assert res[0]["buckets"] >= 2
    from pytorch_distributed_training_tutorials_amd.models.toy import ToyMLP

    torch.manual_seed(100)  # rank 0's init, broadcast by DDP
    m = ToyMLP(20, 16, 5)
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9)
    g = torch.Generator().manual_seed(0)
    X = torch.randn(4, 8 * world, 20, generator=g)
    Y = torch.randint(0, 5, (4, 8 * world), generator=g)
    for it in range(4):
        opt.zero_grad()
        F.cross_entropy(m(X[it]), Y[it]).backward()
        opt.step()
    ref = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
    torch.testing.assert_close(res[0]["params"], ref, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("world", [2, 8])
def test_xgmi_allreduce_and_persistent_engines_across_gpus(tmp_path, world):
    if N_GPU < world:
        pytest.skip(f"needs {world} GPUs, {N_GPU} visible")
    spawn(_mgpu_workers.xgmi_gpu, args=(world, free_port(), str(tmp_path)), nprocs=world)
    res = _ranks(tmp_path, world)
    assert all(r["ok"] for r in res), "xGMI self-test failed across devices"
    for r in res:
        assert r["poll_error"] == 0
        for n, e in r["max_err"].items():
            assert e < 1e-5, (n, e)
            assert r[f"xgmi_in_sync_{n}"]
        assert r["linear_engine"].startswith("wave")
        for kind in ("linear", "mlp"):
            assert r[f"{kind}_persistent_in_sync"] and r[f"{kind}_per_step_rccl_in_sync"]
            assert r[f"{kind}_err"] < 1e-4, (kind, r[f"{kind}_err"])


@pytest.mark.parametrize("world", [2, 8])
def test_trainer_multi_gpu_ddp_toy_job(tmp_path, world):
    if N_GPU < world:
        pytest.skip(f"needs {world} GPUs, {N_GPU} visible")
    spawn(_mgpu_workers.trainer_gpu, args=(world, free_port(), str(tmp_path)), nprocs=world)
    res = _ranks(tmp_path, world)
    steps = 2048 // (32 * world)
    for rank, r in enumerate(res):
        for engine in ("auto", "fused"):
            o = r[engine]
            assert o["in_sync"] and o["fallbacks"] == 0
            for e in range(3):
                assert f"[GPU: {rank} Epoch: {e}, Batch size: 32 | Steps {steps}]" in o["lines"]
        assert r["auto"]["engine"] in ("persistent", "fused")
    torch.testing.assert_close(res[0]["auto"]["params"], res[0]["fused"]["params"], rtol=1e-4, atol=1e-5)


@needs(2)
@pytest.mark.parametrize("micro,batches", [(1, (20, 20, 20)), (4, (20, 20, 20)), (1, (20, 8, 20)),
                                           (4, (18, 6, 18))])
def test_two_gpu_pipeline_send_recv_matches_single_process(tmp_path, micro, batches):
    from ._workers import pipeline_reference_stages

    spawn(_mgpu_workers.pipeline_gpu, args=(2, free_port(), str(tmp_path), micro, batches), nprocs=2)
    r0, r1 = _ranks(tmp_path, 2)
    model = nn.Sequential(*pipeline_reference_stages(2))
    opt = torch.optim.SGD(model.parameters(), lr=1e-3)
    g = torch.Generator().manual_seed(1)
    losses = []
    for b in batches:
        x = torch.randn(b, 1000, generator=g)
        y = torch.randn(b, 5, generator=g)
        opt.zero_grad()
        l = nn.MSELoss()(model(x), y)
        l.backward()
        opt.step()
        losses.append(float(l))
    for r, stage in ((r0, model[0]), (r1, model[1])):
        for a, b in zip(r["params"], list(stage.parameters())):
            torch.testing.assert_close(a, b.detach(), rtol=1e-4, atol=1e-5)
    assert r1["losses"] == pytest.approx(losses, rel=1e-4)


@needs(2)
def test_data_parallel_distinct_gpus_rccl_clique(capsys):
    from pytorch_distributed_training_tutorials_amd.models.toy import SampleModel
    from pytorch_distributed_training_tutorials_amd.parallel.dp import DataParallel, _Clique

    k = min(4, N_GPU)
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = SampleModel(32, 2).to(dev)
    ref = SampleModel(32, 2, verbose=False).to(dev)
    ref.load_state_dict(model.state_dict())
    dp = DataParallel(model, device_ids=list(range(k)))
    assert _Clique.get(dp.devices) is not None  # distinct GPUs: RCCL broadcast/reduce, not copies
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    opt_ref = torch.optim.Adam(ref.parameters(), lr=1e-3)
    x = torch.randn(32, 32, device=dev)
    for _ in range(3):
        opt.zero_grad()
        out = dp(x)
        out.sum().backward()
        opt.step()
        opt_ref.zero_grad()
        ref(x).sum().backward()
        opt_ref.step()
    printed = capsys.readouterr().out
    assert printed.count(f"Input shape: torch.Size([{32 // k}, 32])") == 3 * k  # NB01:300-308 split
    assert out.shape == (32, 2) and out.device == dev
    for p, q in zip(model.parameters(), ref.parameters()):
        torch.testing.assert_close(p.detach(), q.detach(), rtol=1e-5, atol=1e-6)


@needs(2)
def test_toy_model_parallel_two_gpus_matches_unsplit():
    from pytorch_distributed_training_tutorials_amd.models.toy import ToyModel

    torch.manual_seed(1)
    mp = ToyModel(dev0="cuda:0", dev1="cuda:1")
    assert mp.net1.weight.device == torch.device("cuda", 0) and mp.net2.weight.device == torch.device("cuda", 1)
    x = torch.randn(20, 10000)
    y = torch.randn(20, 5)
    ps = [t.detach().cpu().clone().requires_grad_(True) for t in
          (mp.net1.weight, mp.net1.bias, mp.net2.weight, mp.net2.bias)]
    opt = torch.optim.SGD(mp.parameters(), lr=1e-3)
    opt.zero_grad()
    out = mp(x)
    assert out.device == torch.device("cuda", 1)
    loss = F.mse_loss(out, y.to("cuda:1"))
    loss.backward()
    opt.step()
    ref_loss = F.mse_loss(F.linear(F.relu(F.linear(x, ps[0], ps[1])), ps[2], ps[3]), y)
    ref_loss.backward()
    torch.testing.assert_close(loss.cpu(), ref_loss.detach(), rtol=1e-4, atol=1e-5)
    for p, r in zip((mp.net1.weight, mp.net1.bias, mp.net2.weight, mp.net2.bias), ps):
        torch.testing.assert_close(p.detach().cpu(), r.detach() - 1e-3 * r.grad, rtol=1e-4, atol=1e-6)


@needs(2)
def test_mp_resnet50_two_gpus_train_step_matches_single_gpu():
    from pytorch_distributed_training_tutorials_amd.models.mp_resnet import ModelParallelResNet50
    from pytorch_distributed_training_tutorials_amd.models.resnet import resnet50

    torch.manual_seed(2)
    ref = resnet50(num_classes=1000).to("cuda:0")
    mp = ModelParallelResNet50(num_classes=1000, dev0="cuda:0", dev1="cuda:1")
    mp.load_state_dict(ref.state_dict(), strict=False)
    assert mp.seq1[0].weight.device.index == 0 and mp.fc.weight.device.index == 1
    x = torch.randn(8, 3, 64, 64, device="cuda:0")
    y = torch.zeros(8, 1000).scatter_(1, torch.randint(0, 1000, (8, 1)), 1.0)
    losses = []
    for m, dev_out in ((ref, "cuda:0"), (mp, "cuda:1")):
        m.train()
        opt = torch.optim.SGD(m.parameters(), lr=1e-3)
        opt.zero_grad()
        out = m(x)
        assert out.device == torch.device(dev_out)
        loss = F.mse_loss(out, y.to(dev_out))
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert losses[0] == pytest.approx(losses[1], rel=1e-4)
    torch.testing.assert_close(mp.fc.weight.detach().cpu(), ref.fc.weight.detach().cpu(), rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(mp.conv1.weight.detach().cpu(), ref.conv1.weight.detach().cpu(), rtol=1e-4,
                               atol=1e-6)


@needs(2)
def test_stream_pipeline_two_gpus_matches_single_queue_pipeline():
    """Stage streams across cuda:0/cuda:1 (stage 0 of micro-batch i+1 overlapping stage 1
    of micro-batch i, backward on the forward's streams) compute the same training step
    as the reference's single-queue pipeline schedule."""
    from pytorch_distributed_training_tutorials_amd.models.mp_resnet import PipelineParallelResNet50

    torch.backends.cudnn.deterministic = True  # MIOpen's default wgrad solvers vary run to run (~9 %)
    torch.manual_seed(3)
    a = PipelineParallelResNet50(split_size=4, num_classes=10, dev0="cuda:0", dev1="cuda:1", streams=True)
    b = PipelineParallelResNet50(split_size=4, num_classes=10, dev0="cuda:0", dev1="cuda:1", streams=False)
    b.load_state_dict(a.state_dict())
    x = torch.randn(12, 3, 64, 64, device="cuda:0")
    outs = []
    for m in (a, b):
        m.train()
        y = m(x)
        y.square().mean().backward()
        torch.cuda.synchronize("cuda:0")
        torch.cuda.synchronize("cuda:1")
        outs.append((y.detach().cpu(), [p.grad.detach().cpu() for p in m.parameters()]))
    torch.backends.cudnn.deterministic = False
    torch.testing.assert_close(outs[0][0], outs[1][0], rtol=1e-5, atol=1e-6)
    worst = max(((ga - gb).abs().max() / (gb.abs().max() + 1e-30)).item() for ga, gb in zip(outs[0][1], outs[1][1]))
    assert worst <= 1e-5, worst


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_native_resnet_ddp_multi_gpu_equals_accumulated_single_process(tmp_path, world):
    """Native ResNet DDP at world > 1 -- grad sinks, deferred bf16 casts, bucket rebuild (VERDICT r4 #6a):
    replicas bitwise equal, parameters == one process accumulating the ranks' micro-batches. World 1
    runs the same worker on a one-GPU box (the GPU-only paths without the all-reduce)."""
    if N_GPU < world:
        pytest.skip(f"needs {world} GPUs, {N_GPU} visible")
    spawn(_mgpu_workers.resnet_ddp, args=(world, free_port(), str(tmp_path), True), nprocs=world)
    res = _ranks(tmp_path, world)
    assert all(r["in_sync"] for r in res)
    if world > 1:  # (a one-rank reducer issues no all-reduce and keeps its first bucketing)
        assert all(r["rebuilt"] and r["buckets"] >= 2 for r in res)
    assert res[0]["sinks"] > 0 and res[0]["deferred"]
    # reference: the same native bf16 path in ONE process, accumulating the ranks' micro-batches
    # under no_sync (BatchNorm sees the same rows as on each rank); the CPU dry run of this case
    # (tests/test_ddp_cpu.py) checks the host logic against a plain fp32 torch loop instead
    spawn(_mgpu_workers.resnet_ddp, args=(1, free_port(), str(tmp_path), True, world, True), nprocs=1)
    ref = torch.load(os.path.join(tmp_path, "ref.pt"), weights_only=True)
    torch.testing.assert_close(res[0]["params"], ref["params"], rtol=2e-2, atol=5e-3)


@pytest.mark.parametrize("world", [1, 2, 4])
def test_graphed_step_with_rccl_collectives_multi_gpu(tmp_path, world):
    """GraphedStep with the DDP all-reduces captured at world > 1 (VERDICT r4 #6b): replay == eager."""
    if N_GPU < world:
        pytest.skip(f"needs {world} GPUs, {N_GPU} visible")
    spawn(_mgpu_workers.graphed_ddp_gpu, args=(world, free_port(), str(tmp_path)), nprocs=world)
    res = _ranks(tmp_path, world)
    assert all(r["in_sync"] for r in res)
    assert all(r["n_collectives"] >= (1 if world > 1 else 0) for r in res)
    for r in res:
        torch.testing.assert_close(torch.tensor(r["replay_losses"]), torch.tensor(r["eager_losses"]),
                                   rtol=1e-5, atol=1e-6)
        assert r["max_gap"] < 1e-5


@pytest.mark.parametrize("world", [2, 8])
def test_xgmi_self_test_and_peer_matrix(tmp_path, world):
    """The one-shot xGMI path's self-test across devices, with the peer-access matrix printed
    (VERDICT r4 #6c): on an xGMI-connected node every pair must have direct access."""
    if N_GPU < world:
        pytest.skip(f"needs {world} GPUs, {N_GPU} visible")
    spawn(_mgpu_workers.xgmi_peer_matrix, args=(world, free_port(), str(tmp_path)), nprocs=world)
    res = _ranks(tmp_path, world)
    print("peer-access matrix:", res[0]["matrix"], "xGMI ok:", [r["ok"] for r in res], res[0]["why"])
    assert all(all(row[:world]) for row in res[0]["matrix"][:world])
    assert all(r["ok"] for r in res), res[0]["why"]
