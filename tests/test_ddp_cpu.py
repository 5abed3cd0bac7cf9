"""DDP + communicator over gloo with world_size 2 (CPU plumbing)."""
import os

import pytest
import torch
import torch.nn.functional as F

from pytorch_distributed_training_tutorials_amd.parallel.env import free_port
from pytorch_distributed_training_tutorials_amd.parallel.launcher import spawn

from . import _workers

pytestmark = pytest.mark.slow


def _load(d, w):
    return [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(w)]


def test_ddp_matches_single_process_large_batch(tmp_path):
    world = 2
    spawn(_workers.ddp_equivalence, args=(world, free_port(), str(tmp_path), 0.0005), nprocs=world)
    res = _load(tmp_path, world)
    # ranks agree exactly
    for a, b in zip(res[0]["params"], res[1]["params"]):
        torch.testing.assert_close(a, b, rtol=0, atol=0)
    # and equal a single process on the concatenated batch, starting from rank 0's init
    from pytorch_distributed_training_tutorials_amd.models.toy import ToyMLP

    torch.manual_seed(100)
    m = ToyMLP(20, 16, 5)
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9)
    g = torch.Generator().manual_seed(0)
    X = torch.randn(4, 8 * world, 20, generator=g)
    Y = torch.randint(0, 5, (4, 8 * world), generator=g)
    for it in range(4):
        opt.zero_grad()
        F.cross_entropy(m(X[it]), Y[it]).backward()
        opt.step()
    for a, b in zip(res[0]["params"], m.parameters()):
        torch.testing.assert_close(a, b.detach(), rtol=1e-5, atol=1e-6)
    assert len(res[0]["buckets"]) >= 2  # tiny caps -> several buckets (rebuilt after iteration 0)
    assert all(k.startswith("module.") for k in res[0]["keys"])


def test_ddp_no_sync_and_find_unused(tmp_path):
    world = 2
    spawn(_workers.ddp_no_sync_and_unused, args=(world, free_port(), str(tmp_path)), nprocs=world)
    res = _load(tmp_path, world)
    # rank r contributes 3 micro-batches of x=(r+1): d(sum a(x))/dW = 2 rows * x per column
    # rank-local accumulation 3*2*(r+1); the synced step averages the bucket (incl. accumulated grads)
    expect = (3 * 2 * 1 + 3 * 2 * 2) / 2
    torch.testing.assert_close(res[0]["ga"], torch.full((4, 4), expect))
    torch.testing.assert_close(res[1]["ga"], res[0]["ga"])
    assert (res[0]["gu"] == 0).all()


def test_ddp_unused_parameter_error(tmp_path):
    world = 2
    spawn(_workers.ddp_missing_grad_raises, args=(world, free_port(), str(tmp_path)), nprocs=world)
    assert all(r["raised"] for r in _load(tmp_path, world))


@pytest.mark.parametrize("world", [2, 3])
def test_communicator_collectives_gloo(tmp_path, world):
    spawn(_workers.comm_collectives, args=(world, free_port(), str(tmp_path)), nprocs=world)
    res = _load(tmp_path, world)
    tot = sum(range(1, world + 1))
    for r, d in enumerate(res):
        torch.testing.assert_close(d["sum"], torch.full((3,), float(tot)))
        torch.testing.assert_close(d["avg"], torch.full((3,), tot / world))
        torch.testing.assert_close(d["max"], torch.full((3,), float(world)))
        torch.testing.assert_close(d["bcast"], torch.zeros(2))
        torch.testing.assert_close(d["gather"], torch.tensor([v for q in range(world) for v in (q, q * 10.0)]))
        torch.testing.assert_close(d["rs"], torch.tensor([2.0 * r, 2.0 * r + 1]) * world)
        torch.testing.assert_close(d["a2a"], torch.tensor([r + 100.0 * q for q in range(world)]))
        assert d["obj"] == {"r": 0}
    torch.testing.assert_close(res[1]["p2p"], torch.tensor([42.0]))


@pytest.mark.parametrize("diverge", [False, True])
def test_collective_fingerprint_check(tmp_path, diverge):
    spawn(_workers.fingerprint_check, args=(2, free_port(), str(tmp_path), diverge), nprocs=2)
    res = _load(tmp_path, 2)
    if diverge:
        assert not any(r["ok"] for r in res) and "all_reduce.min" in res[0]["msg"]
    else:
        assert all(r["ok"] and r["n"] == 2 for r in res)


@pytest.mark.parametrize("numel", [21, 1 << 18, 1 << 21])  # the toy's 84 B bucket, 1 MiB, 8 MiB
def test_bucket_sized_all_reduce_world4(tmp_path, numel):
    """tiny and bucket-sized messages over 4 ranks (gloo)."""
    world = 4
    spawn(_workers.bucket_all_reduce, args=(world, free_port(), str(tmp_path), numel), nprocs=world)
    res = _load(tmp_path, world)
    expect = sum(range(1, world + 1)) / world
    for r in res:
        assert r["avg_ok"] and r["bcast_ok"]
        assert abs(r["avg0"] - expect) < 1e-6


def test_ddp_wrapper_is_collectable(tmp_path):
    spawn(_workers.ddp_wrapper_collectable, args=(2, free_port(), str(tmp_path)), nprocs=2)
    for r in _load(tmp_path, 2):
        assert r["collected"] and r["grads"]


def test_kernel_choices_agree_across_ranks(tmp_path):
    """Per-shape engine selection (ops/linear.py, ops/convbn.py) is rank 0's on every rank, even when
    the ranks' own timings disagree (ADVICE r3 / VERDICT r3 #7)."""
    world = 2
    spawn(_workers.tuning_agree, args=(world, free_port(), str(tmp_path)), nprocs=world)
    res = _load(tmp_path, world)
    assert res[0]["got"] == res[1]["got"] == ["native", "library", "native"]
    # outside the SPMD scope each rank keeps its own timing (no collective, cannot hang)
    assert res[0]["outside"] == "native" and res[1]["outside"] == "library"
    # a key mismatch inside the scope fails loudly on every rank
    assert all(r["mismatch"] and "different linear shape keys" in r["mismatch"] for r in res)


def test_tuning_scopes_counted_and_gated(tmp_path):
    """ADVICE r5 (both mediums) and VERDICT r5 #8a: two DDP wrappers in one step keep their own scope
    counts; agreement happens inside DDP forwards and backwards only; a shape first decided by rank 0
    alone is agreed again by every rank inside DDP (no rank skips the collective); a grad-enabled
    forward without backward does not make a later rank-0-only inference broadcast alone (no hang)."""
    world = 2
    spawn(_workers.tuning_scopes, args=(world, free_port(), str(tmp_path)), nprocs=world)
    res = _load(tmp_path, world)
    for r in res:
        assert (r["depth_after_fwd"], r["depth_after_a_bwd"], r["depth_after_b_bwd"]) == (2, 1, 0)
        assert (r["depth_stale"], r["depth_end"], r["depth_no_grad"]) == (1, 0, 0)
    shared = {k: v for k, v in res[1]["seen"].items()}
    for k, v in shared.items():  # every decision both ranks took in DDP is rank 0's
        assert res[0]["seen"][k] == v, k
    assert shared["fwd:1:3"] == "native" and shared["bwd:1"] == "library" and shared["bwd:2"] == "library"
    assert res[0]["seen"]["fwd:1:7"] == "native" and "fwd:1:7" not in res[1]["seen"]  # rank 0 alone, local


def test_tuning_table_pins_choice(tmp_path, monkeypatch):
    import json

    from pytorch_distributed_training_tutorials_amd.utils import tuning

    path = tmp_path / "t.json"
    path.write_text(json.dumps({"linear": {"nt,128,1000,2048": "library"}, "convbn": {"401408,64,256,0": "fused"}}))
    monkeypatch.setenv("PTDT_TUNING_TABLE", str(path))
    monkeypatch.setattr(tuning, "_TABLE", None)
    assert tuning.pinned("linear", ("nt", 128, 1000, 2048)) == "library"
    assert tuning.pinned("convbn", (401408, 64, 256, 0)) == "fused"
    assert tuning.pinned("linear", ("nt", 1, 2, 3)) is None
    out = tmp_path / "dump.json"
    tuning.dump(str(out))
    assert json.loads(out.read_text())["linear"]["nt,128,1000,2048"] == "library"


def test_native_resnet_ddp_host_logic_cpu(tmp_path):
    """CPU / gloo dry run of the multi-GPU ResNet DDP case (tests/test_multi_gpu.py): the same worker,
    fp32 -- bucket rebuild and the averaged all-reduce == one process accumulating the micro-batches."""
    from . import _mgpu_workers

    world = 2
    spawn(_mgpu_workers.resnet_ddp, args=(world, free_port(), str(tmp_path), False), nprocs=world)
    res = _load(tmp_path, world)
    assert all(r["in_sync"] for r in res)
    assert all(r["rebuilt"] and r["buckets"] >= 2 for r in res)
    ref = _mgpu_workers.resnet_reference(world, gpu=False)
    torch.testing.assert_close(res[0]["params"], ref, rtol=1e-4, atol=1e-5)
