"""Multi-process worker bodies for CPU/gloo tests (spawned; must be importable)."""
import os

import torch
import torch.nn.functional as F


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    from pytorch_distributed_training_tutorials_amd.parallel import env

    env.ddp_setup(rank, world, master_addr="127.0.0.1", master_port=port, backend="gloo")


def ddp_equivalence(rank, world, port, out_dir, bucket_mb):
    """DDP on W ranks with per-rank batch B == single process on batch W*B."""
    _init(rank, world, port)
    from pytorch_distributed_training_tutorials_amd.models.toy import ToyMLP
    from pytorch_distributed_training_tutorials_amd.ops.optim import FusedSGD
    from pytorch_distributed_training_tutorials_amd.parallel.ddp import DistributedDataParallel
    from pytorch_distributed_training_tutorials_amd.parallel.env import destroy_process_group

    torch.manual_seed(100 + rank)  # different init per rank: DDP must broadcast rank 0's
    model = ToyMLP(20, 16, 5)
    ddp = DistributedDataParallel(model, bucket_cap_mb=0.0005, first_bucket_mb=0.0001)
    opt = FusedSGD(model.parameters(), lr=0.1, momentum=0.9)
    g = torch.Generator().manual_seed(0)
    X = torch.randn(4, 8 * world, 20, generator=g)
    Y = torch.randint(0, 5, (4, 8 * world), generator=g)
    for it in range(4):
        xs = X[it, rank * 8:(rank + 1) * 8]
        ys = Y[it, rank * 8:(rank + 1) * 8]
        ddp.zero_grad()
        F.cross_entropy(ddp(xs), ys).backward()
        opt.step()
    torch.save({"params": [p.detach() for p in model.parameters()], "buckets": ddp.bucket_params(),
                "keys": list(ddp.state_dict().keys())}, os.path.join(out_dir, f"r{rank}.pt"))
    destroy_process_group()


def ddp_no_sync_and_unused(rank, world, port, out_dir):
    _init(rank, world, port)
    import torch.nn as nn

    from pytorch_distributed_training_tutorials_amd.parallel.ddp import DistributedDataParallel
    from pytorch_distributed_training_tutorials_amd.parallel.env import destroy_process_group

    torch.manual_seed(0)

    class Two(nn.Module):
        def __init__(self):
            super().__init__()
            self.a = nn.Linear(4, 4)
            self.unused = nn.Linear(4, 4)

        def forward(self, x):
            return self.a(x)

    m = Two()
    ddp = DistributedDataParallel(m, find_unused_parameters=True)
    x = torch.full((2, 4), float(rank + 1))
    # accumulate 2 micro-batches locally, sync on the 3rd
    with ddp.no_sync():
        ddp(x).sum().backward()
        ddp(x).sum().backward()
    ddp(x).sum().backward()
    torch.save({"ga": m.a.weight.grad.clone(), "gu": m.unused.weight.grad.clone()},
               os.path.join(out_dir, f"r{rank}.pt"))
    destroy_process_group()


def ddp_missing_grad_raises(rank, world, port, out_dir):
    _init(rank, world, port)
    import torch.nn as nn

    from pytorch_distributed_training_tutorials_amd.parallel.ddp import DistributedDataParallel
    from pytorch_distributed_training_tutorials_amd.parallel.env import destroy_process_group

    m = nn.ModuleDict({"a": nn.Linear(3, 3), "b": nn.Linear(3, 3)})

    class W(nn.Module):
        def __init__(self):
            super().__init__()
            self.m = m

        def forward(self, x):
            return self.m["a"](x)

    ddp = DistributedDataParallel(W())
    try:
        ddp(torch.ones(1, 3)).sum().backward()
        ok = False
    except RuntimeError as e:
        ok = "find_unused_parameters" in str(e)
    torch.save({"raised": ok}, os.path.join(out_dir, f"r{rank}.pt"))
    destroy_process_group()


def comm_collectives(rank, world, port, out_dir):
    _init(rank, world, port)
    from pytorch_distributed_training_tutorials_amd.parallel import comm as comm_mod
    from pytorch_distributed_training_tutorials_amd.parallel.env import destroy_process_group

    c = comm_mod.get_default()
    res = {}
    t = torch.tensor([float(rank + 1)] * 3)
    res["sum"] = c.all_reduce(t.clone(), "sum")
    res["avg"] = c.all_reduce(t.clone(), "avg")
    res["max"] = c.all_reduce(t.clone(), "max")
    b = torch.tensor([float(rank)] * 2)
    res["bcast"] = c.broadcast(b, 0)
    out = torch.empty(2 * world)
    res["gather"] = c.all_gather(out, torch.tensor([float(rank), float(rank * 10)]))
    rs_out = torch.empty(2)
    res["rs"] = c.reduce_scatter(rs_out, torch.arange(2 * world, dtype=torch.float32), "sum")
    a2a = torch.empty(world)
    res["a2a"] = c.all_to_all(a2a, torch.arange(world, dtype=torch.float32) + 100 * rank)
    if world >= 2:
        if rank == 0:
            c.send(torch.tensor([42.0]), 1)
        elif rank == 1:
            res["p2p"] = c.recv(torch.zeros(1), 0)
    res["obj"] = c.broadcast_object({"r": rank}, 0)
    c.barrier()
    torch.save(res, os.path.join(out_dir, f"r{rank}.pt"))
    destroy_process_group()


def xgmi_two_procs_one_gpu(rank, world, port, out_dir):
    """Two ranks share cuda:0: exercises the xGMI LL protocol (IPC buffers, parities,
    rank-ordered sums, in-kernel all-reduce + SGD) without a second GPU."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from pytorch_distributed_training_tutorials_amd.models.toy import ToyMLP
    from pytorch_distributed_training_tutorials_amd.ops.fused_step import FusedMLPStep
    from pytorch_distributed_training_tutorials_amd.parallel.comm import Communicator
    from pytorch_distributed_training_tutorials_amd.parallel.xgmi import XgmiAllReduce

    dev = torch.device("cuda", 0)
    ctl = Communicator(device=torch.device("cpu"))
    xg = XgmiAllReduce(ctl, dev, max_elems=4096)
    res = {"ok": xg.ok}
    g = torch.Generator().manual_seed(1234)
    errs = []
    for it in range(40):
        n = [1, 21, 777, 4096][it % 4]
        vals = [torch.randn(n, generator=g) for _ in range(world)]
        t = vals[rank].to(dev)
        xg.all_reduce_avg(t)
        torch.cuda.synchronize()
        want = vals[0].clone()
        for v in vals[1:]:
            want += v
        want /= world
        errs.append(float((t.cpu() - want).abs().max()))
    res["max_err"] = max(errs)
    # fused DDP step with the in-kernel all-reduce: rank r trains on its half of each batch
    torch.manual_seed(5)
    model = ToyMLP(20, 16, 4).to(dev)
    eng = FusedMLPStep(model, loss="ce_index", lr=0.1, momentum=0.9, xgmi=xg)
    X = torch.randn(64, 20, generator=torch.Generator().manual_seed(9)).to(dev)
    Y = torch.randint(0, 4, (64,), generator=torch.Generator().manual_seed(10)).to(dev)
    for s in range(6):
        idx = (torch.arange(8, dtype=torch.int32) + 16 * (s % 4) + 8 * rank).to(dev)
        eng.step(X, Y, idx, 8)
    torch.cuda.synchronize()
    xg.check()
    res["params"] = eng.P.cpu()
    res["grads"] = eng.G.cpu()
    torch.save(res, os.path.join(out_dir, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def pipeline_two_stage(rank, world, port, out_dir, micro, batches=(20, 20, 20)):
    """ToyModel split over ``world`` ranks (net1+ReLU | [Linear(10,10)+ReLU ...] | net2) with
    send/recv; ``batches`` varies the batch size step to step."""
    _init(rank, world, port)
    import torch.nn as nn

    from pytorch_distributed_training_tutorials_amd.parallel import comm as comm_mod
    from pytorch_distributed_training_tutorials_amd.parallel.env import destroy_process_group
    from pytorch_distributed_training_tutorials_amd.parallel.pipeline import PipelineStage

    stages = pipeline_reference_stages(world)
    stage_mod = stages[rank]
    c = comm_mod.get_default()
    st = PipelineStage(stage_mod, c, loss_fn=nn.MSELoss(), micro_batches=micro)
    opt = torch.optim.SGD(stage_mod.parameters(), lr=1e-3)
    g = torch.Generator().manual_seed(1)
    losses = []
    for b in batches:
        x = torch.randn(b, 1000, generator=g)
        y = torch.randn(b, 5, generator=g)
        opt.zero_grad()
        l = st.train_step(x if rank == 0 else None, y if rank == world - 1 else None)
        opt.step()
        losses.append(None if l is None else float(l))
    torch.save({"params": [p.detach() for p in stage_mod.parameters()], "losses": losses,
                "messages": st.messages, "headers": st.headers}, os.path.join(out_dir, f"r{rank}.pt"))
    destroy_process_group()


def pipeline_reference_stages(world):
    """Seeded stage modules: [Linear(1000,10)+ReLU, (Linear(10,10)+ReLU) x (world-2), Linear(10,5)]."""
    import torch.nn as nn

    torch.manual_seed(0)
    mods = [nn.Sequential(nn.Linear(1000, 10), nn.ReLU())]
    mods += [nn.Sequential(nn.Linear(10, 10), nn.ReLU()) for _ in range(world - 2)]
    mods.append(nn.Linear(10, 5))
    return mods


def _per_step_reference(eng, X, Y, sampler, n_steps, B, dev):
    """The same n DDP steps through the per-step kernel + standalone device sampler."""
    import math

    S = math.ceil(sampler.num_samples / B)
    idx = torch.zeros(sampler.num_samples, dtype=torch.int32, device=dev)
    sampler.set_epoch(0)
    for g in range(n_steps):
        j = g % S
        if j == 0:
            sampler.generate(idx)
        b = min(B, sampler.num_samples - j * B)
        eng.step(X, Y, idx[j * B:j * B + b], b)
    eng.flush()


def persistent_two_procs_one_gpu(rank, world, port, out_dir, kind="mlp"):
    if kind == "linear_nopair":  # the chunked exchange instead of the world-2 pair exchange
        os.environ["PTDT_XGMI_PAIR"] = "0"
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from pytorch_distributed_training_tutorials_amd.data.device_sampler import DeviceDistributedSampler
    from pytorch_distributed_training_tutorials_amd.models.toy import ToyMLP
    from pytorch_distributed_training_tutorials_amd.ops.fused_step import FusedMLPStep
    from pytorch_distributed_training_tutorials_amd.parallel.comm import Communicator
    from pytorch_distributed_training_tutorials_amd.parallel.xgmi import XgmiAllReduce

    dev = torch.device("cuda", 0)
    ctl = Communicator(device=torch.device("cpu"))
    xg = XgmiAllReduce(ctl, dev, max_elems=4096)
    X = torch.randn(300, 20, generator=torch.Generator().manual_seed(9)).to(dev)
    Y = torch.randint(0, 4 if kind == "mlp" else 2, (300,), generator=torch.Generator().manual_seed(10)).to(dev)
    out = {}
    for mode in ("persistent", "per_step"):
        torch.manual_seed(5)
        # "mlp": workgroup engine; "linear": single-wave engine (Linear(20, 4) -> KP 10, DOUT 4 is not
        # instantiated, so use Linear(20, 2))
        model = ToyMLP(20, 16, 4) if kind == "mlp" else torch.nn.Linear(20, 2)
        eng = FusedMLPStep(model.to(dev), loss="ce_index", lr=0.05, momentum=0.9, xgmi=xg)
        variant = "wave_rows" if kind == "linear_rows" else None  # linear / linear_nopair: layout F
        if mode == "persistent":
            out["engine"] = eng.persistent_engine(16, DeviceDistributedSampler(300, world, rank, seed=3, device=dev),
                                                  variant)
        sampler = DeviceDistributedSampler(300, world, rank, seed=3, device=dev)
        if mode == "persistent":
            cursor = torch.zeros(2, dtype=torch.int32, device=dev)
            losses = torch.zeros(7, device=dev)
            eng.run_persistent(X, Y, 23, 16, sampler, cursor, losses, max_steps_per_launch=7, variant=variant)
            torch.cuda.synchronize()
            out["cursor"] = cursor.cpu()
        else:
            _per_step_reference(eng, X, Y, sampler, 23, 16, dev)
        torch.cuda.synchronize()
        xg.check()
        out[mode] = eng.P.cpu()
    torch.save(out, os.path.join(out_dir, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def fingerprint_check(rank, world, port, out_dir, diverge):
    os.environ["PTDT_DEBUG_FINGERPRINT"] = "1"
    _init(rank, world, port)
    from pytorch_distributed_training_tutorials_amd.parallel import comm as comm_mod
    from pytorch_distributed_training_tutorials_amd.parallel.env import destroy_process_group
    from pytorch_distributed_training_tutorials_amd.utils.debug import CollectiveMismatch, check_fingerprints

    c = comm_mod.get_default()
    c.all_reduce(torch.ones(4))
    op = "min" if (diverge and rank == 1) else "max"
    c.all_reduce(torch.ones(4), op)  # a rank issuing a different reduction: silent garbage without the check
    res = {}
    try:
        res["n"] = check_fingerprints(c)
        res["ok"] = True
    except CollectiveMismatch as e:
        res["ok"] = False
        res["msg"] = str(e)
    torch.save(res, os.path.join(out_dir, f"r{rank}.pt"))
    destroy_process_group()


def bucket_all_reduce(rank, world, port, out_dir, numel):
    _init(rank, world, port)
    from pytorch_distributed_training_tutorials_amd.parallel import comm as comm_mod
    from pytorch_distributed_training_tutorials_amd.parallel.env import destroy_process_group

    c = comm_mod.get_default()
    t = torch.full((numel,), float(rank + 1))
    t[-1] = rank * 2.0
    c.all_reduce(t, "avg")
    expect = sum(range(1, world + 1)) / world
    b = torch.full((numel,), float(rank))
    c.broadcast(b, world - 1)
    res = {"avg_ok": bool(torch.allclose(t[:-1], torch.full((numel - 1,), expect))) and
           abs(float(t[-1]) - sum(2.0 * r for r in range(world)) / world) < 1e-6,
           "avg0": float(t[0]), "bcast_ok": bool((b == world - 1).all())}
    torch.save(res, os.path.join(out_dir, f"r{rank}.pt"))
    destroy_process_group()


def trainer_xgmi_fallback_one_gpu(rank, world, port, out_dir, inject):
    """Trainer on the persistent xGMI engine, two ranks sharing cuda:0 (gloo control
    plane). With ``inject`` rank 1 stops pushing its gradients to rank 0 from
    collective 20 on (PTDT_FAULT_XGMI_DROP_RANK/SEQ) and the poll budget is short:
    the in-kernel all-reduce times out, and every rank must detect it, restore
    the launch's starting state and re-run the epochs on the fused engine."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    if inject:
        os.environ["PTDT_FAULT_XGMI_DROP_RANK"] = "1"
        os.environ["PTDT_FAULT_XGMI_DROP_SEQ"] = "20"
        os.environ["PTDT_XGMI_MAX_POLLS"] = "20000"
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from pytorch_distributed_training_tutorials_amd.data import DeviceDataLoader, DeviceTensorDataset, DistributedSampler
    from pytorch_distributed_training_tutorials_amd.models.toy import ToyMLP
    from pytorch_distributed_training_tutorials_amd.ops.optim import FusedSGD
    from pytorch_distributed_training_tutorials_amd.parallel.comm import HostStagedComm
    from pytorch_distributed_training_tutorials_amd.utils.trainer import Trainer

    dev = torch.device("cuda", 0)
    comm = HostStagedComm(dev)
    torch.manual_seed(3)
    ds = DeviceTensorDataset.synthetic_classification(256, 20, 4, device=dev, seed=11)
    out = {}
    for engine in ("persistent", "fused"):
        torch.manual_seed(4 + rank)  # different init per rank: the Trainer broadcasts rank 0's
        model = ToyMLP(20, 16, 4)
        loader = DeviceDataLoader(ds, batch_size=16, sampler=DistributedSampler(ds, world, rank, seed=5))
        t = Trainer(model, loader, FusedSGD(model.parameters(), lr=0.05, momentum=0.9), 0, engine=engine,
                    comm=comm, graph=False, verbose=False)
        out[engine + "_engine"] = t.engine_name
        t.train(3)
        torch.cuda.synchronize()
        out[engine] = torch.cat([p.detach().reshape(-1) for p in model.parameters()]).cpu()
        out[engine + "_fallbacks"] = len(t.fallbacks)
        out[engine + "_final_engine"] = t.engine_name
    torch.save(out, os.path.join(out_dir, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def ddp_wrapper_collectable(rank, world, port, out_dir):
    """A dropped DDP wrapper is collected (its hooks hold it weakly) and the model
    trains as a plain module afterwards (sink/hook closures held the wrapper)."""
    _init(rank, world, port)
    import gc
    import weakref

    import torch.nn as nn

    from pytorch_distributed_training_tutorials_amd.parallel.ddp import DistributedDataParallel
    from pytorch_distributed_training_tutorials_amd.parallel.env import destroy_process_group

    torch.manual_seed(0)
    model = nn.Sequential(nn.Linear(8, 8), nn.ReLU(), nn.Linear(8, 2))
    ddp = DistributedDataParallel(model)
    ddp(torch.randn(4, 8)).sum().backward()
    ref = weakref.ref(ddp)
    del ddp
    gc.collect()
    model.zero_grad()
    model(torch.randn(4, 8)).sum().backward()  # no stale hook of the dead wrapper fires
    torch.save({"collected": ref() is None, "grads": all(p.grad is not None for p in model.parameters())},
               os.path.join(out_dir, f"r{rank}.pt"))
    destroy_process_group()


def spin_barrier_check(rank, world, port, out_dir):
    import time

    _init(rank, world, port)
    from pytorch_distributed_training_tutorials_amd.parallel import comm as comm_mod
    from pytorch_distributed_training_tutorials_amd.parallel.env import destroy_process_group
    from pytorch_distributed_training_tutorials_amd.utils import spin_barrier

    os.environ["LOCAL_WORLD_SIZE"] = str(world)
    c = comm_mod.get_default(None)
    bar = spin_barrier.create(c)
    assert bar is not None
    arrive, leave = [], []
    for rnd in range(3):
        if rank == rnd % world:
            time.sleep(0.05)  # the late rank of this round
        arrive.append(time.clock_gettime(time.CLOCK_MONOTONIC))
        bar.wait()
        leave.append(time.clock_gettime(time.CLOCK_MONOTONIC))
    bar.close()
    torch.save({"arrive": arrive, "leave": leave}, os.path.join(out_dir, f"r{rank}.pt"))
    destroy_process_group()


def spin_barrier_setup_failure(rank, world, port, out_dir, failing_rank):
    """One rank cannot map the shared page: every rank gets None from spin_barrier.create (nobody is
    left waiting in a collective), and no /dev/shm file is left behind."""
    _init(rank, world, port)
    from pytorch_distributed_training_tutorials_amd.parallel import comm as comm_mod
    from pytorch_distributed_training_tutorials_amd.parallel.env import destroy_process_group
    from pytorch_distributed_training_tutorials_amd.utils import spin_barrier

    os.environ["LOCAL_WORLD_SIZE"] = str(world)
    c = comm_mod.get_default(None)
    if rank == failing_rank:
        real_mmap = spin_barrier.mmap.mmap

        def broken(*a, **k):
            raise OSError(28, "No space left on device (injected)")

        spin_barrier.mmap.mmap = broken
    bar = spin_barrier.create(c)
    if rank == failing_rank:
        spin_barrier.mmap.mmap = real_mmap
    c.barrier()
    left = [f for f in os.listdir("/dev/shm") if f.startswith(f"ptdt_spin_")]
    torch.save({"none": bar is None, "left": left}, os.path.join(out_dir, f"r{rank}.pt"))
    destroy_process_group()


def tuning_agree(rank, world, port, out_dir):
    """Each rank 'times' a different winner; utils.tuning.agree hands every rank rank 0's."""
    _init(rank, world, port)
    from pytorch_distributed_training_tutorials_amd.parallel.env import destroy_process_group
    from pytorch_distributed_training_tutorials_amd.utils import tuning

    from pytorch_distributed_training_tutorials_amd.parallel import comm as comm_mod

    c = comm_mod.get_default(torch.device("cpu"))
    # outside an SPMD scope (no DDP forward open): own timing, no collective
    outside = tuning.agree("linear", ("nt", 1, 2, 3 + rank), ("native", "library")[rank % 2], ("native", "library"))
    tuning.spmd_begin(c)
    got = []
    with tuning.ddp_forward():  # an armed scope is in effect inside a DDP forward (or a backward)
        for k in range(3):
            local = ("native", "library")[(rank + k) % 2]
            got.append(tuning.agree("linear", ("nt", 128, 1000 + k, 2048), local, ("native", "library")))
        # ranks reaching different keys at the same point: every rank raises
        mismatch = None
        try:
            tuning.agree("linear", ("nt", 64, 64 + rank, 64), "native", ("native", "library"))
        except RuntimeError as e:
            mismatch = str(e)
    tuning.spmd_end(c)
    torch.save({"got": got, "choices": tuning.choices(), "outside": outside, "mismatch": mismatch},
               os.path.join(out_dir, f"r{rank}.pt"))
    destroy_process_group()


def tp_bf16_ranks_one_gpu(rank, world, port, out_dir):
    """bf16 TP engine at world W on one shared GPU (gloo control plane, xGMI exchange over IPC)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from pytorch_distributed_training_tutorials_amd.data.device_sampler import DeviceDistributedSampler
    from pytorch_distributed_training_tutorials_amd.models.toy import ToyMLP
    from pytorch_distributed_training_tutorials_amd.ops.fused_step import FusedMLPStep
    from pytorch_distributed_training_tutorials_amd.parallel.comm import Communicator
    from pytorch_distributed_training_tutorials_amd.parallel.xgmi import XgmiAllReduce

    dev = torch.device("cuda", 0)
    ctl = Communicator(device=torch.device("cpu"))
    xg = XgmiAllReduce(ctl, dev, max_elems=4096)
    X = torch.randn(300, 20, generator=torch.Generator().manual_seed(9)).to(dev)
    Y = torch.randint(0, 10, (300,), generator=torch.Generator().manual_seed(10)).to(dev)
    torch.manual_seed(5)
    model = ToyMLP(20, 64, 10).to(dev)
    init = [p.detach().cpu().clone() for p in model.parameters()]
    eng = FusedMLPStep(model, loss="ce_index", lr=0.05, momentum=0.9, xgmi=xg, dtype="bf16")
    sampler = DeviceDistributedSampler(300, world, rank, seed=3, device=dev)
    orders = []
    for e in range(10):
        sampler.set_epoch(e)
        idx = torch.zeros(sampler.num_samples, dtype=torch.int32, device=dev)
        sampler.generate(idx)
        orders.append(idx.cpu())
    sampler.set_epoch(0)
    cursor = torch.zeros(2, dtype=torch.int32, device=dev)
    losses = torch.zeros(7, device=dev)
    engine = eng.persistent_engine(16, sampler)
    eng.run_persistent(X, Y, 23, 16, sampler, cursor, losses, max_steps_per_launch=7)
    torch.cuda.synchronize()
    xg.check()
    torch.save({"engine": engine, "params": eng.P.cpu(), "init": init, "orders": orders, "X": X.cpu(), "Y": Y.cpu()},
               os.path.join(out_dir, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def fallback_chain(rank, world, port, out_dir, inject):
    """utils/fallback.run_chain over gloo with stages shaped like bench.py's engines (their decision
    points in order); ``inject`` is PTDT_BENCH_INJECT's syntax."""
    _init(rank, world, port)
    import torch.distributed as dist

    from pytorch_distributed_training_tutorials_amd.utils.fallback import (Decider, DesyncError, StageFailed,
                                                                          control_group, run_chain)

    dec = Decider(rank, world, control_group(world), inject=inject)

    def persistent(d):
        d.check("device")
        d.check("xgmi_init")
        d.check("xgmi_poll_warmup")
        dist.barrier()  # stands for the timed region (collective on every rank)
        d.check("xgmi_poll_timed")
        return "persistent-result"

    def fused_graph(d):
        d.check("device")
        if f"early@{rank}" in inject:  # a local exception BEFORE a decision point the others reach
            raise ValueError("local crash before graph_capture")
        d.check("graph_capture")
        d.allclose("graph_replay_check", torch.ones(3), torch.ones(3) * (1.0 if "replay_diff" not in inject else 1.5))
        return "fused-graph-result"

    def fused_eager(d):
        d.check("device")
        if f"crash@{rank}" in inject:  # an unexpected local exception (not a decision point)
            raise ValueError("local crash")
        return "fused-eager-result"

    def reference(d):
        return "reference-result"

    stages = [("persistent", persistent), ("fused_graph", fused_graph), ("fused_eager", fused_eager),
              ("reference", reference)]
    try:
        name, res, failures = run_chain(dec, stages, log=None)
        out = {"name": name, "res": res, "failures": failures, "points": dec.points}
    except StageFailed as e:
        out = {"name": None, "error": str(e), "points": dec.points}
    except DesyncError as e:
        out = {"name": None, "desync": "different decision points" in str(e)}
    torch.save(out, os.path.join(out_dir, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def tuning_scopes(rank, world, port, out_dir):
    """utils/tuning SPMD scopes under the native DDP wrapper: two wrappers in one step
    keep their own counts, a backward agrees inside the scope, a shape first decided by rank 0
    alone is agreed again inside a DDP forward, and a grad-enabled forward without backward does
    not make a later rank-0-only inference broadcast alone."""
    _init(rank, world, port)
    import torch.nn as nn

    from pytorch_distributed_training_tutorials_amd.parallel.ddp import DistributedDataParallel
    from pytorch_distributed_training_tutorials_amd.parallel.env import destroy_process_group
    from pytorch_distributed_training_tutorials_amd.utils import tuning

    seen = {}
    opts = ("native", "library")

    def decide(key, local):  # ops/linear.py's flow: a valid cached decision, else (re-)agree
        hit = tuning.lookup("linear", key)
        if hit is not None:
            return hit
        return tuning.agree("linear", key, tuning.local_choice("linear", key) or local, opts)

    class Pick(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, tag):
            ctx.tag = tag
            seen[f"fwd:{tag}:{x.shape[0]}"] = decide(("fw", tag, x.shape[0]), opts[rank % 2])
            return x * 1.0

        @staticmethod
        def backward(ctx, g):
            seen[f"bwd:{ctx.tag}"] = decide(("bw", ctx.tag), opts[(rank + 1) % 2])
            return g, None

    class M(nn.Module):
        def __init__(self, tag):
            super().__init__()
            self.lin = nn.Linear(4, 4)
            self.tag = tag

        def forward(self, x):
            return Pick.apply(self.lin(x), self.tag)

    torch.manual_seed(0)
    a, b = DistributedDataParallel(M(1)), DistributedDataParallel(M(2))
    c = a.comm
    x = torch.randn(3, 4)
    out = {}
    # two wrappers, one step: B's scope survives A's finalisation (round 5 set depth = 1 / 0)
    yb = b(x)
    ya = a(x)
    out["depth_after_fwd"] = tuning.scope_depth(c)
    ya.sum().backward()
    out["depth_after_a_bwd"] = tuning.scope_depth(c)
    yb.sum().backward()
    out["depth_after_b_bwd"] = tuning.scope_depth(c)
    # a shape decided by rank 0 alone (outside any scope), then reached by every rank in DDP
    if rank == 0:
        a.module(torch.randn(5, 4))  # rank-0-only: local decision, no collective
    a(torch.randn(5, 4)).sum().backward()
    # grad-enabled forward with no backward, then a rank-0-only inference of a new shape
    a(torch.randn(6, 4))
    out["depth_stale"] = tuning.scope_depth(c)
    if rank == 0:
        a.module(torch.randn(7, 4))  # must not broadcast: no DDP forward / backward is running
    a(torch.randn(8, 4)).sum().backward()  # closes the stale scope first
    out["depth_end"] = tuning.scope_depth(c)
    with torch.no_grad():
        a(torch.randn(9, 4))
    out["depth_no_grad"] = tuning.scope_depth(c)
    out["seen"] = seen
    torch.save(out, os.path.join(out_dir, f"r{rank}.pt"))
    destroy_process_group()


def pipeline_late_violation(rank, world, port, out_dir):
    """Stage 0 changes its output width at micro-batch 2 (after the step header went out): it
    raises at the end of the step, every other stage completes the step, and a second step
    after the error still runs (no peer left blocked on a message)."""
    _init(rank, world, port)
    import torch.nn as nn

    from pytorch_distributed_training_tutorials_amd.parallel import comm as comm_mod
    from pytorch_distributed_training_tutorials_amd.parallel.env import destroy_process_group
    from pytorch_distributed_training_tutorials_amd.parallel.pipeline import PipelineStage

    class Flaky(nn.Module):
        def __init__(self):
            super().__init__()
            self.lin = nn.Linear(8, 6)
            self.calls = 0
            self.bad_at = 2

        def forward(self, x):
            self.calls += 1
            y = self.lin(x)
            return y[:, :4] if self.calls - 1 == self.bad_at else y

    torch.manual_seed(0)
    mods = [Flaky()] + [nn.Linear(6, 6) for _ in range(world - 2)] + [nn.Linear(6, 3)]
    c = comm_mod.get_default()
    st = PipelineStage(mods[rank], c, loss_fn=nn.MSELoss(), micro_batches=4)
    g = torch.Generator().manual_seed(1)
    out = {"errors": [], "losses": []}
    for step in range(2):
        x, y = torch.randn(16, 8, generator=g), torch.randn(16, 3, generator=g)
        try:
            l = st.train_step(x if rank == 0 else None, y if rank == world - 1 else None)
            out["losses"].append(None if l is None else float(l))
        except RuntimeError as e:
            out["errors"].append(str(e))
    torch.save(out, os.path.join(out_dir, f"r{rank}.pt"))
    destroy_process_group()
