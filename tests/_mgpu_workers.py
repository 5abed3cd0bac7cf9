"""Worker bodies for the multi-GPU tests (one process per GPU, RCCL over xGMI).
Importable without a GPU; every function runs in a spawned process."""
import contextlib
import os

import torch
import torch.nn.functional as F


def _init_gpu(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["LOCAL_RANK"] = str(rank)
    from pytorch_distributed_training_tutorials_amd.parallel import comm as comm_mod
    from pytorch_distributed_training_tutorials_amd.parallel import env

    env.ddp_setup(rank, world, master_addr="127.0.0.1", master_port=port, backend="nccl")
    dev = torch.device("cuda", rank)
    torch.cuda.set_device(dev)
    return dev, comm_mod.get_default(dev)


def _digest_equal(comm, t: torch.Tensor) -> bool:
    return len(set(comm.all_gather_object(t.detach().float().cpu().numpy().tobytes()))) == 1


def ddp_gpu(rank, world, port, out_dir):
    """Native DDP (C++ reducer, RCCL buckets on the comm stream) on cuda:rank with a
    per-rank batch of 8 rows of a shared global batch (ddp_gpus.py:32-39)."""
    dev, comm = _init_gpu(rank, world, port)
    from pytorch_distributed_training_tutorials_amd.models.toy import ToyMLP
    from pytorch_distributed_training_tutorials_amd.ops.optim import FusedSGD
    from pytorch_distributed_training_tutorials_amd.parallel.ddp import DistributedDataParallel
    from pytorch_distributed_training_tutorials_amd.parallel.env import destroy_process_group

    torch.manual_seed(100 + rank)  # different init per rank: DDP broadcasts rank 0's
    model = ToyMLP(20, 16, 5).to(dev)
    ddp = DistributedDataParallel(model, device_ids=[rank], comm=comm, bucket_cap_mb=0.0005, first_bucket_mb=0.0001)
    opt = FusedSGD(model.parameters(), lr=0.1, momentum=0.9)
    g = torch.Generator().manual_seed(0)
    X = torch.randn(4, 8 * world, 20, generator=g)
    Y = torch.randint(0, 5, (4, 8 * world), generator=g)
    for it in range(4):
        xs = X[it, rank * 8:(rank + 1) * 8].to(dev)
        ys = Y[it, rank * 8:(rank + 1) * 8].to(dev)
        ddp.zero_grad()
        F.cross_entropy(ddp(xs), ys).backward()
        opt.step()
    torch.cuda.synchronize()
    flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
    torch.save({"params": flat.cpu(), "in_sync": _digest_equal(comm, flat),
                "buckets": len(ddp.bucket_sizes_bytes())}, os.path.join(out_dir, f"r{rank}.pt"))
    destroy_process_group()


def xgmi_gpu(rank, world, port, out_dir):
    """In-kernel one-shot xGMI all-reduce across distinct GPUs vs RCCL ncclAvg, and the
    persistent DDP engines (xGMI inside the kernel) vs the fused engine + RCCL."""
    dev, comm = _init_gpu(rank, world, port)
    from tests._workers import _per_step_reference

    from pytorch_distributed_training_tutorials_amd.data.device_sampler import DeviceDistributedSampler
    from pytorch_distributed_training_tutorials_amd.models.toy import ToyMLP
    from pytorch_distributed_training_tutorials_amd.ops.fused_step import FusedMLPStep
    from pytorch_distributed_training_tutorials_amd.parallel.env import destroy_process_group
    from pytorch_distributed_training_tutorials_amd.parallel.xgmi import XgmiAllReduce

    out = {}
    xg = XgmiAllReduce(comm, dev)
    out["ok"] = xg.ok
    errs = {}
    for n in (21, 1994, 65536):
        g = torch.Generator(device=dev).manual_seed(1000 * rank + n)
        t = torch.randn(n, device=dev, generator=g)
        a, b = t.clone(), t.clone()
        if xg.ok:
            xg.all_reduce_avg(a)
        comm.all_reduce(b, "avg")
        torch.cuda.synchronize()
        errs[n] = float((a - b).abs().max()) if xg.ok else None
        out[f"xgmi_in_sync_{n}"] = _digest_equal(comm, a)
    out["max_err"] = errs
    out["poll_error"] = xg.x.error() if xg.ok else None
    X = torch.randn(2048, 20, generator=torch.Generator().manual_seed(9)).to(dev)
    Y = torch.randint(0, 4, (2048,), generator=torch.Generator().manual_seed(10)).to(dev)
    for kind in ("linear", "mlp"):
        res = {}
        for mode in ("persistent", "per_step_rccl"):
            torch.manual_seed(5)
            model = (ToyMLP(20, 16, 4) if kind == "mlp" else torch.nn.Linear(20, 2)).to(dev)
            eng = FusedMLPStep(model, loss="ce_index", lr=0.05, momentum=0.9, comm=comm,
                               xgmi=xg if (mode == "persistent" and xg.ok) else None)
            sampler = DeviceDistributedSampler(2048, world, rank, seed=3, device=dev)
            if mode == "persistent" and xg.ok:
                out[f"{kind}_engine"] = eng.persistent_engine(16, sampler)
                cursor = torch.zeros(2, dtype=torch.int32, device=dev)
                losses = torch.zeros(64, device=dev)
                plan = eng.persistent_plan(X, Y, 16, sampler, cursor, losses)
                for n in (3, 40, 64, 13):  # 120 steps across epoch boundaries
                    plan.launch(n)
                torch.cuda.synchronize()
                xg.check()
            else:
                _per_step_reference(eng, X, Y, sampler, 120, 16, dev)
            torch.cuda.synchronize()
            res[mode] = eng.P.clone()
            out[f"{kind}_{mode}_in_sync"] = _digest_equal(comm, eng.P)
        out[f"{kind}_err"] = float((res["persistent"] - res["per_step_rccl"]).abs().max()) if xg.ok else None
    torch.save(out, os.path.join(out_dir, f"r{rank}.pt"))
    destroy_process_group()


def pipeline_gpu(rank, world, port, out_dir, micro, batches=(20, 20, 20)):
    """ToyModel split over two GPUs and two ranks with RCCL send/recv (NB03:440-450); P2P on
    the stage's side stream, batch size varying step to step."""
    dev, comm = _init_gpu(rank, world, port)
    import torch.nn as nn

    from pytorch_distributed_training_tutorials_amd.parallel.env import destroy_process_group
    from pytorch_distributed_training_tutorials_amd.parallel.pipeline import PipelineStage

    from ._workers import pipeline_reference_stages

    stage_mod = pipeline_reference_stages(world)[rank].to(dev)
    st = PipelineStage(stage_mod, comm, loss_fn=nn.MSELoss(), micro_batches=micro)
    assert st._side is not None  # the overlapped (side-stream) P2P path is the one under test
    opt = torch.optim.SGD(stage_mod.parameters(), lr=1e-3)
    g = torch.Generator().manual_seed(1)
    losses = []
    for b in batches:
        x = torch.randn(b, 1000, generator=g)
        y = torch.randn(b, 5, generator=g)
        opt.zero_grad()
        l = st.train_step(x.to(dev) if rank == 0 else None, y.to(dev) if rank == world - 1 else None)
        opt.step()
        losses.append(None if l is None else float(l))
    torch.save({"params": [p.detach().cpu() for p in stage_mod.parameters()], "losses": losses},
               os.path.join(out_dir, f"r{rank}.pt"))
    destroy_process_group()


def trainer_gpu(rank, world, port, out_dir):
    """The ddp_gpus_torchrun.py job on W GPUs through the product Trainer (persistent
    engine, in-kernel xGMI all-reduce): status lines, steps/epoch, replicas in sync."""
    dev, comm = _init_gpu(rank, world, port)
    import contextlib
    import io

    from pytorch_distributed_training_tutorials_amd.data import DeviceDataLoader, DeviceTensorDataset, DistributedSampler
    from pytorch_distributed_training_tutorials_amd.models.toy import ToyMLP
    from pytorch_distributed_training_tutorials_amd.parallel.env import destroy_process_group
    from pytorch_distributed_training_tutorials_amd.utils.trainer import Trainer

    out = {}
    ds = DeviceTensorDataset.synthetic_classification(2048, 20, 4, device=dev, seed=1)
    for engine in ("auto", "fused"):
        torch.manual_seed(7 + rank)
        model = ToyMLP(20, 32, 4)
        loader = DeviceDataLoader(ds, batch_size=32, sampler=DistributedSampler(ds, world, rank))
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            t = Trainer(model, loader, torch.optim.SGD(model.parameters(), lr=0.05, momentum=0.9), rank,
                        engine=engine, comm=comm)
            t.train(3)
        torch.cuda.synchronize()
        flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
        out[engine] = {"engine": t.engine_name, "lines": buf.getvalue().splitlines(), "params": flat.cpu(),
                       "in_sync": _digest_equal(comm, flat), "fallbacks": len(t.fallbacks)}
    torch.save(out, os.path.join(out_dir, f"r{rank}.pt"))
    destroy_process_group()


def _init_any(rank, world, port, gpu: bool):
    if gpu:
        return _init_gpu(rank, world, port)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    from pytorch_distributed_training_tutorials_amd.parallel import comm as comm_mod
    from pytorch_distributed_training_tutorials_amd.parallel import env

    env.ddp_setup(rank, world, master_addr="127.0.0.1", master_port=port, backend="gloo")
    dev = torch.device("cpu")
    return dev, comm_mod.get_default(dev)


RESNET_CFG = {"layers": (1, 1, 1, 1), "classes": 10, "batch": 2, "image": 32, "steps": 3, "lr": 0.05}


def resnet_ddp(rank, world, port, out_dir, gpu=True, accum=1, ref=False):
    """Native ResNet DDP (small Bottleneck ResNet) on cuda:rank: channels_last, bf16 autocast, FusedSGD
    with bf16 weight shadows -- so the grad sinks, the deferred bf16->fp32 gradient casts and the bucket
    rebuild after iteration 0 all run at world > 1 (VERDICT r4 #6a). Each rank trains on its B rows of
    a shared global batch. ``gpu=False``: the same host logic on CPU / gloo (fp32, no shadows).
    ``accum > 1`` (world 1): the reference -- the same native path, each step accumulating ``accum``
    micro-batches of B rows under ``no_sync`` with the loss scaled by 1/accum; ``ref`` saves to ref.pt."""
    dev, comm = _init_any(rank, world, port, gpu)
    from pytorch_distributed_training_tutorials_amd.models.resnet import Bottleneck, ResNet
    from pytorch_distributed_training_tutorials_amd.ops.loss import cross_entropy
    from pytorch_distributed_training_tutorials_amd.ops.optim import FusedSGD
    from pytorch_distributed_training_tutorials_amd.parallel.ddp import DistributedDataParallel
    from pytorch_distributed_training_tutorials_amd.parallel.env import destroy_process_group

    c = RESNET_CFG
    if gpu:
        torch.backends.cudnn.benchmark, torch.backends.cudnn.deterministic = False, True
    torch.manual_seed(100 + rank)  # different init per rank: DDP broadcasts rank 0's
    model = ResNet(Bottleneck, c["layers"], num_classes=c["classes"]).to(dev)
    if gpu:
        model = model.to(memory_format=torch.channels_last)
    ddp = DistributedDataParallel(model, device_ids=[rank] if gpu else None, comm=comm, bucket_cap_mb=4.0,
                                  first_bucket_mb=1.0)
    opt = FusedSGD(model.parameters(), lr=c["lr"], momentum=0.9, weight_decay=1e-4, bf16_shadow=gpu)
    g = torch.Generator().manual_seed(0)
    B, S = c["batch"], c["steps"]
    G = world * accum
    X = torch.randn(S, B * G, 3, c["image"], c["image"], generator=g)
    Y = torch.randint(0, c["classes"], (S, B * G), generator=g)
    losses = []
    for it in range(S):
        ddp.zero_grad()
        for a in range(accum):
            r = rank * accum + a
            xs = X[it, r * B:(r + 1) * B].to(dev)
            if gpu:
                xs = xs.contiguous(memory_format=torch.channels_last)
            ys = Y[it, r * B:(r + 1) * B].to(dev)
            sync = ddp.no_sync() if a + 1 < accum else contextlib.nullcontext()
            with sync:
                with torch.autocast("cuda", dtype=torch.bfloat16, enabled=gpu, cache_enabled=False):
                    out = ddp(xs)
                loss = cross_entropy(out.float(), ys) / accum
                loss.backward()
        opt.step()
        losses.append(float(loss.detach()))
    if gpu:
        torch.cuda.synchronize()
    flat = torch.cat([p.detach().float().reshape(-1) for p in model.parameters()])
    torch.save({"params": flat.cpu(), "in_sync": _digest_equal(comm, flat), "losses": losses,
                "buckets": len(ddp.bucket_sizes_bytes()), "rebuilt": bool(ddp._rebuilt),
                "sinks": len(getattr(ddp, "_sink_params", [])), "deferred": bool(getattr(ddp, "_defer", False))},
               os.path.join(out_dir, "ref.pt" if ref else f"r{rank}.pt"))
    destroy_process_group()


def resnet_reference(world, gpu: bool):
    """One process on the same global batch: each rank's B rows are a micro-batch (BatchNorm sees the
    same rows as on that rank), gradients accumulated with weight 1/W, torch.optim.SGD -- what
    DDP's averaged all-reduce must reproduce. fp32 (the GPU workers run bf16 autocast)."""
    from pytorch_distributed_training_tutorials_amd.models.resnet import Bottleneck, ResNet

    c = RESNET_CFG
    dev = torch.device("cuda", 0) if gpu else torch.device("cpu")
    torch.manual_seed(100)
    model = ResNet(Bottleneck, c["layers"], num_classes=c["classes"]).to(dev)
    if gpu:  # the native BN kernels take channels_last activations on the GPU
        model = model.to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(model.parameters(), lr=c["lr"], momentum=0.9, weight_decay=1e-4)
    g = torch.Generator().manual_seed(0)
    B, S = c["batch"], c["steps"]
    X = torch.randn(S, B * world, 3, c["image"], c["image"], generator=g)
    Y = torch.randint(0, c["classes"], (S, B * world), generator=g)
    for it in range(S):
        opt.zero_grad()
        for r in range(world):
            xr = X[it, r * B:(r + 1) * B].to(dev)
            out = model(xr.contiguous(memory_format=torch.channels_last) if gpu else xr)
            (F.cross_entropy(out.float(), Y[it, r * B:(r + 1) * B].to(dev)) / world).backward()
        opt.step()
    return torch.cat([p.detach().float().reshape(-1) for p in model.parameters()]).cpu()


def graphed_ddp_gpu(rank, world, port, out_dir):
    """GraphedStep with the DDP bucket all-reduces captured (RCCL inside the replayed graph) at
    world > 1: replays from a snapshot == eager steps from the same snapshot, replicas bitwise equal,
    and the captured collectives counted (VERDICT r4 #6b)."""
    dev, comm = _init_gpu(rank, world, port)
    from pytorch_distributed_training_tutorials_amd.models.toy import ToyMLP
    from pytorch_distributed_training_tutorials_amd.ops.loss import cross_entropy
    from pytorch_distributed_training_tutorials_amd.ops.optim import FusedSGD
    from pytorch_distributed_training_tutorials_amd.parallel.ddp import DistributedDataParallel
    from pytorch_distributed_training_tutorials_amd.parallel.env import destroy_process_group
    from pytorch_distributed_training_tutorials_amd.utils.graphs import GraphedStep

    torch.manual_seed(7)
    model = ToyMLP(20, 64, 10).to(dev)
    ddp = DistributedDataParallel(model, device_ids=[rank], comm=comm, bucket_cap_mb=0.002, first_bucket_mb=0.001)
    opt = FusedSGD(model.parameters(), lr=0.05, momentum=0.9)
    g = torch.Generator().manual_seed(rank)
    x = torch.randn(32, 20, generator=g).to(dev)
    y = torch.randint(0, 10, (32,), generator=g).to(dev)

    def step():
        ddp.zero_grad()
        loss = cross_entropy(ddp(x), y)
        loss.backward()
        opt.step()
        return loss

    gs = GraphedStep(step, dev, comm=comm, warmup=3)
    live = [p.data for p in model.parameters()] + [opt.state[p]["momentum_buffer"] for p in model.parameters()
                                                   if "momentum_buffer" in opt.state.get(p, {})]
    live += list(opt._counters.values())
    snap = [t.clone() for t in live]
    rl = [float(gs()) for _ in range(4)]
    torch.cuda.synchronize()
    pa = torch.cat([p.detach().reshape(-1) for p in model.parameters()]).clone()
    with torch.no_grad():
        for t, s in zip(live, snap):
            t.copy_(s)
    el = [float(step()) for _ in range(4)]
    torch.cuda.synchronize()
    pb = torch.cat([p.detach().reshape(-1) for p in model.parameters()]).clone()
    torch.save({"n_collectives": gs.n_collectives, "replay_losses": rl, "eager_losses": el,
                "max_gap": float((pa - pb).abs().max()), "in_sync": _digest_equal(comm, pa)},
               os.path.join(out_dir, f"r{rank}.pt"))
    destroy_process_group()


def xgmi_peer_matrix(rank, world, port, out_dir):
    """The xGMI self-test across devices plus the peer-access matrix every rank sees (VERDICT r4 #6c)."""
    dev, comm = _init_gpu(rank, world, port)
    from pytorch_distributed_training_tutorials_amd.parallel.env import destroy_process_group
    from pytorch_distributed_training_tutorials_amd.parallel.xgmi import XgmiAllReduce

    n = torch.cuda.device_count()
    matrix = [[i == j or torch.cuda.can_device_access_peer(i, j) for j in range(n)] for i in range(n)]
    xg = XgmiAllReduce(comm, dev)
    torch.save({"ok": xg.ok, "why": getattr(xg, "why", None), "matrix": matrix, "visible": n},
               os.path.join(out_dir, f"r{rank}.pt"))
    destroy_process_group()
