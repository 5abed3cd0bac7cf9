#!/usr/bin/env python3
"""Flagship benchmark: DDP toy training throughput (whole-node samples/s).

Metric / config (BASELINE.json): "samples/sec (whole node) + DDP scaling eff.,
toy MLP at 1/2/4/8 MI355X" on ``ddp_gpus_torchrun.py``'s job -- ``Linear(20, 1)``,
``F.cross_entropy`` on float targets, ``SGD(lr=1e-2)``, per-device batch 32,
2048-sample synthetic dataset, DistributedSampler sharding, DDP gradient
all-reduce every step (reference ddp_gpus_torchrun.py:16-88). Weak scaling:
per-GPU batch fixed, global batch 32*N.

Contract: ``python bench.py --gpus N --steps K --warmup W`` (N>1 under
``torch.distributed.run``); W untimed warmup steps (rounded up to whole
epochs), then EXACTLY K timed steps bracketed by barrier + synchronize, the
MAX elapsed over ranks, one JSON line from rank 0.

Every timed step does the full work: batch gather by sampler index, forward,
loss, backward, all-reduce of the gradient bucket across all ranks, SGD update.
The sampler permutation is produced on device once per epoch, as the reference
produces it once per epoch (``set_epoch``): an epoch that starts inside the timed
steps has its list built inside the timed region (helper waves of the persistent
engines); one that started during the warm-up steps was built then and is read
from the launch-to-launch list cache (the driver's 20 timed steps at positions
5-24 lie inside the first 64-step epoch). Engines:
  persistent (default) many DDP steps per launch, in-kernel xGMI all-reduce
            (single-wave engine for Linear(Din, Dout), LDS workgroup engine otherwise)
  fused     fused step kernel + in-kernel xGMI or RCCL all-reduce, epochs
            captured into hipGraphs (ops/fused_step.py)
  autograd  native DDP reducer + native Linear/CE/SGD kernels, eager
  reference stock PyTorch-ROCm loop (torch DDP, DataLoader + DistributedSampler,
            nn.Linear, F.cross_entropy, torch.optim.SGD) -- the comparator

Comparator: after the headline, the SAME process times the stock PyTorch-ROCm
reference loop (``--engine reference`` body: torch DDP over RCCL, DataLoader +
DistributedSampler, same model/batch/N) and reports ``ref_samples_per_s`` and
``speedup_vs_torch``; ``vs_baseline`` is that same-node ratio ("the
like-for-like comparator is the unmodified reference scripts running on
PyTorch-ROCm on the same node"), the survey's CPU/gloo probe ratio is kept as
``vs_cpu_probe``.

Fallback: if the requested engine fails on ANY rank (no GPU, no peer memory for
the in-kernel xGMI exchange, an xGMI poll timeout, a hipGraph capture error, a
replayed graph that differs from the same steps run eagerly), every rank moves
to the next engine of persistent -> fused (hipGraph) -> fused (eager) ->
autograd -> stock torch together: each decision point is agreed over a gloo
control group (utils/fallback.py). The JSON line names the measured engine
(``engine_path``) and every failure (``fallback``: stage, point, each failing
rank's reason); ``--no_fallback`` measures the requested engine only.

Deadline: the whole run is bounded by ``--deadline`` seconds (default 420, under
the driver's limit) and every communicator by ``PTDT_COMM_TIMEOUT`` (default
120 s here). On expiry every rank aborts its communicators, rank 0 prints one
JSON line -- the headline's record if it was already measured (with
``"incomplete"``), else one with ``"error"`` and the phase the run died in -- and
the process exits non-zero (utils/deadline.py) -- no new process, no re-exec.
"""
from __future__ import annotations

import argparse
import contextlib
import json
import math
import os
import sys
import time

import torch

# BASELINE.md survey probe (unmodified reference loop, CPU/gloo, whole-node samples/s) at N = 1, 2, 4.
# N = 8 was not probed by the survey: benchmarks/reference_cpu_probe.py re-ran the same method here
# (W=1 69.3K, W=8 55.4K samples/s on this slower container) and the W=8/W=1 ratio scales the
# survey's W=1 figure: 99,000 * 55,383 / 69,272 = 79,150 (profiles/r2_reference_cpu_probe.md).
# The reference publishes no GPU DDP number; see BASELINE.md.
BASELINE_SAMPLES_PER_S = {1: 99_000.0, 2: 110_000.0, 4: 102_000.0, 8: 79_150.0}
METRIC = "samples/sec (whole node) + DDP scaling eff., toy MLP at 1/2/4/8 MI355X"


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--batch_size", type=int, default=32, help="per-device batch (reference default 32)")
    ap.add_argument("--dataset_size", type=int, default=2048)
    ap.add_argument("--lr", type=float, default=1e-2)
    ap.add_argument("--model", default="linear", choices=["linear", "mlp"],
                    help="linear = reference Linear(20,1)+soft CE; mlp = Linear(20,64)-ReLU-Linear(64,10)+CE")
    ap.add_argument("--hidden", type=int, default=64,
                    help="hidden width of --model mlp (64 = the north star's toy; probes only)")
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"],
                    help="bf16: the toy MLP (--model mlp) on the bf16 tensor-parallel engine with "
                         "torch.autocast(bfloat16) semantics and fp32 master weights (BASELINE config 2)")
    ap.add_argument("--engine", default="persistent", choices=["persistent", "fused", "autograd", "reference"])
    ap.add_argument("--graph_steps", type=int, default=128, help="target steps per captured hipGraph")
    ap.add_argument("--allreduce", default="auto", choices=["auto", "xgmi", "rccl"],
                    help="gradient all-reduce of the fused engine: in-kernel one-shot xGMI (auto: if its "
                         "self-test passes on every rank) or RCCL")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--persist", default=None, choices=["auto", "wave", "workgroup", "mfma", "tp"],
                    help="persistent engine variant (default: $PTDT_PERSIST or auto)")
    ap.add_argument("--sampler", default="device", choices=["device", "torch"],
                    help="device: in-kernel Feistel permutation (DistributedSampler semantics, different order); "
                         "torch: torch.randperm-identical order (csrc/kernels/torch_perm.hip) generated inside "
                         "the timed region, one launch per run")
    ap.add_argument("--stamps", action="store_true",
                    help="persistent engine: diagnostic run with in-kernel phase timers (separate from the timed run)")
    ap.add_argument("--out", default=None, help="also append the JSON line to this file")
    ap.add_argument("--no_mlp_side", action="store_true",
                    help="skip the extra toy-MLP measurement (mlp_us_per_step) after the headline run")
    ap.add_argument("--deadline", type=float, default=float(os.environ.get("PTDT_BENCH_DEADLINE", 420)),
                    help="whole-run deadline in seconds (0: none); on expiry an error JSON line is printed")
    ap.add_argument("--no_ref", action="store_true",
                    help="skip the same-process stock PyTorch-ROCm comparator after the headline")
    ap.add_argument("--ref_steps", type=int, default=None,
                    help="timed steps of the comparator (default max(--steps, 256); its warmup max(--warmup, 32))")
    ap.add_argument("--no_fallback", action="store_true",
                    help="measure the requested engine only: no agreed fallback chain (persistent -> fused "
                         "hipGraph -> fused eager -> native autograd -> stock torch) when it fails on a rank")
    ap.add_argument("--device", default="auto", choices=["auto", "cuda", "cpu"],
                    help="cpu: the reference engine on gloo (CPU plumbing / deadline tests)")
    ap.add_argument("--share_gpu", action="store_true",
                    help="REHEARSAL ONLY: every rank on cuda:0 with a gloo control plane (RCCL refuses two ranks "
                         "per GPU), to exercise the N>1 path (xGMI self-test, in-kernel all-reduce, replica-sync "
                         "check) on a 1-GPU box; the result is tagged and is not a scaling number")
    return ap.parse_args(argv)


def _setup(args, cpu: bool):
    from pytorch_distributed_training_tutorials_amd.parallel import env

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch N>1 with torch.distributed.run")
    env.init_process_group("gloo" if (args.share_gpu or cpu) else "nccl")
    return env.rank(), env.world_size(), env.local_rank()


def _replicas_in_sync(comm, params: torch.Tensor) -> bool:
    """DDP invariant after training: every rank holds bit-identical parameters."""
    if comm.world == 1:
        return True
    digest = params.detach().float().cpu().numpy().tobytes()
    return len(set(comm.all_gather_object(digest))) == 1


def _build_model(args, dev):
    from pytorch_distributed_training_tutorials_amd.models.toy import ToyMLP, ddp_toy_model

    torch.manual_seed(args.seed)
    if args.model == "linear":
        return ddp_toy_model(20, 1).to(dev), "ce_soft"
    return ToyMLP(20, args.hidden, 10).to(dev), "ce_index"


def _dataset(args, dev, loss):
    from pytorch_distributed_training_tutorials_amd.data import DeviceTensorDataset

    if loss == "ce_soft":
        return DeviceTensorDataset.synthetic_regression(args.dataset_size, 20, 1, device=dev, seed=args.seed)
    return DeviceTensorDataset.synthetic_classification(args.dataset_size, 20, 10, device=dev, seed=args.seed)


# --------------------------------------------------------------------------- fused
def run_fused(args, rank, world, dev, comm, dec, graph=True, allreduce=None):
    """Per-step fused kernel + all-reduce (in-kernel xGMI, or RCCL on the stream). ``graph``: epochs
    captured into hipGraphs, the capture and a replay-vs-eager check agreed across ranks before
    timing; otherwise every step is launched eagerly (the chain's last GPU resort before autograd)."""
    from pytorch_distributed_training_tutorials_amd.data.device_sampler import DeviceDistributedSampler
    from pytorch_distributed_training_tutorials_amd.ops.fused_step import FusedMLPStep

    dec.check("device", dev.type == "cuda", "the fused engine needs a GPU")
    allreduce = allreduce or args.allreduce
    model, loss = _build_model(args, dev)
    ds = _dataset(args, dev, loss)
    X, Y = ds.tensors
    from pytorch_distributed_training_tutorials_amd.parallel.xgmi import maybe_create

    xg = None if allreduce == "rccl" else maybe_create(comm, dev, mode="on" if allreduce == "xgmi" else None)
    if allreduce == "xgmi":
        dec.check("xgmi_init", xg is not None, "--allreduce xgmi requested but the xGMI path is unavailable")
    eng = FusedMLPStep(model, loss=loss, lr=args.lr, comm=comm, xgmi=xg)
    if world > 1:
        comm.broadcast(eng.P, 0)  # DDP init: rank 0's parameters everywhere
    sampler = DeviceDistributedSampler(len(ds), world, rank, seed=args.seed, device=dev)
    B = args.batch_size
    ns = sampler.num_samples
    S = math.ceil(ns / B)
    batches = [(s * B, min(B, ns - s * B)) for s in range(S)]
    idx = torch.zeros(ns, dtype=torch.int32, device=dev)
    losses = torch.zeros(S, device=dev)

    def epochs_fn(n_steps):
        """n_steps from an epoch boundary: sampler at each epoch start, steps, final flush."""
        def fn():
            for g in range(n_steps):
                j = g % S
                if j == 0:
                    sampler.generate(idx)
                st, b = batches[j]
                eng.step(X, Y, idx[st:st + b], b, losses[j:j + 1])
            eng.flush()
        return fn

    m = max(1, round(args.graph_steps / S))
    full = m * S
    warm_steps = math.ceil(max(args.warmup, 1) / S) * S

    def schedule(n):
        out = [full] * (n // full)
        if n % full:
            out.append(n % full)
        return out

    warm, timed = schedule(warm_steps), schedule(args.steps)
    if graph:
        graphs, why = {}, ""
        try:
            for n in sorted(set(warm + timed)):
                graphs[n] = eng.graph(epochs_fn(n), extra_state=(sampler._epoch, losses))
        except Exception as e:  # noqa: BLE001 -- agreed below: every rank leaves the graph path together
            why = f"{type(e).__name__}: {e}"
        dec.check("graph_capture", not why, why)
        # one replay against the same steps run eagerly from the same state (bitwise kernels and the
        # same RCCL reductions: anything but a near-exact match means the graph is not the step)
        saved = [t.clone() for t in eng.state()] + [sampler._epoch.clone(), losses.clone()]
        n0 = timed[0]
        epochs_fn(n0)()
        want = eng.P.clone()
        for t, v in zip(eng.state() + [sampler._epoch, losses], saved):
            t.copy_(v)
        graphs[n0].replay()
        torch.cuda.synchronize(dev)
        got = eng.P.clone()
        for t, v in zip(eng.state() + [sampler._epoch, losses], saved):
            t.copy_(v)
        dec.allclose("graph_replay_check", got, want)
        run = lambda n: graphs[n].replay()  # noqa: E731
    else:
        run = lambda n: epochs_fn(n)()  # noqa: E731
    sampler.set_epoch(0)
    for n in warm:
        run(n)
    # timed region starts on an epoch boundary (warm_steps is a whole number of epochs)
    t = _timed(comm, dev, lambda: [run(n) for n in timed])
    if xg is not None:
        xg.check()
    extra = {"replicas_in_sync": _replicas_in_sync(comm, eng.P),
             "steps_per_epoch": S, "steps_per_graph": full if graph else None, "warmup_steps_run": warm_steps,
             "final_loss": float(losses[(args.steps - 1) % S].item()),
             "allreduce": "xgmi-oneshot (in-kernel)" if xg is not None else "rccl",
             "kernels": ("1 launch per step: fused fwd+loss+bwd+xGMI all-reduce+SGD" if xg is not None
                         else "fused_mlp_step + RCCL all-reduce per step (SGD folded into next step)")
             + (", hipGraph" if graph else ", eager launches")}
    return t, extra


# --------------------------------------------------------------------------- persistent
def run_persistent(args, rank, world, dev, comm, dec):
    """Persistent DDP step engine: K steps in ceil(K/8192) launches, params/momentum/sampler
    shard resident in LDS, in-kernel xGMI all-reduce + SGD every step. Decision points (agreed
    across ranks, utils/fallback.py): device, xgmi_init, xgmi_poll_warmup, xgmi_poll_timed."""
    from pytorch_distributed_training_tutorials_amd.data.device_sampler import DeviceDistributedSampler
    from pytorch_distributed_training_tutorials_amd.ops.fused_step import FusedMLPStep
    from pytorch_distributed_training_tutorials_amd.parallel.xgmi import maybe_create

    dec.check("device", dev.type == "cuda", "the persistent engine needs a GPU")
    model, loss = _build_model(args, dev)
    ds = _dataset(args, dev, loss)
    X, Y = ds.tensors
    xg = None
    if world > 1:
        xg = maybe_create(comm, dev, mode="on")
        dec.check("xgmi_init", xg is not None, "xGMI one-shot all-reduce unavailable (peer memory / self-test)")
    eng = FusedMLPStep(model, loss=loss, lr=args.lr, comm=comm, xgmi=xg, dtype=args.dtype)
    if world > 1:
        comm.broadcast(eng.P, 0)  # DDP init: rank 0's parameters everywhere
    sampler = DeviceDistributedSampler(len(ds), world, rank, seed=args.seed, device=dev)
    variant = args.persist
    pin = _pinned_stream(dev)
    pin_ctx = torch.cuda.stream(pin) if pin is not None else contextlib.nullcontext()
    which = eng.persistent_engine(args.batch_size, sampler, variant)
    S = math.ceil(sampler.num_samples / args.batch_size)
    cursor = torch.zeros(2, dtype=torch.int32, device=dev)
    chunk = 8192
    losses = torch.zeros(min(chunk, max(args.steps, args.warmup, 1)), device=dev)
    launches = [min(chunk, args.steps - d) for d in range(0, args.steps, chunk)]
    n_warm = max(args.warmup, 1)
    if args.sampler == "torch":
        # torch-identical epoch orders: the lists of the epochs a run touches (+1 for the
        # engine's one-position-ahead staging) come from the torch_perm kernel, enqueued
        # right before the engine launch -- inside the timed region for the timed run
        from pytorch_distributed_training_tutorials_amd._ext import native

        C = native()
        n, ns = len(ds), sampler.num_samples

        def order_plan(pos0, steps):
            e_a, e_b = pos0 // S, (pos0 + steps) // S + 1
            seeds = torch.tensor([args.seed + e for e in range(e_a, e_b + 1)], dtype=torch.int64, device=dev)
            buf = torch.empty(e_b - e_a + 1, ns, dtype=torch.int32, device=dev)
            ws = (torch.empty((e_b - e_a + 1) * 4 * n, dtype=torch.int32, device=dev)
                  if C.torch_perm_needs_ws(n) else None)
            pl = eng.persistent_plan(X, Y, args.batch_size, sampler, cursor, losses, variant=variant, idx=buf,
                                     idx_e0=e_a)

            def run():
                C.torch_perm_(seeds, n, world, rank, ns, buf, ws)
                for d in range(0, steps, chunk):
                    pl.launch(min(chunk, steps - d), pos0 + d)
            return run

        order_plan(0, n_warm)()
        timed_steps = order_plan(n_warm, args.steps)
    else:
        # launch planned once (native PersistentPlan): the timed region is hipLaunchKernel(s) + the kernel
        # the bench counts its own steps from cursor 0, so every launch names its start
        # position (launch_at: no dependent cursor load at kernel entry)
        plan = eng.persistent_plan(X, Y, args.batch_size, sampler, cursor, losses, variant=variant)
        # the W warm-up steps: launches through the timed region's own sequence (_untimed) when they
        # fit, so the timed launch below is not the first of its kind in this process
        # (PTDT_BENCH_REHEARSALS: into how many such launches the W steps are split; interleaved A/B at
        # the driver's W = 5: 1 -> 28.2-30.9 us window, 2 -> 25.0-26.1, 3 -> 24.8-26.1 (round 5); round 6,
        # 6 interleaved pairs (profiles/r6_rehearsals_ab.jsonl): 3 -> 23.7-25.2, 5 -> 23.1-26.2 (median 23.7
        # vs 24.6); default 5, i.e. every warm-up step of the driver command its own launch)
        if n_warm <= chunk:
            with pin_ctx:
                _rehearse(comm, dev, plan, n_warm)
        else:
            for d in range(0, n_warm, chunk):
                plan.launch(min(chunk, n_warm - d))
        if os.environ.get("PTDT_BENCH_DEVICE_CURSOR") == "1":  # A/B: start from the device cursor
            launch_at = lambda n, p: plan.launch(n)  # noqa: E731
        else:
            launch_at = plan.launch_at
        starts = [n_warm + d for d in range(0, args.steps, chunk)]

        def timed_steps():
            for n, p in zip(launches, starts):
                launch_at(n, p)
    torch.cuda.synchronize(dev)
    dec.check("xgmi_poll_warmup", not _xgmi_error(xg), "an in-kernel xGMI poll timed out (a peer never arrived)")

    with pin_ctx:
        t = _timed(comm, dev, timed_steps)
    dec.check("xgmi_poll_timed", not _xgmi_error(xg), "an in-kernel xGMI poll timed out (a peer never arrived)")
    in_sync = _replicas_in_sync(comm, eng.P)
    phase = None
    if args.stamps:  # diagnostic pass AFTER the timed region (timers cost a little)
        st = torch.zeros(32, dtype=torch.int64, device=dev)
        if args.sampler == "torch":
            eng.run_persistent(X, Y, args.steps, args.batch_size, sampler, cursor, losses, chunk, stamps=st,
                               variant=variant)
        else:  # the timed path: a plan (list cache warmed by a first pass) launched at known positions
            p2 = eng.persistent_plan(X, Y, args.batch_size, sampler, cursor, losses, variant=variant, stamps=st)
            pos = n_warm + args.steps
            for rep in range(2):
                torch.cuda.synchronize(dev)
                st.zero_()
                for n in launches:
                    p2.launch_at(n, pos)
                    pos += n
            torch.cuda.synchronize(dev)
        v = st.tolist()
        names = (["fetch", "forward", "loss", "backward", "allreduce", "sgd_loss_report"] if which.startswith("wave") else
                 ["helper_wave_staging", "forward", "logits_loss_rows", "barrier2_dz", "backward", "sgd", "allreduce"]
                 if which.startswith("tp") else
                 ["prefetch_issue", "forward", "loss", "backward", "allreduce", "sgd_land", "epoch_indices"])
        clk = v[7] / (v[8] * 10e-9) if v[8] else 0.0
        phase = {"cycles_per_step": {n: round(v[k] / args.steps, 1) for k, n in enumerate(names)},
                 "total_cycles_per_step": round(v[7] / args.steps, 1), "clock_GHz": round(clk / 1e9, 3)}
        if which.startswith("wave"):  # kernel entry -> first step (10 ns ticks), per launch
            nl = math.ceil(args.steps / chunk)
            phase["prologue_us_per_launch"] = round(v[10] * 0.01 / nl, 2)
            # entry -> position known, -> epoch list in LDS, -> past the barrier (waits forced in this pass)
            phase["prologue_split_us"] = [round(v[k] * 0.01 / nl, 2) for k in (11, 12, 13)]
        if which.startswith("tp"):  # each wave's barrier + logit-sum phase (load balance)
            nl = math.ceil(args.steps / chunk)
            # kernel entry -> resident state loaded, -> list e0, -> list e0+1 + keys, -> lists/init done,
            # -> past the barrier, -> step 0 staged (10 ns ticks, per launch; waits forced at each mark)
            phase["prologue_split_us"] = [round(v[k] * 0.01 / nl, 2) for k in (20, 21, 22, 17, 18, 19)]
            nw = int(which.split(":")[1].split("w")[0])
            phase["logits_loss_per_wave"] = [round(x / args.steps, 1) for x in v[9:9 + nw]]
            phase["barrier_wait_per_wave"] = [round(x / args.steps, 1) for x in v[9 + nw:9 + 2 * nw]]
            # the helper wave (staging, sampler lists, loss flush): its work per step, then its waits
            phase["helper_per_step"] = {n: round(v[23 + k] / args.steps, 1) for k, n in enumerate(
                ("other", "barrier1_wait", "barrier2_wait", "produce", "stage_write", "stage_sel_issue", "loss_flush"))}
    last = (args.steps - 1) % chunk
    extra = {"replicas_in_sync": in_sync, "steps_per_epoch": S, "launches_timed": math.ceil(args.steps / chunk),
             "sampler": ("torch.randperm-identical DistributedSampler order (torch_perm kernel in the timed region)"
                         if args.sampler == "torch" else
                         "device Feistel permutation: DistributedSampler semantics (per-epoch reshuffle, padded "
                         "disjoint rank shards) in a different order than torch.randperm; --sampler torch runs "
                         "the torch-identical order"),
             "final_loss": float(losses[last].item()),
             "allreduce": "xgmi-oneshot (in-kernel)" if world > 1 else "identity (world 1)",
             "persistent_engine": which,
             "kernels": ("persistent DDP step engine, single-wave variant: batch/weights/momentum/grads in VGPRs, "
                         "DPP row/column reductions, in-kernel xGMI all-reduce + SGD per step, sampler shard "
                         "rebuilt each epoch by helper waves" if which.startswith("wave") else
                         "persistent DDP step engine: per step gather+fwd+loss+bwd+all-reduce+SGD in one resident "
                         "workgroup; sampler shard recomputed in-kernel each epoch")}
    if phase:
        extra["phase_timers"] = phase
    if args.model == "linear" and not args.no_mlp_side:
        extra.update(_mlp_side(args, rank, world, dev, comm, xg, "fp32", dec))
        extra.update(_mlp_side(args, rank, world, dev, comm, xg, "bf16", dec))
    return t, extra


def _mlp_side(args, rank, world, dev, comm, xg, dtype, dec):
    """Side measurement (AFTER the headline, same protocol, same K/W): the toy MLP
    Linear(20,64)-ReLU-Linear(64,10) + CE + SGD on the persistent engine -- the
    workload BASELINE.json's north star names (config 2: bf16) -- in fp32 (keys mlp_*) and
    on bf16 operands with autocast semantics (keys mlp_bf16_*); reported as extra keys only."""
    from pytorch_distributed_training_tutorials_amd.data.device_sampler import DeviceDistributedSampler
    from pytorch_distributed_training_tutorials_amd.ops.fused_step import FusedMLPStep

    side = argparse.Namespace(**vars(args))
    side.model = "mlp"
    model, loss = _build_model(side, dev)
    ds = _dataset(side, dev, loss)
    X, Y = ds.tensors
    eng = FusedMLPStep(model, loss=loss, lr=args.lr, comm=comm, xgmi=xg, dtype=dtype)
    if world > 1:
        comm.broadcast(eng.P, 0)
    sampler = DeviceDistributedSampler(len(ds), world, rank, seed=args.seed, device=dev)
    cursor = torch.zeros(2, dtype=torch.int32, device=dev)
    n_w, n_t = max(args.warmup, 1), args.steps
    losses = torch.zeros(max(n_w, n_t), device=dev)
    plan = eng.persistent_plan(X, Y, args.batch_size, sampler, cursor, losses)
    _rehearse(comm, dev, plan, n_w)
    key = "mlp" if dtype == "fp32" else "mlp_bf16"
    t = _timed(comm, dev, lambda: plan.launch_at(n_t, n_w), label=f"{key}_side")
    failed = bool(dec.gather("xGMI poll timeout" if _xgmi_error(xg) else None))
    return {f"{key}_us_per_step": None if failed else round(1e6 * t / n_t, 3),
            f"{key}_samples_per_s": None if failed else round(n_t * args.batch_size * world / t, 1),
            f"{key}_dtype": dtype + (" operands (torch.autocast(bfloat16) rounding points), fp32 master weights/SGD"
                                     if dtype == "bf16" else ""),
            f"{key}_engine": eng.persistent_engine(args.batch_size, sampler),
            f"{key}_replicas_in_sync": _replicas_in_sync(comm, eng.P),
            f"{key}_final_loss": float(losses[n_t - 1].item())}


def _xgmi_error(xg) -> bool:
    """This rank's in-kernel xGMI poll-timeout flag (a peer never arrived): the run's numbers are void."""
    return xg is not None and xg.handle.error() != 0


# --------------------------------------------------------------------------- autograd
def run_autograd(args, rank, world, dev, comm, dec):
    dec.check("device", dev.type == "cuda", "the native autograd engine needs a GPU")
    from pytorch_distributed_training_tutorials_amd.data import DeviceDataLoader, DistributedSampler
    from pytorch_distributed_training_tutorials_amd.ops.loss import cross_entropy
    from pytorch_distributed_training_tutorials_amd.ops.optim import FusedSGD
    from pytorch_distributed_training_tutorials_amd.parallel.ddp import DistributedDataParallel

    model, loss = _build_model(args, dev)
    ds = _dataset(args, dev, loss)
    loader = DeviceDataLoader(ds, batch_size=args.batch_size,
                              sampler=DistributedSampler(ds, world, rank, seed=args.seed))
    ddp = DistributedDataParallel(model, device_ids=[dev.index], comm=comm)
    opt = FusedSGD(model.parameters(), lr=args.lr)
    state = {"epoch": 0, "it": None}

    def steps(n):
        for _ in range(n):
            batch = next(state["it"], None) if state["it"] is not None else None
            if batch is None:
                loader.set_epoch(state["epoch"])
                state["epoch"] += 1
                state["it"] = iter(loader)
                batch = next(state["it"])
            xs, ys = batch
            ddp.zero_grad()
            out = ddp(xs)
            l = cross_entropy(out, ys)
            l.backward()
            opt.step()
        return l

    steps(max(args.warmup, 1))
    t = _timed(comm, dev, lambda: steps(args.steps))
    return t, {"kernels": "native DDP reducer + native linear/CE/SGD, eager"}


# --------------------------------------------------------------------------- reference
def run_reference(args, rank, world, dev, comm, dec=None, steps=None, warmup=None, label: str = "headline"):
    """Stock PyTorch-ROCm loop with the reference's structure (comparator):
    reference ddp_gpus_torchrun.py:16-88 with synthetic data of the same shape."""
    import torch.nn.functional as F
    from torch.nn.parallel import DistributedDataParallel as TorchDDP
    from torch.utils.data import DataLoader, TensorDataset
    from torch.utils.data.distributed import DistributedSampler as TorchSampler

    from pytorch_distributed_training_tutorials_amd.utils.faults import FaultInjector

    faults = FaultInjector(rank)
    steps = args.steps if steps is None else steps
    warmup = args.warmup if warmup is None else warmup
    cuda = dev.type == "cuda"

    torch.manual_seed(args.seed)
    g = torch.Generator().manual_seed(args.seed)
    if args.model == "linear":
        ds = TensorDataset(torch.rand(args.dataset_size, 20, generator=g), torch.rand(args.dataset_size, 1, generator=g))
        model = torch.nn.Linear(20, 1).to(dev)
    else:
        ds = TensorDataset(torch.randn(args.dataset_size, 20, generator=g),
                           torch.randint(0, 10, (args.dataset_size,), generator=g))
        model = torch.nn.Sequential(torch.nn.Linear(20, args.hidden), torch.nn.ReLU(),
                                    torch.nn.Linear(args.hidden, 10)).to(dev)
    sampler = TorchSampler(ds, num_replicas=world, rank=rank)
    loader = DataLoader(ds, batch_size=args.batch_size, pin_memory=cuda, shuffle=False, sampler=sampler)
    ddp = TorchDDP(model, device_ids=[dev.index] if cuda else None)
    opt = torch.optim.SGD(model.parameters(), lr=args.lr)
    state = {"epoch": 0, "it": None, "step": 0}

    def run(n):
        for _ in range(n):
            batch = next(state["it"], None) if state["it"] is not None else None
            if batch is None:
                sampler.set_epoch(state["epoch"])
                state["epoch"] += 1
                state["it"] = iter(loader)
                batch = next(state["it"])
            faults.check(state["step"])
            state["step"] += 1
            xs, ys = batch
            xs, ys = xs.to(dev), ys.to(dev)
            opt.zero_grad()
            with torch.autocast(dev.type, dtype=torch.bfloat16, enabled=args.dtype == "bf16"):
                l = F.cross_entropy(ddp(xs), ys)
            l.backward()
            opt.step()

    run(max(warmup, 1))
    t = _timed(comm, dev, lambda: run(steps), label=label)
    return t, {"kernels": "stock torch: DataLoader+DistributedSampler, nn.Linear, F.cross_entropy, torch DDP, SGD"}


# --------------------------------------------------------------------------- timing
def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


_TIMINGS: dict = {}  # label -> start skew / whole-node window of each timed region (reported in the JSON line)
_SPIN: dict = {}


def _spin(comm):
    """The node-local spin barrier for ``comm`` (utils/spin_barrier.py), created once."""
    key = id(comm)
    if key not in _SPIN:
        from pytorch_distributed_training_tutorials_amd.utils import spin_barrier

        _SPIN[key] = spin_barrier.create(comm) if os.environ.get("PTDT_BENCH_SPIN", "1") != "0" else None
    return _SPIN[key]


_GPU_WARM_MS = float(os.environ.get("PTDT_BENCH_GPU_WARM_MS", "0"))
_WARM_BUF: dict = {}


def _gpu_warm(dev, ms: float) -> None:
    """A/B knob (default off): ~``ms`` of HBM streaming right before a timed region (untimed, no
    training work). Measured counter-productive: the fresh-process 20-step window went from 29-30 us
    to 34-37 us with 2 ms of it (profiles/r5_driver_timeline.md) -- what helps is running the
    warm-up steps through the timed region's own sequence (_untimed)."""
    if dev.type != "cuda" or ms <= 0:
        return
    buf = _WARM_BUF.get(dev.index)
    if buf is None:
        buf = _WARM_BUF[dev.index] = torch.zeros(16 << 20, device=dev)  # 64 MiB: ~30 us per pass
    for _ in range(max(1, int(ms * 1000 / 30))):
        buf.add_(1.0)
    torch.cuda.synchronize(dev)


def _pinned_stream(dev):
    """A/B knob PTDT_BENCH_PIN_CU=<cu>: a stream restricted to one CU (hipExtStreamCreateWithCUMask),
    so the single-workgroup engine lands on the same CU -- instruction cache and XCD L2 -- launch after
    launch. None when unset."""
    cu = os.environ.get("PTDT_BENCH_PIN_CU")
    if cu is None or dev.type != "cuda":
        return None
    from pytorch_distributed_training_tutorials_amd._ext import native

    return torch.cuda.ExternalStream(native().cu_masked_stream(dev.index, [int(cu)]), device=dev)


def _untimed(comm, dev, fn) -> None:
    """The timed region's exact sequence (spin barrier resolved, barrier, sync, launch, sync) with
    nothing recorded: the bench runs its warm-up steps through it, so the timed launch is not the
    first of its kind in the process (the first such launch after setup measured 29-30 us for the
    20-step window, the next ones 23-24 us; profiles/r5_driver_timeline.md)."""
    spin = _spin(comm)
    comm.barrier()
    _sync(dev)
    if spin is not None:
        spin.wait()
    fn()
    _sync(dev)


def _rehearse(comm, dev, plan, n_warm: int) -> None:
    """Run exactly ``n_warm`` warm-up steps of a persistent plan (positions 0 .. n_warm-1) as
    PTDT_BENCH_REHEARSALS launches through the timed region's own sequence (_untimed)."""
    reh = max(1, min(n_warm, int(os.environ.get("PTDT_BENCH_REHEARSALS", "5"))))
    p0 = 0
    for r in range(reh):
        k = n_warm // reh + (1 if r < n_warm % reh else 0)
        _untimed(comm, dev, lambda k=k, p0=p0: plan.launch_at(k, p0))
        p0 += k



def _timed(comm, dev, fn, label: str = "headline"):
    """Elapsed seconds of ``fn`` (MAX over ranks): GPU power-state warm-up (untimed, _gpu_warm),
    collective barrier + device sync, then the node-local spin barrier (ranks released within
    ~1-2 us instead of the collective's tens of us), then every rank reads CLOCK_MONOTONIC (one
    clock per node), runs ``fn``, syncs and reads it again. The per-rank stamps are gathered
    afterwards: ``start_skew_us`` = max - min of the start stamps, ``window_us`` = last end - first
    start (the whole-node wall window)."""
    spin = _spin(comm)  # resolved BEFORE the barrier: its first call imports a module (~0.4 ms), and a GPU
    _gpu_warm(dev, _GPU_WARM_MS)  # left idle that long adds ~8-13 us to the next launch
    comm.barrier()
    _sync(dev)
    if spin is not None:
        spin.wait()
    m0 = time.clock_gettime_ns(time.CLOCK_MONOTONIC)
    fn()
    _sync(dev)
    m1 = time.clock_gettime_ns(time.CLOCK_MONOTONIC)  # this rank's work is done
    comm.barrier()
    mine = (m1 - m0) * 1e-9
    if comm.world > 1:
        stamps = comm.all_gather_object((m0, m1))
        t0s, t1s = [a for a, _ in stamps], [b for _, b in stamps]
        el = max((b - a) * 1e-9 for a, b in stamps)
        _TIMINGS[label] = {"start_skew_us": round((max(t0s) - min(t0s)) * 1e-3, 2),
                           "end_skew_us": round((max(t1s) - min(t1s)) * 1e-3, 2),
                           "window_us": round((max(t1s) - min(t0s)) * 1e-3, 2),
                           "per_rank_elapsed_us": [round((b - a) * 1e-3, 2) for a, b in stamps],
                           "release": "spin barrier (/dev/shm)" if spin is not None else "collective barrier"}
        return el
    _TIMINGS[label] = {"start_skew_us": 0.0, "window_us": round(mine * 1e6, 2)}
    return mine


def _record(args, world, value, elapsed, extra):
    gb = args.batch_size * world
    base = BASELINE_SAMPLES_PER_S.get(world)
    ref = extra.get("ref_samples_per_s")
    rec = {
        "metric": METRIC,
        "value": None if value is None else round(value, 1),
        "unit": "samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": None if elapsed is None else round(1e3 * elapsed / args.steps, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(value / ref, 3) if (value and ref) else None,
        "vs_cpu_probe": round(value / base, 3) if (value and base) else None,
        "dtype": args.dtype,
        "data": "synthetic (uniform [0,1) features/targets generated on device, 2048 samples), random-init weights",
        "config": {"model": "ddp_gpus_torchrun toy: Linear(20,1) + F.cross_entropy(soft targets) + SGD(lr=1e-2)"
                   if args.model == "linear" else f"toy MLP Linear(20,{args.hidden})-ReLU-Linear({args.hidden},10) + CE + SGD",
                   "global_batch": gb, "per_device_batch": args.batch_size, "seq_len": None,
                   "dataset_size": args.dataset_size, "parallelism": f"dp{world}",
                   "engine": getattr(args, "engine_used", args.engine)},
        "baseline_note": "vs_baseline = value / ref_samples_per_s: the stock PyTorch-ROCm reference loop (torch DDP "
                         "over RCCL, DataLoader+DistributedSampler, same model/batch/N) timed in this same process "
                         "after the headline; vs_cpu_probe divides by BASELINE.md's CPU/gloo survey probe; the "
                         "reference publishes no GPU DDP number",
        **extra,
    }
    return rec


def _error_line(args, world, phase, elapsed_s, why):
    rec = _record(args, world, None, None, {})
    rec.update({"error": why, "phase": phase, "elapsed_s": round(elapsed_s, 1)})
    return json.dumps(rec)


def _comparator(args, rank, world, dev, comm):
    """The stock PyTorch-ROCm loop at the same N, in this process, after the headline."""
    steps = args.ref_steps or max(args.steps, 256)
    warm = max(args.warmup, 32)
    t, _ = run_reference(args, rank, world, dev, comm, steps=steps, warmup=warm, label="comparator")
    sps = steps * args.batch_size * world / t
    return {"ref_samples_per_s": round(sps, 1), "ref_ms_per_step": round(1e3 * t / steps, 4), "ref_steps": steps,
            "ref_warmup": warm, "ref_engine": "stock torch DDP (RCCL) + DataLoader/DistributedSampler + nn.Linear + "
                                              "F.cross_entropy + torch.optim.SGD, same process"}


# engine chains: what is tried after the requested engine fails on any rank (utils/fallback.py)
CHAINS = {"persistent": ["persistent", "fused_graph", "fused_eager", "autograd", "reference"],
          "fused": ["fused_graph", "fused_eager", "autograd", "reference"],
          "autograd": ["autograd", "reference"], "reference": ["reference"]}


def _chain(args):
    names = CHAINS[args.engine]
    if args.dtype == "bf16":  # the bf16 engine is the persistent one; last resort: autocast(bf16) stock loop
        names = [n for n in names if n in ("persistent", "reference")]
    if args.share_gpu:  # RCCL needs one GPU per rank: the host-staged engines only
        names = [n for n in names if n in ("persistent", "fused_graph", "fused_eager")]
    return names[:1] if args.no_fallback else names


def main(argv=None):
    args = parse(argv)
    if args.dtype == "bf16" and args.model != "mlp":
        raise SystemExit("--dtype bf16 runs the toy MLP (--model mlp); the reference Linear(20,1) job is fp32")
    if args.dtype == "bf16" and args.engine not in ("persistent", "reference"):
        raise SystemExit("--dtype bf16 runs on the persistent engine (the bf16 tensor-parallel kernel)")
    cpu = args.device == "cpu" or (args.device == "auto" and not torch.cuda.is_available())
    if cpu and args.no_fallback and args.engine != "reference":
        raise SystemExit("bench.py needs a GPU (MI355X) for the framework engines; --device cpu runs "
                         "--engine reference (or the engine chain down to it)")
    os.environ.setdefault("PTDT_COMM_TIMEOUT", "120")  # a hung collective aborts well inside --deadline
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    rank_env = int(os.environ.get("RANK", "0"))
    from pytorch_distributed_training_tutorials_amd.utils.deadline import Deadline
    from pytorch_distributed_training_tutorials_amd.utils.fallback import (Decider, DesyncError, StageFailed,
                                                                      control_group, run_chain)

    done = {}  # the headline record once measured: a later phase that hangs still reports it

    def expire(phase, elapsed):
        why = f"deadline of {args.deadline:.0f} s expired"
        if rank_env == 0:  # own line even if another process left a partial one on the shared stdout
            if "rec" in done:
                rec = dict(done["rec"], incomplete=f"{why} in phase {phase!r}, after the headline was measured")
                print("\n" + json.dumps(rec), flush=True)
            else:
                print("\n" + _error_line(args, world_env, phase, elapsed, why), flush=True)
        print(f"[bench] rank {rank_env}: {why} in phase {phase!r}; aborting communicators and exiting",
              file=sys.stderr, flush=True)

    dl = Deadline(args.deadline, expire, exit_delay_s=0.0 if rank_env == 0 else 5.0)
    dl.set_phase("process group init")
    rank, world, local = _setup(args, cpu)
    dec = Decider(rank, world, control_group(world))
    dev = torch.device("cpu") if cpu else torch.device("cuda", 0 if args.share_gpu else local)
    from pytorch_distributed_training_tutorials_amd.parallel import comm as comm_mod
    from pytorch_distributed_training_tutorials_amd.parallel.env import destroy_process_group

    dl.set_phase("communicator init")
    if args.share_gpu:
        if args.engine not in ("persistent", "fused") or args.allreduce == "rccl":
            raise SystemExit("--share_gpu rehearses the xGMI engines only (RCCL needs one GPU per rank)")
        torch.cuda.set_device(dev)
        comm = comm_mod.HostStagedComm(dev)
    else:
        comm = comm_mod.get_default(dev)
        dl.register(getattr(comm, "handle", None))
    names = _chain(args)

    def stage(name):
        # a fused stage reached by falling back runs the RCCL all-reduce (the xGMI path already failed)
        ar = None if name == names[0] else "rccl"
        fns = {"persistent": lambda d: run_persistent(args, rank, world, dev, comm, d),
               "fused_graph": lambda d: run_fused(args, rank, world, dev, comm, d, graph=True, allreduce=ar),
               "fused_eager": lambda d: run_fused(args, rank, world, dev, comm, d, graph=False, allreduce=ar),
               "autograd": lambda d: run_autograd(args, rank, world, dev, comm, d),
               "reference": lambda d: run_reference(args, rank, world, dev, comm, d)}
        return fns[name]

    dl.set_phase(f"headline ({args.engine} engine: build, warmup, timed run)")
    try:
        used, (elapsed, extra), failures = run_chain(dec, [(n, stage(n)) for n in names])
    except (StageFailed, DesyncError) as e:
        if rank == 0:
            what = "every engine failed" if isinstance(e, StageFailed) else "fallback chain desynchronised"
            print("\n" + _error_line(args, world, "headline", time.monotonic() - dl.t0, f"{what}: {e}"), flush=True)
        destroy_process_group()
        dl.cancel()
        sys.exit(4)
    args.engine_used = used
    extra["engine_path"] = used
    if failures:
        extra["fallback"] = failures
    value = args.steps * args.batch_size * world / elapsed
    extra["timing"] = dict(_TIMINGS)
    done["rec"] = _record(args, world, value, elapsed, extra)
    if not (args.no_ref or args.share_gpu or used == "reference"):
        dl.set_phase("comparator (stock PyTorch-ROCm reference loop)")
        cmp, why = {}, None
        try:
            cmp = _comparator(args, rank, world, dev, comm)
        except Exception as e:  # noqa: BLE001 -- the headline stands; agreed so every rank reports alike
            why = f"{type(e).__name__}: {e}"
        bad = dec.gather(why)
        if bad:
            extra["comparator_error"] = {str(r): w[:400] for r, w in bad.items()}
        else:
            extra.update(cmp)
            extra["speedup_vs_torch"] = round(value / extra["ref_samples_per_s"], 3)
    dl.set_phase("report")
    extra["timing"] = dict(_TIMINGS)
    extra["gpu_warmup_ms_before_timed"] = _GPU_WARM_MS if dev.type == "cuda" else 0.0
    rec = _record(args, world, value, elapsed, extra)
    if args.share_gpu:
        rec["rehearsal"] = f"{world} ranks sharing cuda:0 (no xGMI hop): protocol/correctness check, not a scaling number"
    if cpu:
        rec["device"] = "cpu (gloo): plumbing run of the reference loop, not an MI355X number"
    if rank == 0:
        line = json.dumps(rec)
        print("\n" + line, flush=True)  # starts a line even after another rank's partial output
        if args.out:
            with open(args.out, "a") as f:
                f.write(line + "\n")
    dl.set_phase("teardown")
    destroy_process_group()
    dl.cancel()


if __name__ == "__main__":
    main(sys.argv[1:])
