#!/usr/bin/env python3
"""ResNet-50 DDP stress benchmark (BASELINE.json config 5).

Synthetic ImageNet-shaped data (generated on the GPU), torchvision-layout ResNet-50,
native DDP reducer: gradients are bucket views, buckets all-reduced with RCCL
(ncclAvg) on a high-priority comm stream overlapped with backward, bucket caps
sized for xGMI (parallel/bucketing.py) and rebuilt in gradient-ready order
after iteration 0. Compute: bf16 autocast + channels_last (MIOpen NHWC conv
solvers) by default, fp32 master weights, fused SGD (momentum) on flat spans.

  python benchmarks/resnet_ddp.py --steps 30 --warmup 5                       # 1 GPU
  python -m torch.distributed.run --nproc-per-node 8 benchmarks/resnet_ddp.py  # 8 GPUs

Prints one JSON line (rank 0): images/s over the whole job, ms/step, bucket layout.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _choices():
    from pytorch_distributed_training_tutorials_amd.utils import tuning

    return tuning.choices()


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--batch_size", type=int, default=128, help="per-GPU batch")
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no_channels_last", action="store_true")
    ap.add_argument("--bucket_cap_mb", type=float, default=None)
    ap.add_argument("--impl", default="native", choices=["native", "torch"],
                    help="native DDP reducer + fused optimizer, or stock torch DDP + torch.optim.SGD (comparator)")
    ap.add_argument("--no_shadow", action="store_true",
                    help="cast the fp32 weights in every forward instead of using FusedSGD's bf16 shadows")
    ap.add_argument("--tag", default=None, help="free-form label copied into the JSON line")
    ap.add_argument("--deterministic", action="store_true",
                    help="diagnostic: deterministic MIOpen solvers (cudnn.deterministic, no exhaustive find)")
    ap.add_argument("--loss_curve", action="store_true",
                    help="diagnostic: record every executed step's loss (one clone per step) into the JSON line")
    ap.add_argument("--graph", default="auto", choices=["auto", "on", "off"],
                    help="native impl: replay one captured hipGraph per step (on), launch eagerly (off), or time "
                         "both in this process after warm-up and keep the faster (auto: the eager loop's cost "
                         "depends on the host, the graph's does not)")
    ap.add_argument("--no_graph", action="store_true", help="= --graph off")
    ap.add_argument("--pre_steps", type=int, default=None,
                    help="untimed training steps before --warmup (default: torch impl runs as many as the native "
                         "--graph auto path does before its warm-up, so both report the loss after the same number "
                         "of steps)")
    ap.add_argument("--no_cudnn_benchmark", action="store_true",
                    help="keep MIOpen's heuristic solver choice (default: exhaustive find per conv shape)")
    a = ap.parse_args(argv)
    torch.backends.cudnn.benchmark = not a.no_cudnn_benchmark and not a.deterministic
    torch.backends.cudnn.deterministic = a.deterministic

    from pytorch_distributed_training_tutorials_amd import native
    from pytorch_distributed_training_tutorials_amd.models.resnet import resnet50
    from pytorch_distributed_training_tutorials_amd.ops.loss import cross_entropy
    from pytorch_distributed_training_tutorials_amd.ops.optim import FusedSGD
    from pytorch_distributed_training_tutorials_amd.parallel import comm as comm_mod
    from pytorch_distributed_training_tutorials_amd.parallel import env
    from pytorch_distributed_training_tutorials_amd.parallel.ddp import DistributedDataParallel

    env.init_process_group("nccl")
    rank, world = env.rank(), env.world_size()
    dev = env.device()
    comm = comm_mod.get_default(dev)
    torch.manual_seed(0)
    model = resnet50(num_classes=1000).to(dev)
    if not a.no_channels_last:
        model = model.to(memory_format=torch.channels_last)
    if a.impl == "native":
        ddp = DistributedDataParallel(model, device_ids=[dev.index], comm=comm, bucket_cap_mb=a.bucket_cap_mb)
        opt = FusedSGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4,
                       bf16_shadow=a.dtype == "bf16" and not a.no_shadow)
    else:
        from torch.nn.parallel import DistributedDataParallel as TorchDDP

        ddp = TorchDDP(model, device_ids=[dev.index], bucket_cap_mb=a.bucket_cap_mb or 25)
        opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    x = torch.empty(a.batch_size, 3, a.image, a.image, device=dev)
    native().philox_(x, 1234 + rank, 0, 1)
    if not a.no_channels_last:
        x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (a.batch_size,), device=dev)
    amp = a.dtype == "bf16"
    mode = "off" if (a.no_graph or a.impl != "native") else a.graph
    if mode == "auto" and world > 1 and os.environ.get("PTDT_GRAPH_MULTI", "0") != "1":
        # RCCL collectives captured in a replayed step have only run at world 1 (RCCL refuses two
        # ranks on one GPU, so no one-GPU rehearsal exists): the default stays eager across GPUs;
        # --graph on or PTDT_GRAPH_MULTI=1 opts in
        mode = "off"
    graphed = mode != "off"
    from pytorch_distributed_training_tutorials_amd.utils.graphs import GraphedStep

    def step():
        if a.impl == "native":
            ddp.zero_grad()
        else:
            opt.zero_grad()
        # no autocast weight cache under capture (the cast kernels must be in the graph)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp, cache_enabled=not graphed):
            out = ddp(x)
        loss = cross_entropy(out.float(), y)
        loss.backward()
        opt.step()
        if a.loss_curve and not torch.cuda.is_current_stream_capturing():
            curve.append(loss.detach().clone())
        return loss

    curve = []

    def replayed(fn):  # loss of a graph replay (the captured step's Python body does not run)
        def run():
            loss = fn()
            if a.loss_curve and isinstance(fn, GraphedStep):
                curve.append(loss.detach().clone())
            return loss
        return run

    ab = None
    graph_info = None
    executed = 0  # training steps run before the timed loop's warm-up (the comparator runs as many)
    if graphed:  # utils/graphs.py: eager warm-up steps on a side stream, then one hipGraph per step
        eager = step
        if mode == "auto":
            # eager rounds FIRST, then capture and replay rounds. (The captured step's memset nodes,
            # which the runtime executes only partially from a graph's second launch on, are
            # rewritten as fill kernels by GraphedStep: profiles/r5_graph_memset.md)
            ab = {"eager": [], "graph": []}
            for _ in range(max(3, a.warmup)):
                eager()
            executed += max(3, a.warmup)

            def rounds(name, fn):
                nonlocal executed
                for _ in range(3):
                    comm.barrier()
                    torch.cuda.synchronize(dev)
                    t0 = time.perf_counter()
                    for _ in range(4):
                        replayed(fn)()
                    torch.cuda.synchronize(dev)
                    ab[name].append((time.perf_counter() - t0) / 4 * 1e3)
                    executed += 4

            rounds("eager", eager)
        gstep = GraphedStep(eager, dev, comm=comm, warmup=max(3, a.warmup))
        graph_info = {"nodes": gstep.node_count, "memset_nodes": gstep.memset_nodes,
                      "memsets_replaced": gstep.memsets_replaced}
        executed += max(3, a.warmup)
        step = gstep
        if mode == "auto":
            rounds("graph", gstep)
            med = {k: sorted(v)[1] for k, v in ab.items()}
            win = "graph" if med["graph"] <= med["eager"] else "eager"
            if world > 1:  # every rank must take the same path (the graph holds collectives)
                flag = torch.tensor([1.0 if win == "graph" else 0.0], device=dev)
                comm.all_reduce(flag, "min")
                win = "graph" if float(flag.item()) == 1.0 else "eager"
            graphed = win == "graph"
            step = gstep if graphed else gstep.eager
            ab = {k: round(v, 3) for k, v in med.items()}
    step = replayed(step)
    for _ in range(a.pre_steps if a.pre_steps is not None else (2 * max(3, a.warmup) + 24 if a.impl == "torch" else 0)):
        # comparator: as many steps before the timed region as the native default mode runs
        # (eager warm-up + 3 x 4 eager steps, GraphedStep warm-up + 3 x 4 replays: 2 max(3, warmup) + 24)
        step()
        executed += 1
    for _ in range(a.warmup):
        step()
    executed += a.warmup
    comm.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize(dev)
    comm.barrier()
    el = torch.tensor([time.perf_counter() - t0], device=dev, dtype=torch.float64)
    if world > 1:
        comm.all_reduce(el, "max")
    el = float(el.item())
    final = float(loss.detach())
    finite = final == final and abs(final) != float("inf")
    if world > 1:  # every replica must be finite
        f = torch.tensor([1.0 if finite else 0.0], device=dev)
        comm.all_reduce(f, "min")
        finite = bool(f.item() == 1.0)
    if rank == 0 and not finite:
        print(json.dumps({"metric": "ResNet-50 DDP training throughput (whole node)", "value": None,
                          "error": f"non-finite training loss {final} after {executed + a.steps} steps: no throughput "
                                   "is reported for a diverged run", "finite": False, "impl": a.impl,
                          "graph_mode": mode, **({"tag": a.tag} if a.tag else {})}), flush=True)
    elif rank == 0:
        print(json.dumps({
            "metric": "ResNet-50 DDP training throughput (whole node)", "value": round(a.steps * a.batch_size * world / el, 1),
            "unit": "images/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(1e3 * el / a.steps, 3), "higher_is_better": True, "scaling": "weak",
            "dtype": a.dtype, "data": "synthetic ImageNet-shaped (generated on device)",
            "config": {"model": "resnet50", "per_device_batch": a.batch_size, "image": a.image,
                       "parallelism": f"dp{world}", "channels_last": not a.no_channels_last},
            "impl": a.impl, "hipgraph": graphed, "graph_mode": mode, **({"ab_ms_per_step": ab} if ab else {}), "bn_dir": os.environ.get("PTDT_BN_DIR", "0"), "miopen_find": "exhaustive (cudnn.benchmark)" if torch.backends.cudnn.benchmark else "heuristic",
            "buckets_MB": [round(b / 2 ** 20, 2) for b in ddp.bucket_sizes_bytes()] if a.impl == "native" else None,
            **({"loss_curve": [round(float(v), 4) for v in curve]} if a.loss_curve else {}),
            **({"graph": graph_info} if graph_info else {}),
            "final_loss": final, "finite": True, "kernel_choices": _choices(), "steps_total": executed + a.steps, **({"tag": a.tag} if a.tag else {}),
        }), flush=True)
    env.destroy_process_group()


if __name__ == "__main__":
    main()
