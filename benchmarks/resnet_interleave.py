#!/usr/bin/env python3
"""Eager / hipGraph-replay interleaving check for the native ResNet-50 DDP step.

``benchmarks/resnet_ddp.py --graph auto`` warms up, captures one graph, then alternates
blocks of eager steps and graph replays before the timed loop. This script runs that
pattern (and any other, e.g. ``--pattern EERR``) from one init, next to a pure-eager run of
the same number of EXECUTED steps (the capture call itself executes nothing), and prints
per-step losses plus the largest parameter difference between the two trajectories.

    python benchmarks/resnet_interleave.py --deterministic --pattern EEEERRRR --repeat 3

One JSON line per run. ``--sync`` synchronises the device after every step (removes any
host/device overlap from the picture).
"""
from __future__ import annotations

import argparse
import copy
import json
import os
import sys
import time

import torch

T0 = time.time()

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--warmup", type=int, default=5, help="GraphedStep eager warm-up steps")
    ap.add_argument("--pattern", default="EEEERRRR", help="E = eager step, R = graph replay")
    ap.add_argument("--repeat", type=int, default=3)
    ap.add_argument("--tail", type=int, default=0, help="graph replays after the pattern")
    ap.add_argument("--deterministic", action="store_true")
    ap.add_argument("--sync", action="store_true")
    ap.add_argument("--variants", default="eager,interleave")
    ap.add_argument("--no_shadow", action="store_true", help="FusedSGD without bf16 weight shadows")
    a = ap.parse_args(argv)
    torch.backends.cudnn.benchmark = not a.deterministic
    torch.backends.cudnn.deterministic = a.deterministic
    from pytorch_distributed_training_tutorials_amd import native
    from pytorch_distributed_training_tutorials_amd.models.resnet import resnet50
    from pytorch_distributed_training_tutorials_amd.ops.loss import cross_entropy
    from pytorch_distributed_training_tutorials_amd.ops.optim import FusedSGD
    from pytorch_distributed_training_tutorials_amd.parallel import comm as comm_mod
    from pytorch_distributed_training_tutorials_amd.parallel import env
    from pytorch_distributed_training_tutorials_amd.parallel.ddp import DistributedDataParallel
    from pytorch_distributed_training_tutorials_amd.utils.graphs import GraphedStep

    env.init_process_group("nccl")
    dev = env.device()
    comm = comm_mod.get_default(dev)
    torch.manual_seed(0)
    base = resnet50(num_classes=1000).to(dev).to(memory_format=torch.channels_last)
    x = torch.empty(a.batch, 3, a.image, a.image, device=dev)
    native().philox_(x, 1234, 0, 1)
    x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (a.batch,), device=dev, generator=torch.Generator(device=dev).manual_seed(5))
    seq = a.pattern * a.repeat + "R" * a.tail
    n_exec = a.warmup + len(seq)
    results, captures = {}, {}
    for variant in a.variants.split(","):
        model = copy.deepcopy(base)
        ddp = DistributedDataParallel(model, device_ids=[dev.index], comm=comm)
        opt = FusedSGD(model.parameters(), lr=a.lr, momentum=0.9, weight_decay=1e-4, bf16_shadow=not a.no_shadow)
        graphed = variant != "eager"
        losses = []

        def step(ddp=ddp, opt=opt, graphed=graphed):
            ddp.zero_grad()
            with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=not graphed):
                out = ddp(x)
            loss = cross_entropy(out.float(), y)
            loss.backward()
            opt.step()
            return loss

        def rec(fn, variant=variant):
            v = fn()
            if torch.cuda.is_current_stream_capturing():  # a (re-)capture executes nothing
                return v
            losses.append(v.detach().clone())
            if a.sync and not torch.cuda.is_current_stream_capturing():
                torch.cuda.synchronize(dev)
            print(f"[{time.time() - T0:7.1f}s] {variant} step {len(losses)}", file=sys.stderr, flush=True)
            return v

        if variant == "eager":
            for _ in range(n_exec):
                rec(step)
        else:
            gs = GraphedStep(lambda: rec(step), dev, comm=comm, warmup=a.warmup)
            # interleave: the pattern with GraphedStep.eager (re-captures before the next replay);
            # interleave_raw: eager steps by calling the step function directly (the round-3 bench's
            # hazard); graph: replays only; eager_after_capture: eager only
            for c in seq:
                if variant == "eager_after_capture" or (variant == "interleave_raw" and c == "E"):
                    rec(step)
                elif variant == "interleave" and c == "E":
                    gs.eager()  # runs rec(step) (GraphedStep's fn): recorded there
                else:
                    rec(gs)
        torch.cuda.synchronize(dev)
        if variant != "eager":
            captures[variant] = gs.captures
        results[variant] = ([float(v) for v in losses],
                            {k: v.detach().float().clone() for k, v in model.state_dict().items()})
        del ddp, opt, model
    ref_l, ref_s = results[a.variants.split(",")[0]]
    for variant, (ls, st) in results.items():
        dmax, dkey = 0.0, None
        for k, v in st.items():
            d = float((v - ref_s[k]).abs().max()) if v.numel() else 0.0
            if d > dmax or dkey is None:
                dmax, dkey = d, k
        first_diff = next((i for i, (p, q) in enumerate(zip(ls, ref_l)) if abs(p - q) > 1e-3 * max(1, abs(q))), None)
        print(json.dumps({"variant": variant, "pattern": seq, "warmup": a.warmup, "executed_steps": len(ls),
                          "lr": a.lr, "batch": a.batch, "image": a.image, "deterministic": a.deterministic,
                          "sync": a.sync, "shadow": not a.no_shadow, "finite": all(v == v and abs(v) < float("inf") for v in ls),
                          "final_loss": round(ls[-1], 4), "first_loss_divergence_step": first_diff,
                          "max_param_diff_vs_first_variant": dmax, "worst_param": dkey,
                          "env": {k: v for k, v in os.environ.items() if k.startswith("PTDT_")},
                          "captures": captures.get(variant), "losses": [round(v, 4) for v in ls]}), flush=True)
    env.destroy_process_group()


if __name__ == "__main__":
    main()
