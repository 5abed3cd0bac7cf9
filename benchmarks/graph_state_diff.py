#!/usr/bin/env python3
"""Which state does a hipGraph replay get wrong after eager steps? (diagnostic)

Warm up + capture a native ResNet-50 DDP step (utils/graphs.py), run ``--eager`` eager
steps, snapshot every piece of training state (parameters, buffers incl. BN tickets,
momentum buffers, bf16 shadows, optimizer counters, gradient buckets), run ONE eager step
and record the state, restore the snapshot in place, run ONE replay, and print the
tensors whose post-step values differ most between the two.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--image", type=int, default=128)
    ap.add_argument("--eager", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--top", type=int, default=12)
    ap.add_argument("--nondet", action="store_true", help="cudnn.benchmark instead of deterministic MIOpen")
    ap.add_argument("--replays", type=int, default=0,
                    help="replay-first mode: right after the capture, K replays from a snapshot, then (restored) "
                         "K eager steps; per-step losses and the state diff after K (no eager step precedes a replay)")
    a = ap.parse_args(argv)
    torch.backends.cudnn.benchmark = a.nondet
    torch.backends.cudnn.deterministic = not a.nondet
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
    model = resnet50(num_classes=1000).to(dev).to(memory_format=torch.channels_last)
    x = torch.empty(a.batch, 3, a.image, a.image, device=dev)
    native().philox_(x, 1234, 0, 1)
    x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (a.batch,), device=dev, generator=torch.Generator(device=dev).manual_seed(5))
    ddp = DistributedDataParallel(model, device_ids=[dev.index], comm=comm)
    opt = FusedSGD(model.parameters(), lr=a.lr, momentum=0.9, weight_decay=1e-4, bf16_shadow=True)

    def step():
        ddp.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
            out = ddp(x)
        loss = cross_entropy(out.float(), y)
        loss.backward()
        opt.step()
        return loss

    gs = GraphedStep(step, dev, comm=comm, warmup=a.warmup)
    if a.replays == 0:
        for _ in range(a.eager):
            step()
    torch.cuda.synchronize(dev)

    def state():
        out = {}
        for n, t in model.named_parameters():
            out["param:" + n] = t.data
            sh = getattr(t, "_ptdt_bf16", None)
            if sh is not None:
                out["shadow:" + n] = sh
            st = opt.state.get(t, {})
            if "momentum_buffer" in st:
                out["mom:" + n] = st["momentum_buffer"]
        for n, b in model.named_buffers():
            out["buf:" + n] = b
        for k, c in opt._counters.items():
            out[f"counter:{k}"] = c
        for i, b in enumerate(ddp.reducer.bucket_tensors()):
            out[f"bucket:{i}"] = b
        return out

    live = state()
    snap = {k: v.detach().clone() for k, v in live.items()}

    def restore():
        with torch.no_grad():
            for k, v in live.items():
                v.copy_(snap[k])
        torch.cuda.synchronize(dev)

    if a.replays > 0:
        lr_list = [float(gs()) for _ in range(a.replays)]
        torch.cuda.synchronize(dev)
        after_r = {k: v.detach().clone() for k, v in live.items()}
        restore()
        le_list = [float(step()) for _ in range(a.replays)]
        torch.cuda.synchronize(dev)
        after_e = {k: v.detach().clone() for k, v in live.items()}
        out = []
        for k in after_e:
            d = (after_e[k].double() - after_r[k].double()).abs()
            m = float(d.max()) if d.numel() else 0.0
            out.append((m if m == m else float("inf"), k))
        out.sort(reverse=True)
        nan_r = [k for k, v in after_r.items() if v.is_floating_point() and not bool(torch.isfinite(v).all())]
        print(json.dumps({"mode": "replay_first", "replays": a.replays, "losses_replay": lr_list,
                          "losses_eager": le_list, "replay_vs_eager_top": out[:a.top],
                          "n_tensors_differing": sum(1 for m, _ in out if m > 0), "nonfinite_after_replay": nan_r[:40]}),
              flush=True)
        env.destroy_process_group()
        return
    le = float(step())
    torch.cuda.synchronize(dev)
    after_e = {k: v.detach().clone() for k, v in live.items()}
    restore()
    lr_ = float(gs())
    torch.cuda.synchronize(dev)
    after_r = {k: v.detach().clone() for k, v in live.items()}
    restore()
    le2 = float(step())  # eager again from the same snapshot: the run-to-run floor
    torch.cuda.synchronize(dev)
    after_e2 = {k: v.detach().clone() for k, v in live.items()}

    def diffs(A, B):
        out = []
        for k in A:
            d = (A[k].double() - B[k].double()).abs()
            m = float(d.max()) if d.numel() else 0.0
            ref = float(A[k].double().abs().max()) if A[k].numel() else 0.0
            out.append((m, ref, k))
        out.sort(reverse=True)
        return out

    dr = diffs(after_e, after_r)
    de = diffs(after_e, after_e2)
    nan_r = [k for k, v in after_r.items() if v.is_floating_point() and not bool(torch.isfinite(v).all())]
    nan_e = [k for k, v in after_e.items() if v.is_floating_point() and not bool(torch.isfinite(v).all())]
    dr = [t for t in dr if t[0] == t[0]]
    print(json.dumps({"eager_steps_before": a.eager, "loss_eager": le, "loss_replay": lr_, "loss_eager_again": le2,
                      "replay_vs_eager_top": [(k, m, r) for m, r, k in dr[:a.top]],
                      "eager_vs_eager_top": [(k, m, r) for m, r, k in de[:4]],
                      "n_tensors_differing": sum(1 for m, _, _ in dr if m > 0),
                      "nonfinite_after_replay": nan_r, "nonfinite_after_eager": nan_e}), flush=True)
    env.destroy_process_group()


if __name__ == "__main__":
    main()
