#!/usr/bin/env python3
"""Root cause of the ResNet-50 graph-replay divergence: what do the
memset nodes of a captured exhaustive-find step look like, and does the runtime's
memset-node path execute them correctly?

1. Capture a native ResNet-50 DDP step (cudnn.benchmark=True: MIOpen's atomic
   weight-gradient solvers zero their outputs with hipMemsetAsync) and dump every
   memset node's parameters (hipGraphMemsetNodeGetParams: dst, value, elementSize,
   width, height, pitch) -- one JSON line ("nodes").
2. Replay each memset node ALONE (a fresh graph holding one memset node with the same
   parameters, over a scratch buffer pre-filled with 0xAB) and count the bytes the
   node should have set but did not -- before and after eager hipMemsetAsync calls of
   other sizes ("isolated").
3. The same captured graph with and without the fill-kernel rewrite, replayed
   ``--replays`` times from one snapshot vs the same number of eager steps: the
   per-step loss gap and the largest parameter gap ("trajectory").
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _span(esize, width, height, pitch):
    rows = max(1, height)
    p = pitch if pitch > 0 else width * esize
    return (rows - 1) * p + width * esize, rows, p


def isolated(native, dev, params, dirty: bool):
    out = []
    for dst, value, esize, width, height, pitch in params:
        span, rows, p = _span(esize, width, height, pitch)
        buf = torch.full((span + 64,), 0xAB, dtype=torch.uint8, device=dev)
        if dirty:  # eager memsets of other sizes first (the r3/r4 trigger hypothesis)
            for n in (4096, 1000, 3 * 4096 + 7):
                native.memset_async_(torch.empty(n, dtype=torch.uint8, device=dev), 0x11)
        native.graph_memset_run(buf, value, esize, width, height, pitch, 2)
        torch.cuda.synchronize(dev)
        want = torch.tensor([value & 0xFF, (value >> 8) & 0xFF, (value >> 16) & 0xFF, (value >> 24) & 0xFF],
                            dtype=torch.uint8, device=dev)[:esize].repeat(width)
        bad = 0
        for r in range(rows):
            got = buf[r * p: r * p + width * esize]
            bad += int((got != want).sum())
        tail = int((buf[span:] != 0xAB).sum())  # bytes written past the memset
        out.append({"bytes": width * esize * rows, "esize": esize, "width": width, "height": height, "pitch": pitch,
                    "dst_align": dst % 256, "unset_bytes": bad, "overrun_bytes": tail})
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--image", type=int, default=128)
    ap.add_argument("--replays", type=int, default=4)
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--out", default=None)
    ap.add_argument("--synthetic", action="store_true",
                    help="the captured step's memset parameters (sizes, value, dst alignment mod 4 KiB) as "
                         "hipMemsetAsync calls captured alone into one torch graph, plus a memset of another "
                         "value; replayed with eager memsets / fills in between; counts unzeroed bytes per replay")
    ap.add_argument("--trace_only", action="store_true",
                    help="capture WITHOUT the rewrite and replay twice, each replay bracketed by philox_kernel "
                         "markers, nothing else: run under rocprofv3 --kernel-trace and read the replays' dispatch "
                         "order / queues with tools/graph_replay_order.py")
    a = ap.parse_args(argv)
    torch.backends.cudnn.benchmark, torch.backends.cudnn.deterministic = True, False
    from pytorch_distributed_training_tutorials_amd import native as _native
    from pytorch_distributed_training_tutorials_amd.models.resnet import resnet50
    from pytorch_distributed_training_tutorials_amd.ops.loss import cross_entropy
    from pytorch_distributed_training_tutorials_amd.ops.optim import FusedSGD
    from pytorch_distributed_training_tutorials_amd.parallel import comm as comm_mod
    from pytorch_distributed_training_tutorials_amd.parallel import env
    from pytorch_distributed_training_tutorials_amd.parallel.ddp import DistributedDataParallel
    from pytorch_distributed_training_tutorials_amd.utils import graphs

    native = _native()
    env.init_process_group("nccl")
    dev = env.device()
    comm = comm_mod.get_default(dev)
    lines = []

    def emit(d):
        s = json.dumps(d)
        print(s, flush=True)
        lines.append(s)

    def build():
        torch.manual_seed(0)
        model = resnet50(num_classes=1000).to(dev).to(memory_format=torch.channels_last)
        ddp = DistributedDataParallel(model, device_ids=[dev.index], comm=comm)
        opt = FusedSGD(model.parameters(), lr=a.lr, momentum=0.9, weight_decay=1e-4, bf16_shadow=True)
        return model, ddp, opt

    x = torch.empty(a.batch, 3, a.image, a.image, device=dev)
    native.philox_(x, 1234, 0, 1)
    x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (a.batch,), device=dev, generator=torch.Generator(device=dev).manual_seed(5))

    results = {}
    if a.synthetic:
        params = [(0, 1, 131072, 3584)] * 4 + [(0, 1, 131072, 0)] * 3 + [(0, 1, 65536, 0), (0, 1, 32768, 3584),
                                                                        (0, 1, 32768, 3584), (0, 1, 8192, 3584)]
        bufs, views = [], []
        for value, esize, width, align in params:
            b = torch.empty(width + 8192, dtype=torch.uint8, device=dev)
            off = (align - b.data_ptr()) % 4096
            bufs.append(b)
            views.append(b[off:off + width])
        other = torch.empty(3 * 4096 + 100, dtype=torch.uint8, device=dev)
        side = torch.cuda.Stream(dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=side):
            for v in views:
                native.memset_async_(v, 0)
            native.memset_async_(other, 0x3F)  # a memset of another value in the same graph
        for mode in ("plain", "eager_memsets_between", "eager_fills_between"):
            bad = []
            for rep in range(4):
                for v in views:
                    v.fill_(0xAB)
                if mode == "eager_memsets_between":
                    for n in (4096, 1000, 3 * 4096 + 7, 131072):
                        native.memset_async_(torch.empty(n, dtype=torch.uint8, device=dev), 0x11)
                elif mode == "eager_fills_between":
                    torch.empty(1 << 20, device=dev).fill_(1.0)
                torch.cuda.synchronize(dev)
                g.replay()
                torch.cuda.synchronize(dev)
                bad.append([int((v != 0).sum()) for v in views] + [int((other != 0x3F).sum())])
            emit({"what": "synthetic", "mode": mode, "unset_bytes_per_replay": bad})
        env.destroy_process_group()
        return
    if a.trace_only:
        graphs._MEMSET_FIX = False
        model, ddp, opt = build()

        def step():
            ddp.zero_grad()
            with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
                out = ddp(x)
            loss = cross_entropy(out.float(), y)
            loss.backward()
            opt.step()
            return loss

        gs = graphs.GraphedStep(step, dev, comm=comm, warmup=3)
        emit({"what": "nodes", "nodes": gs.node_count, "memset_nodes": gs.memset_nodes,
              "params": [dict(zip(("dst", "value", "esize", "width", "height", "pitch"), p)) for p in gs.memset_params]})
        marker = torch.empty(64, device=dev)
        for _ in range(2):
            native.philox_(marker, 1, 0, 1)  # marker: philox_kernel runs nowhere else in this process
            torch.cuda.synchronize(dev)
            gs()
            torch.cuda.synchronize(dev)
        native.philox_(marker, 1, 0, 1)
        torch.cuda.synchronize(dev)
        env.destroy_process_group()
        return
    for fix in (False, True):
        graphs._MEMSET_FIX = fix
        model, ddp, opt = build()
        losses = []

        def step():
            ddp.zero_grad()
            with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
                out = ddp(x)
            loss = cross_entropy(out.float(), y)
            loss.backward()
            opt.step()
            return loss

        gs = graphs.GraphedStep(step, dev, comm=comm, warmup=3)
        if not fix:
            emit({"what": "nodes", "nodes": gs.node_count, "memset_nodes": gs.memset_nodes,
                  "params": [dict(zip(("dst", "value", "esize", "width", "height", "pitch"), p))
                             for p in gs.memset_params]})
            params = gs.memset_params
            emit({"what": "isolated", "dirty": False, "cases": isolated(native, dev, params, False)})
            emit({"what": "isolated", "dirty": True, "cases": isolated(native, dev, params, True)})
        # snapshot -> K replays -> A; restore -> K eager steps -> B; restore -> K eager -> B2 (the
        # run-to-run floor of the atomic solvers)
        live = _state(model, opt, ddp)
        snap = [t.detach().clone() for t in live]

        def restore():
            with torch.no_grad():
                for t, s_ in zip(live, snap):
                    t.copy_(s_)
            torch.cuda.synchronize(dev)

        def params():
            torch.cuda.synchronize(dev)
            return [t.detach().double().clone() for t in model.parameters()]

        rl = [float(gs().item()) for _ in range(a.replays)]
        pa = params()
        restore()
        el = [float(step().item()) for _ in range(a.replays)]
        pb = params()
        restore()
        el2 = [float(step().item()) for _ in range(a.replays)]
        pb2 = params()

        def gap(P, Q):
            return max(float(((p - q).abs().max() / (q.abs().max() + 1e-12))) for p, q in zip(P, Q))

        results[fix] = {"replay_losses": rl, "eager_losses": el, "eager2_losses": el2,
                        "max_rel_param_gap_replay_vs_eager": gap(pa, pb),
                        "max_rel_param_gap_eager_vs_eager": gap(pb2, pb),
                        "nonfinite_replay": any(not bool(torch.isfinite(p).all()) for p in pa)}
        emit({"what": "trajectory", "memset_fix": fix, "memset_nodes": gs.memset_nodes,
              "memsets_replaced": gs.memsets_replaced, **results[fix]})
        del gs, ddp, opt, model
        torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "a") as f:
            f.write("\n".join(lines) + "\n")
    env.destroy_process_group()


def _state(model, opt, ddp):
    """Every tensor a training step reads and writes (as benchmarks/graph_state_diff.py)."""
    ts = []
    for t in model.parameters():
        ts.append(t.data)
        sh = getattr(t, "_ptdt_bf16", None)
        if sh is not None:
            ts.append(sh)
        st = opt.state.get(t, {})
        if "momentum_buffer" in st:
            ts.append(st["momentum_buffer"])
    ts += list(model.buffers())
    ts += list(opt._counters.values())
    ts += list(ddp.reducer.bucket_tensors())
    return ts


if __name__ == "__main__":
    main()
