#!/usr/bin/env python3
"""Per-pass bandwidth of the native BatchNorm kernels on the ResNet-50 step's shapes.

Drives ``native().bn_fwd_train`` / ``native().bn_bwd`` directly (no autograd) for
the three BN kinds of a ResNet-50 bottleneck (bf16 NHWC, batch 128):

  res : bn3 -- y = ReLU(BN(x) + residual), bit mask out; backward with the next
        block's residual gradient added (dy2) and g = d(residual) materialised
  relu: bn1 / bn2 -- y = ReLU(BN(x)); backward recomputes the mask from x
  lin : downsample BN -- no ReLU

and reports each forward / backward's time and effective bandwidth over its
minimum traffic, plus ``resnet_bn_ms``: the per-step BN time weighted by how
many BNs of each kind and shape one ResNet-50 step runs (the profile in
profiles/r3_resnet_bn.md). The kernels' geometry knobs are read from the
environment once per process (PTDT_BN_TC, PTDT_BN_AU, PTDT_BN_APPLY_BLOCKS),
so a sweep runs this once per setting.

    python benchmarks/bn_kernel_bench.py [--iters 30]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

B = 128
# (kind, C, HW, count per ResNet-50 step)
CASES = [("res", 256, 56, 3), ("res", 512, 28, 4), ("res", 1024, 14, 6), ("res", 2048, 7, 3),
         ("relu", 64, 112, 1), ("relu", 64, 56, 6), ("relu", 128, 56, 1), ("relu", 128, 28, 7),
         ("relu", 256, 14, 12), ("relu", 256, 28, 1), ("relu", 512, 7, 6), ("relu", 512, 14, 1),
         ("lin", 256, 56, 1), ("lin", 512, 28, 1), ("lin", 1024, 14, 1), ("lin", 2048, 7, 1)]


def timed(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--kinds", default="res,relu,lin", help="comma list of BN kinds to run")
    a = ap.parse_args()
    kinds = set(a.kinds.split(","))
    from pytorch_distributed_training_tutorials_amd._ext import native

    C_ = native()
    dev = torch.device("cuda", 0)
    knobs = {k: os.environ.get(k, "default") for k in ("PTDT_BN_TC", "PTDT_BN_AU", "PTDT_BN_APPLY_BLOCKS", "PTDT_BN_DIR")}
    total = 0.0
    for kind, C, HW, count in CASES:
        if kind not in kinds:
            continue
        shape = (B, C, HW, HW)
        mk = lambda: torch.randn(shape, device=dev, dtype=torch.bfloat16).contiguous(  # noqa: E731
            memory_format=torch.channels_last)
        x, dy = mk(), mk()
        res = mk() if kind == "res" else None
        dy2 = mk() if kind == "res" else None
        w = torch.ones(C, device=dev)
        b = torch.zeros(C, device=dev)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        nbt = torch.zeros((), dtype=torch.long, device=dev)
        relu = kind != "lin"
        want_mask = kind == "res"
        out = {}

        def fwd():
            out["f"] = C_.bn_fwd_train(x, w, b, rm, rv, nbt, res, relu, 0.1, 1e-5, None, want_mask)

        fwd()
        y, stats, mask = out["f"]

        def bwd():
            C_.bn_bwd(dy, x, None, w, stats, relu, kind == "res", True, None, None, None, dy2,
                      mask if want_mask else None)

        tf, tb = timed(fwd, a.iters), timed(bwd, a.iters)
        E = x.numel() * x.element_size()
        if kind == "res":
            bf, bb = E + 3 * E + E / 16, (4 * E + E / 16) + 3 * E
        else:
            bf, bb = 3 * E, 5 * E
        total += count * (tf + tb)
        print(json.dumps({"kind": kind, "shape": list(shape), "fwd_us": round(tf * 1e6, 1),
                          "bwd_us": round(tb * 1e6, 1), "fwd_TBps": round(bf / tf / 1e12, 2),
                          "bwd_TBps": round(bb / tb / 1e12, 2), **knobs}), flush=True)
    for C, HW in ((256, 56), (256, 28)):  # calibration: torch's own streaming kernels on the same sizes
        shape = (B, C, HW, HW)
        x, r, y = (torch.randn(shape, device=dev, dtype=torch.bfloat16) for _ in range(3))
        E = x.numel() * x.element_size()
        tc = timed(lambda: y.copy_(x), a.iters)
        ta = timed(lambda: torch.add(x, r, out=y), a.iters)
        print(json.dumps({"kind": "calib", "shape": list(shape), "copy_TBps": round(2 * E / tc / 1e12, 2),
                          "add_TBps": round(3 * E / ta / 1e12, 2)}), flush=True)
    print(json.dumps({"metric": "resnet_bn_ms", "value": round(total * 1e3, 3), **knobs}), flush=True)


if __name__ == "__main__":
    main()
