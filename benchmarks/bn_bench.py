#!/usr/bin/env python3
"""Fused BatchNorm(+residual+ReLU) training step vs PyTorch-ROCm's composite, ResNet-50 shapes.

native: ops.norm.BatchNorm2d(x, residual, relu=True) forward + backward
        (csrc/kernels/batchnorm.hip: stats+apply, reduce+apply = 4 launches)
torch : nn.BatchNorm2d (MIOpen) -> + residual -> ReLU, forward + backward

bf16 channels_last activations (the ResNet-50 DDP bench layout), batch 128. Reports
the time of one forward+backward and the effective bandwidth of the native path's
minimum traffic (fwd: read x twice, residual once, write y; bwd: read dy, x, y twice,
write dx and d(residual)).

    python benchmarks/bn_bench.py [--batch 128] [--iters 50]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [(64, 112), (256, 56), (512, 28), (1024, 14), (2048, 7)]  # (C, H=W) of ResNet-50 block outputs


def timed(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
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
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--native_only", action="store_true", help="skip the PyTorch composite arm")
    a = ap.parse_args()
    from pytorch_distributed_training_tutorials_amd.ops.norm import BatchNorm2d

    dev = torch.device("cuda", 0)
    for C, HW in SHAPES:
        shape = (a.batch, C, HW, HW)
        x = torch.randn(shape, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        r = torch.randn(shape, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        g = torch.randn(shape, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        xr, rr = x.clone().requires_grad_(), r.clone().requires_grad_()
        ours, ref = BatchNorm2d(C).to(dev), nn.BatchNorm2d(C).to(dev)

        # autograd.grad: no .grad accumulation kernels in either arm
        def native():
            y = ours(xr, rr, relu=True)
            torch.autograd.grad(y, (xr, rr, ours.weight, ours.bias), g)

        def composite():
            y = torch.relu(ref(xr) + rr)
            torch.autograd.grad(y, (xr, rr, ref.weight, ref.bias), g)

        t_nat = timed(native, a.iters)
        t_ref = float("nan") if a.native_only else timed(composite, a.iters)
        elem = x.numel() * x.element_size()
        min_bytes = elem * (4 + 7)  # fwd x,x,res,y; bwd dy,x,y,dy,x,y,dx (+dres below)
        min_bytes += elem  # d(residual)
        print(json.dumps({"metric": "BatchNorm+residual+ReLU fwd+bwd (bf16 NHWC)", "shape": list(shape),
                          "native_us": round(t_nat * 1e6, 1),
                          "red_blocks": os.environ.get("PTDT_BN_RED_BLOCKS", "default"),
                          "pipe": os.environ.get("PTDT_BN_PIPE", "1"), "torch_us": round(t_ref * 1e6, 1),
                          "speedup": round(t_ref / t_nat, 2),
                          "native_GBps_min_traffic": round(min_bytes / t_nat / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
