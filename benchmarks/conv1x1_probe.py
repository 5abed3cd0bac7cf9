#!/usr/bin/env python3
"""ResNet-50's stride-1 1x1 convolutions: MIOpen (F.conv2d, NHWC bf16, exhaustive find) vs the
same products as plain GEMMs on the NHWC activations viewed as [N*H*W, C].

fwd   Y[M, Cout]  = X[M, Cin] . W[Cout, Cin]^T
dX    dX[M, Cin]  = dY[M, Cout] . W[Cout, Cin]
dW    dW[Cout, Cin] = dY^T . X          (K = M = N*H*W)

Arms, each timed as fwd + dX + dW on the same bf16 operands (median of rounds, interleaved):
  miopen  F.conv2d forward + torch.autograd.grad (MIOpen's fwd / bwd-data / wrw solvers)
  mm      torch.mm for all three (hipBLASLt)
  native  gemm_nt_big (csrc/kernels/gemm_big.hip) for fwd and dX, torch.mm for dW

    python benchmarks/conv1x1_probe.py [--batch 128] [--rounds 5]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (H=W, Cin, Cout, count per step) of torchvision ResNet-50's stride-1 1x1 convolutions
SHAPES = [(56, 64, 64, 1), (56, 64, 256, 4), (56, 256, 64, 2), (56, 256, 128, 1), (28, 128, 512, 4),
          (28, 512, 128, 3), (28, 512, 256, 1), (14, 256, 1024, 6), (14, 1024, 256, 5), (14, 1024, 512, 1),
          (7, 512, 2048, 3), (7, 2048, 512, 2)]


def timed(fn, iters=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    from pytorch_distributed_training_tutorials_amd.ops.linear import gemm_nt_big

    dev = torch.device("cuda", 0)
    tot = {"miopen": 0.0, "mm": 0.0, "native": 0.0}
    for hw, cin, cout, cnt in SHAPES:
        M = a.batch * hw * hw
        x4 = torch.randn(a.batch, cin, hw, hw, device=dev, dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last).requires_grad_()
        w4 = (torch.randn(cout, cin, 1, 1, device=dev) * 0.05).to(torch.bfloat16).requires_grad_()
        g4 = torch.randn(a.batch, cout, hw, hw, device=dev, dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        x2 = x4.detach().permute(0, 2, 3, 1).reshape(M, cin)  # NHWC storage: a view
        w2 = w4.detach().reshape(cout, cin)
        g2 = g4.permute(0, 2, 3, 1).reshape(M, cout)

        def miopen():
            y = F.conv2d(x4, w4)
            torch.autograd.grad(y, (x4, w4), g4)

        def mm():
            torch.mm(x2, w2.t())
            torch.mm(g2, w2)
            torch.mm(g2.t(), x2)

        def native():
            gemm_nt_big(x2, w2, torch.bfloat16)
            gemm_nt_big(g2, w2.t().contiguous(), torch.bfloat16)
            torch.mm(g2.t(), x2)

        # numerics of the GEMM forms against the convolution
        y_ref = F.conv2d(x4.detach(), w2.reshape(cout, cin, 1, 1)).permute(0, 2, 3, 1).reshape(M, cout).float()
        err = float((gemm_nt_big(x2, w2, torch.bfloat16).float() - y_ref).abs().max() / y_ref.abs().max())
        arms = {"miopen": miopen, "mm": mm, "native": native}
        res = {k: [] for k in arms}
        for _ in range(a.rounds):
            for k, f in arms.items():
                res[k].append(timed(f))
        rec = {"H": hw, "Cin": cin, "Cout": cout, "M": M, "per_step": cnt, "native_fwd_rel_err": round(err, 5)}
        for k, ts in res.items():
            rec[f"{k}_us"] = round(statistics.median(ts), 1)
            tot[k] += cnt * statistics.median(ts)
        print(json.dumps(rec), flush=True)
    print(json.dumps({"total_us_per_step": {k: round(v, 1) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
