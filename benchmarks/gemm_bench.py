#!/usr/bin/env python3
"""Throughput of the native bf16 GEMMs vs PyTorch-ROCm's library GEMM (hipBLASLt).

Kernels:
  auto      ops.linear.gemm_nt_big: csrc/kernels/gemm_big.hip with plan_big's (tile, split-K)
  big256    gemm_big.hip, 256x256x64 tile, 8 waves, ping-pong      C = A . Bt^T
  big128    gemm_big.hip, 128x128x64 tile, 4 waves, 2 workgroups per CU
  big128_sS big128 with split-K over S slices (f32 atomics + zero fill + bf16 cast, all timed)
  tile      csrc/kernels/gemm.hip      (64x64 strided tile, the small-shape path)
  torch     torch.matmul (hipBLASLt), same operands

Operands are uniform [-1, 1) (zero-filled operands read high: DVFS), variants are
timed in interleaved rounds inside one process (cdna_hip_programming.md §5.4 rules
24-25) and the median is reported. One JSON line per shape.

    python benchmarks/gemm_bench.py [--shapes 4096x4096x4096,8192x8192x8192] [--rounds 5]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--shapes", default="4096x4096x4096,8192x8192x8192,8192x8192x1024,4096x11008x4096,"
                                        "120x1000x2048,2048x2048x2048,"
                                        "1024x1024x1024,4096x4096x1024,3072x3072x3072,256x4096x4096,"
                                        "128x2048x8192,120x2048x1024")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--tile", action="store_true", help="also time the 64x64 strided kernel")
    ap.add_argument("--extra_sched", type=int, nargs="*", default=[],
                    help="also time these schedules of the 256 kernel (0: 8 waves read-then-multiply, "
                         "1: 8 waves ping-pong (default))")
    ap.add_argument("--splits", default="2,4,8,16", help="split-K slice counts to time with the 128 tile")
    a = ap.parse_args()
    from pytorch_distributed_training_tutorials_amd import native
    from pytorch_distributed_training_tutorials_amd.ops.linear import gemm_nt_big, plan_big

    C_ = native()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    for spec in a.shapes.split(","):
        M, N, K = (int(v) for v in spec.split("x"))
        A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        Bt = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
        Cb = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        Ct = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        flops = 2.0 * M * N * K
        variants = {"torch": lambda: torch.matmul(A, Bt.t(), out=Ct)}
        outs = {"torch": Ct}
        if C_.gemm_big_ok(A, Bt):
            def auto():
                outs["auto"] = gemm_nt_big(A, Bt, torch.bfloat16)
            variants["auto"] = auto
            variants["big256"] = lambda: C_.gemm_big_(A, Bt, Cb)  # default schedule (4)
            for sc in a.extra_sched:
                variants[f"big256_sched{sc}"] = (lambda sc=sc: C_.gemm_big_(A, Bt, Cb, sched=sc))
            variants["big128"] = lambda: C_.gemm_big_(A, Bt, Cb, tile=128)
            for sp in (int(v) for v in a.splits.split(",") if v):
                if sp <= K // 64:
                    def split_fn(sp=sp):
                        acc = torch.zeros(M, N, device=dev, dtype=torch.float32)
                        C_.gemm_big_(A, Bt, acc, tile=128, split_k=sp)
                        outs[f"big128_s{sp}"] = acc.to(torch.bfloat16)
                    variants[f"big128_s{sp}"] = split_fn
        if a.tile:
            variants["tile"] = lambda: C_.gemm_(A, Bt.t(), Cb, None, None, False, 1.0, 0.0, None, 1)
        # numerics vs fp32 on the same bf16 operands
        ref = A.float() @ Bt.float().t()
        err = {}
        for k, f in variants.items():
            f()
            torch.cuda.synchronize()
            out = outs.get(k, Cb)
            err[k] = float((out.float() - ref).abs().max() / ref.abs().max())
        iters = max(3, min(200, int(2e13 / flops)))
        for f in variants.values():
            timed(f, 2)
        res = {k: [] for k in variants}
        for _ in range(a.rounds):
            for k, f in variants.items():
                res[k].append(timed(f, iters))
        rec = {"metric": "bf16 GEMM TFLOP/s (C = A.Bt^T, uniform[-1,1) operands)", "M": M, "N": N, "K": K,
               "iters": iters, "rounds": a.rounds}
        res_med = {k: statistics.median(ts) for k, ts in res.items()}
        for k, ts in res.items():
            med = res_med[k]
            rec[f"{k}_tflops"] = round(flops / med / 1e12, 1)
            rec[f"{k}_us"] = round(med * 1e6, 2)
            rec[f"{k}_max_rel_err"] = round(err[k], 5)
        if "auto" in res:
            rec["plan"] = list(plan_big(M, N, K))
            rec["auto_vs_torch"] = round(res_med["torch"] / res_med["auto"], 3)  # time ratio: tiny shapes round TFLOP/s to 0
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
