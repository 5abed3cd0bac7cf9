#!/usr/bin/env python3
"""LLM.int8 GEMM throughput on Llama-7B projection shapes (reference NB03:52-56, R24/K20).

Per shape (M tokens x N out x K in), timed in interleaved rounds inside one process, median:
  int8_mm     csrc/kernels/int8_mm.hip: int8 x int8 -> int32 on v_mfma_i32_16x16x64_i8, LDS-staged
              128x128 tiles, dequant (+ bias) epilogue, fp16 out -- the LLM.int8 matmul proper
  llm_int8    the whole Int8Linear(llm_int8=True) forward on fp16 activations without outliers
              (column absmax + row quantisation + int8_mm)
  bf16_big    the framework's bf16 GEMM (gemm_big.hip) on the same shape
  torch_bf16  torch.matmul bf16 (hipBLASLt)
  torch_fp16  torch.matmul fp16 (hipBLASLt), the reference's unquantised dtype
One JSON line per shape: TOPS / TFLOP/s per variant (2 M N K ops).

    python benchmarks/int8_bench.py [--shapes 4096x11008x4096,...] [--rounds 5]
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
    ap.add_argument("--shapes", default="4096x11008x4096,4096x4096x11008,4096x4096x4096,2048x11008x4096,"
                                        "512x11008x4096,16x11008x4096")
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    from pytorch_distributed_training_tutorials_amd import native
    from pytorch_distributed_training_tutorials_amd.ops.quant import Int8Linear

    C = native()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    for spec in a.shapes.split(","):
        M, N, K = (int(v) for v in spec.split("x"))
        Aq = torch.randint(-127, 128, (M, K), device=dev, dtype=torch.int8)
        Bq = torch.randint(-127, 128, (N, K), device=dev, dtype=torch.int8)
        sa, sb = torch.rand(M, device=dev) * 1e-3, torch.rand(N, device=dev) * 1e-3
        xh = (torch.rand(M, K, device=dev) * 2 - 1).half()
        wh = (torch.rand(N, K, device=dev) * 2 - 1).half() * 0.05
        xb, wb = xh.bfloat16(), wh.bfloat16()
        lin = torch.nn.Linear(K, N, bias=False, device=dev, dtype=torch.float16)
        with torch.no_grad():
            lin.weight.copy_(wh)
        q = Int8Linear.from_linear(lin, llm_int8=True, threshold=1e9)  # no outliers: the pure int8 product
        cb = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        variants = {
            "int8_mm": lambda: C.int8_mm(Aq, sa, Bq, sb, None, None, "float16"),
            "llm_int8": lambda: q(xh),
            "torch_bf16": lambda: torch.matmul(xb, wb.t()),
            "torch_fp16": lambda: torch.matmul(xh, wh.t()),
        }
        if C.gemm_big_ok(xb, wb):
            variants["bf16_big"] = lambda: C.gemm_big_(xb, wb, cb)
        times = {k: [] for k in variants}
        for fn in variants.values():  # warm-up / autotune
            fn()
        torch.cuda.synchronize()
        ops = 2.0 * M * N * K
        iters = max(3, min(200, int(2e12 / ops)))
        for _ in range(a.rounds):
            for k, fn in variants.items():
                times[k].append(timed(fn, iters))
        rec = {"M": M, "N": N, "K": K}
        for k, ts in times.items():
            t = statistics.median(ts)
            rec[f"{k}_us"] = round(t * 1e6, 1)
            rec[f"{k}_T"] = round(ops / t / 1e12, 1)
        rec["int8_vs_bf16_big"] = round(rec["bf16_big_us"] / rec["int8_mm_us"], 2) if "bf16_big_us" in rec else None
        rec["int8_vs_torch_fp16"] = round(rec["torch_fp16_us"] / rec["int8_mm_us"], 2)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
