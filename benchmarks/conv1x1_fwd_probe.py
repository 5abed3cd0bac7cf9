#!/usr/bin/env python3
"""ResNet-50's stride-1 1x1 convolutions, FORWARD only: what a native 1x1-conv forward with the
BatchNorm statistics in its epilogue would replace.

Per shape (bf16 NHWC, batch 128), medians of interleaved rounds:
  miopen_us     F.conv2d forward (MIOpen, exhaustive find)
  gemm256_us    gemm_big on the NHWC view [N*H*W, Cin] x W[Cout, Cin]^T, 256x256 tile
  gemm128_us    the same, 128x128 tile
  mm_us         torch.mm (hipBLASLt)
  bnfwd_us      the native BN forward over the conv output (statistics pass + apply pass)
  apply_us      the apply pass alone (bnfwd - apply = the statistics pass the fusion removes)
  fused*_us     conv1x1_bn_stats (native GEMM + BN statistics in the epilogue), 256 / 128 tiles
  stream_us     the streaming conv + statistics kernel (conv1x1_bn.hip), where it has an instance

    python benchmarks/conv1x1_fwd_probe.py [--batch 128] [--rounds 5]
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

from benchmarks.conv1x1_probe import SHAPES, timed  # noqa: E402


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--sweep", action="store_true",
                    help="streaming kernel only: time every pipeline configuration (PTDT_C1_CFG 0-3) per shape")
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    from pytorch_distributed_training_tutorials_amd._ext import native
    from pytorch_distributed_training_tutorials_amd.ops.linear import gemm_nt_big

    C = native()
    dev = torch.device("cuda", 0)
    tot = {}
    if a.sweep:
        from pytorch_distributed_training_tutorials_amd.ops.convbn import conv1x1_stats_probe

        for hw, cin, cout, cnt in SHAPES:
            if not C.conv1x1_bn_stream_supported(cin, cout):
                continue
            M = a.batch * hw * hw
            x2 = torch.randn(M, cin, device=dev).to(torch.bfloat16)
            w2 = (torch.randn(cout, cin, device=dev) * 0.05).to(torch.bfloat16)
            rec = {"H": hw, "Cin": cin, "Cout": cout, "M": M, "per_step": cnt}
            res = {}
            splits = (0, 1) if (cin, cout) == (64, 256) else (0,)
            for _ in range(a.rounds):
                for sp in splits:
                    os.environ["PTDT_C1_SPLIT"] = str(sp)
                    for cfg in range(4):
                        os.environ["PTDT_C1_CFG"] = str(cfg)
                        res.setdefault(cfg + 10 * sp, []).append(timed(conv1x1_stats_probe(x2, w2, 0)))
            os.environ.pop("PTDT_C1_CFG")
            os.environ.pop("PTDT_C1_SPLIT")
            for cfg, ts in res.items():
                rec[f"cfg{cfg % 10}{'_split' if cfg >= 10 else ''}_us"] = round(statistics.median(ts), 1)
            rec["GBps_cfg0"] = round(2 * M * (cin + cout) / (rec["cfg0_us"] * 1e-6) / 1e9)
            print(json.dumps(rec), flush=True)
        return
    for hw, cin, cout, cnt in SHAPES:
        M = a.batch * hw * hw
        x4 = torch.randn(a.batch, cin, hw, hw, device=dev, dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        w4 = (torch.randn(cout, cin, 1, 1, device=dev) * 0.05).to(torch.bfloat16)
        x2 = x4.permute(0, 2, 3, 1).reshape(M, cin)
        w2 = w4.reshape(cout, cin)
        y4 = F.conv2d(x4, w4)
        bn = torch.nn.BatchNorm2d(cout).to(dev)
        sc, sh = torch.ones(cout, device=dev), torch.zeros(cout, device=dev)
        arms = {
            "miopen": lambda: F.conv2d(x4, w4),
            "gemm256": lambda: gemm_nt_big(x2, w2, torch.bfloat16, plan=(256, 1)),
            "gemm128": lambda: gemm_nt_big(x2, w2, torch.bfloat16, plan=(128, 1)),
            "mm": lambda: torch.mm(x2, w2.t()),
            "bnfwd": lambda: C.bn_fwd_train(y4, bn.weight, bn.bias, None, None, None, None, False, 0.1, 1e-5,
                                            None, False),
            "apply": lambda: C.bn_apply(y4, None, sc, sh, False),
        }
        if hasattr(C, "conv1x1_bn_stats"):
            from pytorch_distributed_training_tutorials_amd.ops.convbn import conv1x1_stats_probe

            arms["fused256"] = conv1x1_stats_probe(x2, w2, 256)
            arms["fused128"] = conv1x1_stats_probe(x2, w2, 128)
            if C.conv1x1_bn_stream_supported(cin, cout):
                arms["stream"] = conv1x1_stats_probe(x2, w2, 0)
        res = {k: [] for k in arms}
        with torch.no_grad():
            for _ in range(a.rounds):
                for k, f in arms.items():
                    res[k].append(timed(f))
        rec = {"H": hw, "Cin": cin, "Cout": cout, "M": M, "per_step": cnt}
        for k, ts in res.items():
            rec[f"{k}_us"] = round(statistics.median(ts), 1)
            tot[k] = tot.get(k, 0.0) + cnt * statistics.median(ts)
        # bytes of the forward (read X and W, write Y) at the measured MIOpen time
        rec["miopen_TBps"] = round(2 * (M * cin + M * cout) / (rec["miopen_us"] * 1e-6) / 1e12, 2)
        print(json.dumps(rec), flush=True)
    print(json.dumps({"total_us_per_step": {k: round(v, 1) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
