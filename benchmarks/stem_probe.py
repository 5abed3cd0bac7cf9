#!/usr/bin/env python3
"""ResNet-50 stem probe: the 7x7/2 convolution on 3 input channels is MIOpen's worst conv
of the step (~180 us forward + ~180 us weight gradient at batch 128, bf16 NHWC: C = 3 is
a poor fit for 16x16x32 MFMA K-tiles; profiles/r3_resnet_graph.md). This times the conv's
forward + input-free backward (weight gradient only: the stem's input needs no gradient)
with the input channels zero-padded to 4 and 8 -- the same arithmetic result, since the
padded weight channels meet zero inputs -- to see whether a padded stem is cheaper than
the pad copy it costs.

    python benchmarks/stem_probe.py [--batch 128] [--iters 20]
"""
from __future__ import annotations

import argparse
import json

import torch
import torch.nn.functional as F


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda", 0)
    x3 = torch.randn(a.batch, 3, 224, 224, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w3 = torch.randn(64, 3, 7, 7, device=dev, dtype=torch.bfloat16) * 0.05
    gy = torch.randn(a.batch, 64, 112, 112, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    ref = None
    for cin in (3, 4, 8):
        w = F.pad(w3, (0, 0, 0, 0, 0, cin - 3)).contiguous(memory_format=torch.channels_last).requires_grad_(True)

        def step():
            x = x3 if cin == 3 else F.pad(x3, (0, 0, 0, 0, 0, cin - 3)).contiguous(memory_format=torch.channels_last)
            y = F.conv2d(x, w, stride=2, padding=3)
            (gw,) = torch.autograd.grad(y, w, gy)
            return y, gw

        for _ in range(3):
            y, gw = step()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            y, gw = step()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / a.iters * 1e3
        if ref is None:
            ref = (y.float(), gw.float())
            err_y = err_w = 0.0
        else:
            err_y = ((y.float() - ref[0]).abs().max() / ref[0].abs().max()).item()
            err_w = ((gw[:, :3].float() - ref[1]).abs().max() / ref[1].abs().max()).item()
        print(json.dumps({"cin": cin, "fwd_plus_wgrad_us": round(us, 1), "rel_err_y": err_y, "rel_err_dw": err_w}),
              flush=True)


if __name__ == "__main__":
    main()
