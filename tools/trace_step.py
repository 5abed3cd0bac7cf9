#!/usr/bin/env python3
"""One training step out of a rocprofv3 kernel trace (CSV), grouped by kernel family.

``python tools/trace_step.py gpurun_out/prof/run_kernel_trace.csv [--marker ce_fwd] [--top 25]``

The step is the span between the last two dispatches whose name contains ``--marker`` (the loss
kernel runs once per step). Prints busy time per family, the idle time between consecutive
dispatches, and the top kernels by time -- the ResNet-50 breakdown of profiles/r3_resnet_graph.md.
"""
from __future__ import annotations

import argparse
import csv
import re
from collections import defaultdict

FAMILIES = [
    ("conv1x1+BN stats (native)", r"conv1x1_bn_stream|gemm_bn_stats"),
    ("conv1x1 dgrad+wgrad with BN apply (native)", r"conv1x1_bwd"),
    ("BN fwd (native)", r"bn_stats_kernel|bn_apply_kernel"),
    ("BN bwd (native)", r"bn_bwd"),
    ("MIOpen conv (CK / ASM igemm)", r"igemm|ck::|_ZN2ck|conv|Conv|gridwise|xdlops|miopenSp3AsmConv|naive_conv"),
    ("MIOpen helpers (fill/SubTensorOp/transpose)", r"SubTensorOp|Op2d|fill|Fill|transpose|Transpose|Set|Copy"),
    ("pool (native)", r"maxpool"),
    ("SGD / casts / reducer (native)", r"sgd|cast|bucket|optim"),
    # Cijk_* are rocBLAS / hipBLASLt (Tensile) GEMMs: in a ResNet step these are mostly MIOpen's
    # GEMM-based convolutions (1x1 / strided), plus the fc when the Linear selector picked the
    # library; the native Linear kernels are named gemm_* / linear_*
    ("rocBLAS/hipBLASLt GEMM (MIOpen GEMM-convs; fc if library)", r"Cijk"),
    ("GEMM (native Linear / fc)", r"gemm|linear_"),
    ("loss", r"ce_|cross"),
]


def family(name: str) -> str:
    for fam, pat in FAMILIES:
        if re.search(pat, name):
            return fam
    return "other"


def main():
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("csv")
    ap.add_argument("--marker", default="ce_fwd")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if a.marker in r[2]]
    if len(marks) < 2:
        raise SystemExit(f"fewer than two {a.marker!r} dispatches")
    lo, hi = marks[-2], marks[-1]
    step = rows[lo:hi]
    span = (rows[hi][0] - rows[lo][0]) / 1e3
    busy = defaultdict(float)
    per = defaultdict(lambda: [0, 0.0])
    idle = 0.0
    for k, (s, e, n) in enumerate(step):
        busy[family(n)] += (e - s) / 1e3
        short = re.sub(r"\(.*$", "", n.replace("(anonymous namespace)::", "").replace("void ", ""))[:90]
        per[short][0] += 1
        per[short][1] += (e - s) / 1e3
        if k + 1 < len(step):
            idle += max(0, step[k + 1][0] - e) / 1e3
    print(f"step span {span:.1f} us, {len(step)} dispatches, busy {sum(busy.values()):.1f} us, idle {idle:.1f} us\n")
    print("| family | us / step |\n|---|---:|")
    for fam, t in sorted(busy.items(), key=lambda x: -x[1]):
        print(f"| {fam} | {t:.1f} |")
    print(f"\n| top kernels | calls | us |\n|---|---:|---:|")
    for n, (c, t) in sorted(per.items(), key=lambda x: -x[1][1])[: a.top]:
        print(f"| `{n}` | {c} | {t:.1f} |")


if __name__ == "__main__":
    main()
