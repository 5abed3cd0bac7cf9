#!/usr/bin/env python3
"""Comm/compute overlap of a DDP training trace (rocprofv3 ``--kernel-trace`` database).

``python tools/overlap_report.py gpurun_out/prof/resnet_results.db [--steps 3]``

Splits the dispatches into RCCL kernels (names containing ``nccl``/``rccl``) and
everything else ("compute"), finds the last ``--steps`` iterations (an iteration
ends at the last optimizer kernel before the next forward; here: the boundaries
are the dispatches of the SGD kernel ``sgd_multi``/``sgd_flat``), and reports per
iteration:

* comm busy time, and how much of it runs concurrently with compute kernels;
* the post-backward tail: time from the end of the last non-RCCL kernel before
  the optimizer to the end of the last all-reduce (what the optimizer waits for);
* each bucket all-reduce's start/end relative to the iteration start.
"""
from __future__ import annotations

import argparse
import re
import sqlite3

COMM = re.compile(r"nccl|rccl|oneRankReduce", re.I)  # oneRankReduce: RCCL at world 1
OPT = re.compile(r"sgd_multi|sgd_flat")


def merge(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def inter(a, b):
    i = j = 0
    tot = 0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if s < e:
            tot += e - s
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--table", type=int, default=0, help="also print the top-N kernels of those iterations")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end, stream_id from kernels order by start").fetchall()
    opt_idx = [k for k, r in enumerate(rows) if OPT.search(r[0])]
    # iteration boundaries: first optimizer dispatch of each optimizer group
    bounds = [opt_idx[0]] if opt_idx else []
    for k in opt_idx[1:]:
        if k - bounds[-1] > 50:
            bounds.append(k)
    print("| iter | step ms | comm busy ms | comm concurrent w/ compute | tail after last bwd kernel us | buckets |")
    print("|---|---|---|---|---|---|")
    for it in range(max(0, len(bounds) - a.steps), len(bounds)):
        lo = bounds[it - 1] + 1 if it > 0 else 0
        hi = bounds[it]
        seg = rows[lo:hi]
        if not seg:
            continue
        t0 = seg[0][1]
        comm = [(r[1], r[2]) for r in seg if COMM.search(r[0])]
        comp = [(r[1], r[2]) for r in seg if not COMM.search(r[0])]
        mc, mp = merge(comm), merge(comp)
        busy = sum(e - s for s, e in mc)
        conc = inter(mc, mp)
        last_comp = max(e for s, e in comp) if comp else t0
        last_comm = max(e for s, e in comm) if comm else last_comp
        tail = max(0, last_comm - last_comp)
        bk = ", ".join(f"{(s - t0) / 1e6:.2f}-{(e - t0) / 1e6:.2f}" for s, e in comm)
        step = (rows[hi][1] - t0) / 1e6
        print(f"| {it} | {step:.2f} | {busy / 1e6:.3f} | {100 * conc / max(busy, 1):.0f}% | {tail / 1e3:.0f} | {bk} |")
    if a.table and len(bounds) > a.steps:
        lo, hi = bounds[len(bounds) - a.steps - 1] + 1, bounds[-1] + 1
        agg = {}
        for name, s0, e0, _ in rows[lo:hi]:
            n, t = agg.get(name, (0, 0))
            agg[name] = (n + 1, t + e0 - s0)
        tot = sum(t for _, t in agg.values())
        print(f"\nkernels of the last {a.steps} iterations (busy {tot / 1e6 / a.steps:.2f} ms per iteration)\n")
        print("| kernel | calls/iter | us/iter | % |")
        print("|---|---|---|---|")
        for name, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.table]:
            short = name.replace("void ", "").replace("(anonymous namespace)::", "")
            short = re.sub(r"\(.*$", "", short)[:90]
            print(f"| `{short}` | {n / a.steps:.0f} | {t / 1e3 / a.steps:.0f} | {100 * t / tot:.1f} |")


if __name__ == "__main__":
    main()
