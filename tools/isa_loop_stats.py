#!/usr/bin/env python3
"""Instruction mix of every loop in one kernel of a device assembly file (hipcc --cuda-device-only -S).

    python3 tools/isa_loop_stats.py flag.s [kernel-symbol-substring] [--min-span 150] [--max-span 1000] [--steps]

A loop is a backward branch (s_branch / s_cbranch_* to an earlier label of the same kernel); for each
one spanning at least --min-span lines it prints the counts of VALU, DPP, permlane, SALU, vector
memory, LDS, waitcnt and s_nop instructions. Used to compare step-loop bodies of the persistent
engines between builds (profiles/r6_wave_step.md)."""
from __future__ import annotations

import re
import sys


def kernels(lines):
    out, cur, start = {}, None, 0
    for n, l in enumerate(lines):
        m = re.match(r"^(_Z\w+):", l)
        if m:
            cur, start = m.group(1), n
        elif cur and l.startswith(".Lfunc_end"):
            out[cur] = (start, n)
            cur = None
    return out


CLASSES = [
    ("valu", r"^v_(?!mfma)"),
    ("dpp", r"^v_\w+_dpp|^v_\w+.*(row_|quad_perm)"),
    ("permlane", r"^v_permlane"),
    ("pk", r"^v_pk_"),
    ("salu", r"^s_(?!waitcnt|nop|cbranch|branch|barrier)"),
    ("branch", r"^s_(cbranch|branch)"),
    ("vmem", r"^(global_|buffer_|flat_)"),
    ("lds", r"^ds_"),
    ("waitcnt", r"^s_waitcnt"),
    ("nop", r"^s_nop"),
]


def stats(body):
    c = {k: 0 for k, _ in CLASSES}
    for l in body:
        t = l.strip()
        if not t or t.startswith((";", ".")) or t.endswith(":"):
            continue
        for k, pat in CLASSES:
            if re.search(pat, t):
                c[k] += 1
    return c


def main(argv):
    path = argv[0]
    sub = argv[1] if len(argv) > 1 and not argv[1].startswith("--") else ""
    min_span = int(argv[argv.index("--min-span") + 1]) if "--min-span" in argv else 150
    max_span = int(argv[argv.index("--max-span") + 1]) if "--max-span" in argv else 1000
    steps_only = "--steps" in argv  # only loops with permlane instructions (the engines' step loops)
    lines = open(path).read().split("\n")
    for name, (a, b) in kernels(lines).items():
        if sub not in name:
            continue
        print(name)
        labels = {}
        for n in range(a, b):
            m = re.match(r"^(\.LBB\d+_\d+):", lines[n])
            if m:
                labels[m.group(1)] = n
        for n in range(a, b):
            m = re.search(r"s_(?:cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", lines[n])
            if m and labels.get(m.group(1), 1 << 60) < n and n - labels[m.group(1)] >= min_span:
                if n - labels[m.group(1)] > max_span:
                    continue
                s = stats(lines[labels[m.group(1)]:n + 1])
                if steps_only and not s["permlane"]:
                    continue
                print(f"  loop {labels[m.group(1)]}-{n}: " + " ".join(f"{k} {v}" for k, v in s.items()))


if __name__ == "__main__":
    main(sys.argv[1:])
