#!/usr/bin/env python3
"""One training step out of a rocprofv3 database (``*_results.db``), grouped by kernel family
(``tools/trace_step.py`` families): ``python tools/step_breakdown.py DB [--marker ce_fwd_kernel]``.
Prints markdown (family table + top kernels of the step), so a large trace can be summarised on the
GPU box and only the summary copied back."""
from __future__ import annotations

import argparse
import re
import sqlite3
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from trace_step import family  # noqa: E402


def main():
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("db")
    ap.add_argument("--marker", default="ce_fwd_kernel")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    rows = sqlite3.connect(a.db).execute("select name,start,end from kernels order by start").fetchall()
    marks = [i for i, r in enumerate(rows) if a.marker in r[0]]
    if len(marks) < 2:
        raise SystemExit(f"fewer than two {a.marker!r} dispatches")
    lo, hi = marks[-2], marks[-1]
    step = rows[lo:hi]
    busy, per = defaultdict(float), defaultdict(lambda: [0, 0.0])
    for n, s, e in step:
        busy[family(n)] += (e - s) / 1e3
        short = re.sub(r"\(.*$", "", n.replace("(anonymous namespace)::", "").replace("void ", ""))[:90]
        per[short][0] += 1
        per[short][1] += (e - s) / 1e3
    print(f"step span {(rows[hi][1] - rows[lo][1]) / 1e3:.1f} us, {len(step)} dispatches, "
          f"busy {sum(busy.values()):.1f} us\n")
    print("| family | us / step |\n|---|---:|")
    for f, t in sorted(busy.items(), key=lambda x: -x[1]):
        print(f"| {f} | {t:.1f} |")
    print("\n| top kernels | calls | us |\n|---|---:|---:|")
    for n, (k, t) in sorted(per.items(), key=lambda x: -x[1][1])[: a.top]:
        print(f"| `{n}` | {k} | {t:.1f} |")


if __name__ == "__main__":
    main()
