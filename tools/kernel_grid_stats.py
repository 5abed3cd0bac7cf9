#!/usr/bin/env python3
"""Mean duration per (kernel, grid) from rocprofv3 ``--kernel-trace --output-format csv`` output:
``python tools/kernel_grid_stats.py DIR [--match REGEX]``. Separates launches of one kernel by grid
size, i.e. by problem shape, which ``--stats`` folds together. Markdown on stdout."""
from __future__ import annotations

import argparse
import csv
import glob
import re
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("dir")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    d = defaultdict(list)
    for f in glob.glob(f"{a.dir}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            n = r.get("Kernel_Name", "")
            if not re.search(a.match, n):
                continue
            n = re.sub(r"\(.*$", "", n.replace("(anonymous namespace)::", "").replace("void ", ""))[:70]
            grid = "x".join(r.get(k, "?") for k in ("Grid_Size_X", "Grid_Size_Y") if k in r)
            d[(n, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
    print("| kernel | grid (threads) | calls | mean us | min us |\n|---|---|---:|---:|---:|")
    for (n, g), v in sorted(d.items()):
        print(f"| `{n}` | {g} | {len(v)} | {sum(v) / len(v):.1f} | {min(v):.1f} |")


if __name__ == "__main__":
    main()
