#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 ``--pmc`` passes (counter_collection.csv), for kernels whose name
matches a pattern: ``python tools/pmc_kernels.py DIR [DIR ...] --match conv1x1_bn_stream``.

Prints one markdown row per kernel (template arguments kept, argument list dropped) with every
counter averaged over its dispatches, plus derived shares where the counters allow: MFMA busy /
wave-cycles... as raw quad-cycle counts (SQ_* busy/wait counters are in quad-cycles)."""
from __future__ import annotations

import argparse
import csv
import glob
import re
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    acc = defaultdict(lambda: defaultdict(list))
    for d in a.dirs:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            per = defaultdict(dict)
            for r in csv.DictReader(open(f)):
                name = r.get("Kernel_Name", "")
                if a.match and not re.search(a.match, name):
                    continue
                key = (name, r.get("Dispatch_Id", r.get("Correlation_Id", "")))
                per[key][r["Counter_Name"]] = per[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            for (name, _), cs in per.items():
                short = re.sub(r"\(.*$", "", name.replace("(anonymous namespace)::", "").replace("void ", ""))
                for c, v in cs.items():
                    acc[short][c].append(v)
    counters = sorted({c for k in acc.values() for c in k})
    print("| kernel | " + " | ".join(counters) + " |")
    print("|---|" + "---:|" * len(counters))
    for k, cs in sorted(acc.items()):
        vals = [(sum(cs[c]) / len(cs[c])) if cs.get(c) else float("nan") for c in counters]
        print(f"| `{k[:80]}` | " + " | ".join(f"{v:.4g}" for v in vals) + " |")


if __name__ == "__main__":
    main()
