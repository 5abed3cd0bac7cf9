#!/usr/bin/env python3
"""Achieved HBM bandwidth per kernel from rocprofv3 ``--pmc FETCH_SIZE`` / ``--pmc WRITE_SIZE`` passes
(each with ``--kernel-trace --output-format csv``):
``python tools/pmc_bandwidth.py FETCH_DIR WRITE_DIR --match 'conv1x1_bwd|bn_'``.
Per kernel name: mean FETCH_SIZE and WRITE_SIZE (KB), mean duration (from each pass's kernel trace),
and (fetch + write) / duration in TB/s. Markdown on stdout."""
from __future__ import annotations

import argparse
import csv
import glob
import re
from collections import defaultdict


def _short(n: str) -> str:
    return re.sub(r"\(.*$", "", n.replace("(anonymous namespace)::", "").replace("void ", ""))[:80]


def load(d: str, counter: str, pat: str):
    vals, durs = defaultdict(list), defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        per = defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter or not re.search(pat, r.get("Kernel_Name", "")):
                continue
            key = r.get("Dispatch_Id", r.get("Correlation_Id", ""))
            per[key] += float(r["Counter_Value"])
            names[key] = _short(r["Kernel_Name"])
        for k, v in per.items():
            vals[names[k]].append(v)
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if re.search(pat, r.get("Kernel_Name", "")):
                durs[_short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    return vals, durs


def main():
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    fv, fd = load(a.fetch_dir, "FETCH_SIZE", a.match)
    wv, wd = load(a.write_dir, "WRITE_SIZE", a.match)
    print("| kernel | calls | FETCH KB | WRITE KB | us | TB/s |\n|---|---:|---:|---:|---:|---:|")
    for k in sorted(set(fv) | set(wv)):
        f = sum(fv[k]) / len(fv[k]) if fv.get(k) else 0.0
        w = sum(wv[k]) / len(wv[k]) if wv.get(k) else 0.0
        ds = fd.get(k, []) + wd.get(k, [])
        t = sum(ds) / len(ds) if ds else float("nan")
        bw = (f + w) * 1024 / t / 1e12 if ds and t > 0 else float("nan")
        print(f"| `{k}` | {len(fv.get(k, []))} | {f:.0f} | {w:.0f} | {t * 1e6:.1f} | {bw:.2f} |")


if __name__ == "__main__":
    main()
