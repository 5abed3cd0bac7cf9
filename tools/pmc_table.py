#!/usr/bin/env python3
"""Per-step PMC table of a persistent-engine run (rocprofv3 --pmc CSV passes).

``python tools/pmc_table.py --steps 20000 tp=gpurun_out/pmc20_tp_1,gpurun_out/pmc20_tp_2 mfma=...``

Takes the largest dispatch of the engine kernel in each pass and prints, per engine,
the counters per DDP step (per wave: / (steps * waves)). SQ_WAVE_CYCLES and the
SQ_WAIT_* / SQ_ACTIVE_* counters are in quad-cycles (x4 = cycles).
"""
from __future__ import annotations

import csv
import glob
import sys
from collections import defaultdict

ENGINE = ("mlp_tp", "fused_mlp_persistent", "linear_wave")


def load(dirs):
    out = {}
    for d in dirs:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            byd = defaultdict(dict)
            for r in csv.DictReader(open(f)):
                if any(e in r["Kernel_Name"] for e in ENGINE):
                    byd[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
                    byd[r["Dispatch_Id"]]["_k"] = r["Kernel_Name"]
            if byd:
                best = max(byd.values(), key=lambda x: max(v for k, v in x.items() if k != "_k"))
                out.update(best)
    return out


def main():
    steps = 20000
    engines = []
    for a in sys.argv[1:]:
        if a.startswith("--steps"):
            continue
        if a.isdigit():
            steps = int(a)
            continue
        name, dirs = a.split("=")
        engines.append((name, load(dirs.split(","))))
    keys = sorted({k for _, e in engines for k in e if k != "_k"})
    print("| counter (per DDP step, per wave) | " + " | ".join(n for n, _ in engines) + " |")
    print("|---|" + "---|" * len(engines))
    for k in keys:
        row = []
        for _, e in engines:
            waves = e.get("SQ_WAVES", 4) or 4
            v = e.get(k)
            row.append("" if v is None else (f"{v / waves:.0f} (x1)" if k == "SQ_WAVES" else f"{v / steps / waves:.1f}"))
        print(f"| {k} | " + " | ".join(row) + " |")
    for n, e in engines:
        wc = e.get("SQ_WAVE_CYCLES")
        if wc:
            parts = {k: e.get(k, 0) / wc for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")}
            mf = e.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (4 * wc)
            print(f"\n{n}: {e.get('_k', '')[:80]}\n  wave time: waiting {100 * parts['SQ_WAIT_ANY']:.0f}%, "
                  f"issue-stalled {100 * parts['SQ_WAIT_INST_ANY']:.0f}%, issuing {100 * parts['SQ_ACTIVE_INST_ANY']:.0f}%;"
                  f" MFMA busy {100 * mf:.0f}% of SIMD cycles")


if __name__ == "__main__":
    main()
