#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter_collection.csv files into a markdown table.

Per kernel (matching --filter), the mean of each counter over its dispatches, plus
derived ratios when their inputs are present:
  wait_frac     = SQ_WAIT_ANY / SQ_WAVE_CYCLES        (waves parked on s_waitcnt / barrier)
  issue_stall   = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES   (waves with an instruction blocked)
  lds_conflict  = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
Usage: pmc_summary.py TITLE FILTER csv [csv ...]
"""
import collections
import csv
import sys


def main(title, filt, paths):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in paths:
        for r in csv.DictReader(open(p)):
            name = r["Kernel_Name"]
            if filt and not any(f in name for f in filt.split("|")):
                continue
            short = name.replace("(anonymous namespace)", "anon").replace("void ", "").split("(")[0][:90]
            agg[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = [f"### {title}", ""]
    for k, d in agg.items():
        m = {c: sum(v) / len(v) for c, v in d.items()}
        n = max(len(v) for v in d.values())
        out.append(f"**`{k}`** ({n} dispatches, mean per dispatch)")
        out.append("")
        out.append("| counter | value |")
        out.append("|---|---:|")
        for c in sorted(m):
            out.append(f"| {c} | {m[c]:,.0f} |")
        ratios = []
        if "SQ_WAIT_ANY" in m and m.get("SQ_WAVE_CYCLES"):
            ratios.append(("wait_frac (SQ_WAIT_ANY / SQ_WAVE_CYCLES)", m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"]))
        if "SQ_WAIT_INST_ANY" in m and m.get("SQ_WAVE_CYCLES"):
            ratios.append(("issue_stall (SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES)", m["SQ_WAIT_INST_ANY"] / m["SQ_WAVE_CYCLES"]))
        if "SQ_LDS_BANK_CONFLICT" in m and m.get("SQ_LDS_IDX_ACTIVE"):
            ratios.append(("lds_conflict (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE)",
                           m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"]))
        for name, v in ratios:
            out.append(f"| *{name}* | {v:.3f} |")
        out.append("")
    print("\n".join(out))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3:])
