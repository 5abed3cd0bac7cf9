#!/usr/bin/env python3
"""Summarise a rocprofv3 ``--stats --output-format csv`` kernel_stats.csv into markdown."""
import csv
import sys


def main(path, title, top=15, steps=None):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    out = [f"### {title}", "", f"source: `{path}` (rocprofv3 --kernel-trace --stats)", "",
           "| kernel | calls | total us | avg us | % |", "|---|---:|---:|---:|---:|"]
    for r in rows[:top]:
        name = r["Name"].replace("|", "/")[:110]
        out.append(f"| `{name}` | {r['Calls']} | {float(r['TotalDurationNs'])/1e3:.1f} | "
                   f"{float(r['AverageNs'])/1e3:.2f} | {float(r['Percentage']):.1f} |")
    out.append(f"\ntotal kernel time {tot/1e3:.1f} us over {sum(int(r['Calls']) for r in rows)} launches")
    if steps:
        out.append(f"; {tot/1e3/steps:.2f} us of kernel time per step ({steps} steps incl. warmup/capture)")
    print("\n".join(out) + "\n")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], steps=int(sys.argv[3]) if len(sys.argv) > 3 else None)
