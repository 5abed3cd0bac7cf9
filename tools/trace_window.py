#!/usr/bin/env python3
"""Per-kernel stats over the LAST window of a rocprofv3 kernel trace.

Autotuning (MIOpen find) and warmup dominate a whole-run ``--stats`` table; this
keeps only dispatches that start within the final ``--ms`` milliseconds of the
trace (the timed steady-state steps) and prints a markdown table.

    python tools/trace_window.py gpurun_out/prof_resnet/run_kernel_trace.csv --ms 272 --title "..." [--top 25]
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--ms", type=float, required=True, help="window length before the last kernel end")
    ap.add_argument("--title", default="steady-state window")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--steps", type=int, default=None, help="steps inside the window (per-step column)")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    end = max(int(r["End_Timestamp"]) for r in rows)
    t0 = end - int(a.ms * 1e6)
    agg = collections.defaultdict(lambda: [0, 0])
    busy = 0
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s < t0:
            continue
        agg[r["Kernel_Name"]][0] += 1
        agg[r["Kernel_Name"]][1] += e - s
        busy += e - s
    items = sorted(agg.items(), key=lambda kv: -kv[1][1])
    print(f"### {a.title}\n\nsource: `{a.trace}`, dispatches starting in the last {a.ms:g} ms "
          f"(kernel busy {busy / 1e6:.2f} ms = {100 * busy / (a.ms * 1e6):.1f}% of the window)\n")
    per = f" | us/step" if a.steps else ""
    print(f"| kernel | calls | total us | avg us | %{per} |\n|---|---:|---:|---:|---:|" + ("---:|" if a.steps else ""))
    for name, (n, t) in items[: a.top]:
        extra = f" | {t / 1e3 / a.steps:.1f}" if a.steps else ""
        print(f"| `{name.replace('|', '/')[:100]}` | {n} | {t / 1e3:.1f} | {t / 1e3 / n:.2f} | {100 * t / busy:.1f}{extra} |")
    rest = sum(t for _, (n, t) in items[a.top:])
    print(f"\n{len(items)} distinct kernels; the rest: {rest / 1e3:.1f} us")


if __name__ == "__main__":
    main()
