#!/usr/bin/env python3
"""Dispatch order of graph replays in a rocprofv3 kernel trace (benchmarks/graph_memset_probe.py
--trace_only): the replays are the dispatches between the ``philox_kernel`` marker dispatches. For every
memset blit (``__amd_rocclr_fillBuffer*``) of a replay it prints its queue, its time window, and
every dispatch that STARTED before the blit ENDED (on any queue) among the next dispatches in
graph order -- a dependent kernel starting before its memset finished is the race the graph-replay
divergence needs.

usage: graph_replay_order.py run_kernel_trace.csv [--after N]
"""
import csv
import sys


def main():
    path = sys.argv[1]
    after = int(sys.argv[sys.argv.index("--after") + 1]) if "--after" in sys.argv else 6
    ks = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, k in enumerate(ks) if "philox_kernel" in k["Kernel_Name"]]
    print(f"{len(ks)} dispatches, {len(marks)} philox markers")
    marks = marks[-3:]  # the probe's three markers bracket its two replays (earlier philox: input init)
    for r in range(len(marks) - 1):
        win = ks[marks[r] + 1:marks[r + 1]]
        t0 = int(win[0]["Start_Timestamp"]) if win else 0
        queues = sorted({k["Queue_Id"] for k in win})
        fills = [i for i, k in enumerate(win) if "fillBuffer" in k["Kernel_Name"]]
        print(f"\n== replay {r}: {len(win)} dispatches on queues {queues}, {len(fills)} memset blits")
        for i in fills:
            f = win[i]
            fs, fe = int(f["Start_Timestamp"]), int(f["End_Timestamp"])
            early = [k for k in win[i + 1:i + 200] if int(k["Start_Timestamp"]) < fe]
            print(f"  blit #{i} q{f['Queue_Id']} [{(fs - t0) / 1e3:9.2f}, {(fe - t0) / 1e3:9.2f}] us  "
                  f"grid {f['Grid_Size_X']}  started before it ended: {len(early)}")
            for k in early[:after]:
                print(f"      q{k['Queue_Id']} [{(int(k['Start_Timestamp']) - t0) / 1e3:9.2f}, "
                      f"{(int(k['End_Timestamp']) - t0) / 1e3:9.2f}] {k['Kernel_Name'][:90]}")
            nxt = win[i + 1:i + 1 + 3]
            for k in nxt:
                print(f"      next: q{k['Queue_Id']} [{(int(k['Start_Timestamp']) - t0) / 1e3:9.2f}] {k['Kernel_Name'][:90]}")


if __name__ == "__main__":
    main()
