#!/usr/bin/env python3
"""Summarise a rocprofv3 database (``*_results.db``, rocpd schema) as markdown.

``python tools/rocpd_summary.py gpurun_out/prof12/drv_results.db [--match NAME] [--timeline N]``

* per-kernel table: calls, total/avg/min/max us, share, VGPR/SGPR/LDS/scratch;
* ``--timeline N``: the last N dispatches (start offset, duration, stream, queue),
  e.g. to read the timed region of a bench run or the overlap of two streams;
* ``--overlap A B``: total time kernels matching A run concurrently with kernels
  matching B (interval intersection, across streams) -- the comm/compute overlap
  measure for the DDP reducer traces.
"""
from __future__ import annotations

import argparse
import re
import sqlite3


def _short(name: str, width: int = 80) -> str:
    name = re.sub(r"\(ptdt::.*$", "", name)
    name = name.replace("void ", "").replace("ptdt::(anonymous namespace)::", "")
    return name if len(name) <= width else name[: width - 3] + "..."


def load(db: str):
    c = sqlite3.connect(db)
    cols = ("name", "start", "end", "duration", "stream_id", "queue_id", "vgpr_count", "accum_vgpr_count",
            "sgpr_count", "lds_size", "scratch_size", "grid_x", "workgroup_x")
    rows = c.execute(f"select {','.join(cols)} from kernels order by start").fetchall()
    return [dict(zip(cols, r)) for r in rows]


def table(rows, match=None) -> str:
    agg: dict[str, dict] = {}
    for r in rows:
        if match and not re.search(match, r["name"]):
            continue
        a = agg.setdefault(r["name"], {"n": 0, "tot": 0, "min": 1 << 62, "max": 0, "r": r})
        a["n"] += 1
        a["tot"] += r["duration"]
        a["min"] = min(a["min"], r["duration"])
        a["max"] = max(a["max"], r["duration"])
    total = sum(a["tot"] for a in agg.values()) or 1
    out = ["| kernel | calls | total us | avg us | min us | max us | % | vgpr/agpr/sgpr | lds | scratch |",
           "|---|---|---|---|---|---|---|---|---|---|"]
    for name, a in sorted(agg.items(), key=lambda kv: -kv[1]["tot"]):
        r = a["r"]
        out.append(f"| `{_short(name)}` | {a['n']} | {a['tot'] / 1e3:.1f} | {a['tot'] / a['n'] / 1e3:.2f} | "
                   f"{a['min'] / 1e3:.2f} | {a['max'] / 1e3:.2f} | {100 * a['tot'] / total:.1f} | "
                   f"{r['vgpr_count']}/{r['accum_vgpr_count']}/{r['sgpr_count']} | {r['lds_size']} | "
                   f"{r['scratch_size']} |")
    return "\n".join(out)


def timeline(rows, n: int, match=None) -> str:
    sel = [r for r in rows if not match or re.search(match, r["name"])][-n:]
    if not sel:
        return ""
    t0 = sel[0]["start"]
    out = ["| t+us | dur us | stream | queue | kernel |", "|---|---|---|---|---|"]
    for r in sel:
        out.append(f"| {(r['start'] - t0) / 1e3:.1f} | {r['duration'] / 1e3:.2f} | {r['stream_id']} | "
                   f"{r['queue_id']} | `{_short(r['name'], 60)}` |")
    return "\n".join(out)


def overlap_ns(rows, pat_a: str, pat_b: str) -> tuple[int, int, int]:
    """(ns of A, ns of B, ns where an A kernel and a B kernel run at the same time)."""
    A = [(r["start"], r["end"]) for r in rows if re.search(pat_a, r["name"])]
    B = [(r["start"], r["end"]) for r in rows if re.search(pat_b, r["name"])]

    def merge(iv):
        iv = sorted(iv)
        out = []
        for s, e in iv:
            if out and s <= out[-1][1]:
                out[-1][1] = max(out[-1][1], e)
            else:
                out.append([s, e])
        return out

    ma, mb = merge(A), merge(B)
    i = j = 0
    inter = 0
    while i < len(ma) and j < len(mb):
        s, e = max(ma[i][0], mb[j][0]), min(ma[i][1], mb[j][1])
        if s < e:
            inter += e - s
        if ma[i][1] < mb[j][1]:
            i += 1
        else:
            j += 1
    return sum(e - s for s, e in ma), sum(e - s for s, e in mb), inter


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--match", default=None)
    ap.add_argument("--timeline", type=int, default=0)
    ap.add_argument("--overlap", nargs=2, default=None, metavar=("A", "B"))
    a = ap.parse_args()
    rows = load(a.db)
    print(table(rows, a.match))
    if a.timeline:
        print()
        print(timeline(rows, a.timeline, a.match))
    if a.overlap:
        ta, tb, ti = overlap_ns(rows, *a.overlap)
        print(f"\nbusy(A={a.overlap[0]!r}) = {ta / 1e3:.1f} us, busy(B={a.overlap[1]!r}) = {tb / 1e3:.1f} us, "
              f"concurrent = {ti / 1e3:.1f} us ({100 * ti / max(ta, 1):.1f}% of A)")


if __name__ == "__main__":
    main()
