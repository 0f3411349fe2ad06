#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace (``--kernel-trace`` .db or
``kernel_stats.csv``/``kernel_trace.csv``) into a per-kernel table
(calls, total/avg/min/max µs, share) for profiles/.

Usage: python tools/prof_summary.py <results.db | kernel_trace.csv> [--out profiles/x.md]
"""
import argparse
import csv
import sqlite3
import sys
from collections import defaultdict


def from_db(path, by_grid=False, by_base=False):
    c = sqlite3.connect(path)
    cols = [d[0] for d in c.execute("select * from kernels limit 1").description]
    gcols = [g for g in cols if "grid" in g.lower()] if by_grid else []
    q = "select name, duration" + "".join(f", {g}" for g in gcols) + " from kernels"
    rows = []
    for r in c.execute(q).fetchall():
        name = r[0]
        if by_grid or by_base:
            name = name.split("(")[0]
        if by_base:
            name = name.split("<")[0].replace("void ", "")
        if gcols:
            name += " " + " ".join(f"{g}={v}" for g, v in zip(gcols, r[2:]))
        rows.append((name, r[1]))
    return rows


def from_csv(path, by_grid=False, by_base=False):
    rows = []
    with open(path) as f:
        r = csv.DictReader(f)
        for d in r:
            name = d.get("Kernel_Name") or d.get("KernelName") or d.get("Name")
            name = name.split("(")[0] if (by_grid or by_base) else name
            if by_base:  # one row per kernel family: template arguments dropped
                name = name.split("<")[0].replace("void ", "")
            if by_grid and "Grid_Size_X" in d:
                name += " grid=%sx%sx%s" % (d["Grid_Size_X"], d["Grid_Size_Y"], d["Grid_Size_Z"])
            if "Start_Timestamp" in d:
                dur = int(d["End_Timestamp"]) - int(d["Start_Timestamp"])
            else:
                dur = int(float(d.get("DurationNs") or d.get("duration")))
            rows.append((name, dur))
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("--out")
    ap.add_argument("--title", default="rocprofv3 --kernel-trace summary")
    ap.add_argument("--by-grid", action="store_true", help="one row per (kernel, grid size) = per launch shape")
    ap.add_argument("--by-base", action="store_true", help="one row per kernel family (all template instances)")
    ap.add_argument("--seq", type=int, default=0, help="instead: the last SEQ dispatches in start order (.db only)")
    a = ap.parse_args()
    if a.seq:
        c = sqlite3.connect(a.src)
        cols = [d[0] for d in c.execute("select * from kernels limit 1").description]
        order = "start" if "start" in cols else "rowid"
        gx = [g for g in cols if g.lower() in ("grid_x", "grid_size_x", "grid_size")][:1]
        se = ", start, end" if ("start" in cols and "end" in cols) else ""
        q = f"select name, duration{', ' + gx[0] if gx else ''}{se} from kernels order by {order}"
        rows = c.execute(q).fetchall()[-a.seq:]
        prev_end = None
        for r in rows:
            gap = ""
            if se:
                st, en = r[-2], r[-1]
                if prev_end is not None:
                    gap = f"gap {(st - prev_end) / 1e3:7.1f} us  "
                prev_end = en
            grid = ("grid " + str(r[2])) if gx else ""
            print(f"{gap}{r[1] / 1e3:10.1f} us  {r[0].split('(')[0][:90]}  {grid}")
        return
    rows = from_db(a.src, a.by_grid, a.by_base) if a.src.endswith(".db") else from_csv(a.src, a.by_grid, a.by_base)
    agg = defaultdict(list)
    for name, dur in rows:
        agg[name].append(dur)
    total = sum(sum(v) for v in agg.values())
    lines = [f"# {a.title}", "", f"source: `{a.src}`", "",
             "| kernel | calls | total ms | avg µs | min µs | max µs | share |",
             "|---|---:|---:|---:|---:|---:|---:|"]
    for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        s = sum(v)
        nm = name.replace("|", "\\|")
        if len(nm) > 110:
            nm = nm[:107] + "..."
        lines.append(f"| `{nm}` | {len(v)} | {s / 1e6:.3f} | {s / len(v) / 1e3:.1f} | {min(v) / 1e3:.1f} | "
                     f"{max(v) / 1e3:.1f} | {100.0 * s / max(total, 1):.1f}% |")
    text = "\n".join(lines) + "\n"
    if a.out:
        with open(a.out, "w") as f:
            f.write(text)
    sys.stdout.write(text)


if __name__ == "__main__":
    main()
