#!/usr/bin/env python3
"""Per-kernel PMC counter table from rocprofv3 --pmc result .db files.
Usage: python tools/pmc_dump.py <results.db>... [--filter substr]"""
import argparse
import sqlite3
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("dbs", nargs="+")
ap.add_argument("--filter", default="")
ap.add_argument("--calls", type=int, default=0,
                help="also print each counter summed over all dispatches / CALLS (per API call: "
                     "a call may launch a kernel more than once, e.g. the top-K main + rescue pairs)")
a = ap.parse_args()
agg = defaultdict(lambda: defaultdict(float))
cnt = defaultdict(lambda: defaultdict(set))
for db in a.dbs:
    c = sqlite3.connect(db)
    for name, ctr, val, disp, dur in c.execute(
            "select kernel_name, counter_name, value, dispatch_id, duration from counters_collection"):
        if a.filter and a.filter not in name:
            continue
        key = name.split("(")[0][:90]
        agg[key][ctr] += val
        cnt[key][ctr].add((db, disp))
for k, d in agg.items():
    print(k)
    for ctr in sorted(d):
        n = len(cnt[k][ctr])
        extra = f"   per call {d[ctr] / a.calls:.4g}" if a.calls else ""
        print(f"    {ctr:32s} {d[ctr] / n:16.4g}   (dispatches {n}){extra}")
