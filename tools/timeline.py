#!/usr/bin/env python3
"""Per-step timeline of a rocprofv3 kernel trace (csv): steps are delimited by
the optimizer kernel; prints wall span, GPU-busy union (any kernel running),
idle gaps and the busiest kernels of the median step.
Usage: python tools/timeline.py <kernel_trace.csv> [--marker clip_adam_kernel]"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("--marker", default="clip_adam_kernel")
    a = ap.parse_args()
    rows = []
    with open(a.src) as f:
        for d in csv.DictReader(f):
            rows.append((int(d["Start_Timestamp"]), int(d["End_Timestamp"]), d["Kernel_Name"].split("(")[0],
                         d.get("Queue_Id", "?")))
    rows.sort()
    ends = [e for s, e, n, q in rows if a.marker in n]
    steps = []
    for i in range(1, len(ends)):
        ks = [r for r in rows if ends[i - 1] < r[1] <= ends[i]]
        steps.append((ends[i - 1], ends[i], ks))
    out = []
    for t0, t1, ks in steps:
        iv = sorted((max(s, t0), e) for s, e, _, _ in ks)
        busy, cur_s, cur_e = 0, None, None
        for s, e in iv:
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        if cur_e is not None:
            busy += cur_e - cur_s
        out.append(((t1 - t0) / 1e3, busy / 1e3, len(ks), ks))
    out.sort(key=lambda x: x[0])
    med = out[len(out) // 2]
    print(f"steps={len(out)}  median wall {med[0]:.1f} us  busy {med[1]:.1f} us  idle {med[0] - med[1]:.1f} us  "
          f"kernels/step {med[2]}")
    ks = sorted(med[3])
    base = ks[0][0]
    for s, e, n, q in ks:
        print(f"  q{q:>3} {(s - base) / 1e3:8.1f} +{(e - s) / 1e3:6.1f}  {n[:90]}")


if __name__ == "__main__":
    main()
