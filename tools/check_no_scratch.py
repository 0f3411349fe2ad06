#!/usr/bin/env python3
"""Fail if any kernel whose name matches a pattern spills VGPRs to scratch.
Kernels that hold untracked inline-asm load destinations (the 16-bit Flat-IP
top-K, csrc/topk_v2.h) must keep them in registers.
Usage: check_no_scratch.py <hipcc -Rpass-analysis=kernel-resource-usage log> <name regex>"""
import re
import sys

log, pat = sys.argv[1], sys.argv[2]
name, bad = None, []
for line in open(log):
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        name = m.group(1)
        continue
    m = re.search(r"VGPRs Spill: (\d+)", line)
    if m and name and re.search(pat, name) and int(m.group(1)) > 0:
        bad.append((name, int(m.group(1))))
if bad:
    for n, b in bad:
        print(f"ERROR: {n} spills {b} VGPRs (untracked loads must stay in registers)")
    sys.exit(1)
print(f"check_no_scratch: no VGPR spills in kernels matching '{pat}'")
