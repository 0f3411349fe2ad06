#!/usr/bin/env python3
"""Interleaved A/B of librtrec_hip.so variants on the C3 top-10 (6,040 x 3,416 x
128 fp32), one subprocess per variant (RTREC_HIP_LIB). GPU box.
Usage: python tools/ab_topk_c3.py ROUNDS lib1.so lib2.so ..."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import sys, torch
sys.path[:0] = [%r, %r]
from rtrec_amd import kernels
g = torch.Generator(device="cuda").manual_seed(0)
q = torch.nn.functional.normalize(torch.randn(6040, 128, device="cuda", generator=g), dim=1)
x = torch.nn.functional.normalize(torch.randn(3416, 128, device="cuda", generator=g), dim=1)
for _ in range(20): kernels.flatip_topk(q, x, 10)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(200): kernels.flatip_topk(q, x, 10)
e1.record(); torch.cuda.synchronize()
print(e0.elapsed_time(e1) / 200)
""" % (REPO, os.path.join(REPO, "real-time-recommendation-system-with-feature-store_amd"))

if __name__ == "__main__":
    rounds = int(sys.argv[1])
    for r in range(rounds):
        for lib in sys.argv[2:]:
            env = dict(os.environ, RTREC_HIP_LIB=os.path.join(REPO, lib))
            out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=120)
            if out.returncode:
                print(out.stderr[-2000:])
                sys.exit(1)
            print(json.dumps({"lib": lib, "round": r, "ms": float(out.stdout.strip().splitlines()[-1])}), flush=True)
