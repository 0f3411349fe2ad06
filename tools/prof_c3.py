#!/usr/bin/env python3
"""Flat-IP top-K on the C3 serving shape (6,040 queries x 3,416 fp32 rows,
d=128, k=10) for rocprofv3 kernel traces. Usage: prof_c3.py [reps] [k]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "real-time-recommendation-system-with-feature-store_amd")]

import torch  # noqa: E402

from rtrec_amd import kernels  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
k = int(sys.argv[2]) if len(sys.argv) > 2 else 10
g = torch.Generator(device="cuda").manual_seed(7)
q = torch.nn.functional.normalize(torch.randn(6040, 128, device="cuda", generator=g), dim=1)
x = torch.nn.functional.normalize(torch.randn(3416, 128, device="cuda", generator=g), dim=1)
for _ in range(reps):
    kernels.flatip_topk(q, x, k)
torch.cuda.synchronize()
print("done", reps, k)
