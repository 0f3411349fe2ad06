#!/usr/bin/env python3
"""Flat-IP top-K on the C4 shard shape (65,536 queries x 125,000 fp16 rows,
d=128) for rocprofv3 kernel-trace / counter runs. Usage: prof_topk.py [k] [reps]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "real-time-recommendation-system-with-feature-store_amd")]

import torch  # noqa: E402

from rtrec_amd import kernels  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 100
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
g = torch.Generator(device="cuda").manual_seed(0)
q = torch.nn.functional.normalize(torch.randn(65536, 128, device="cuda", generator=g), dim=1).half()
x = torch.nn.functional.normalize(torch.randn(125000, 128, device="cuda", generator=g), dim=1).half()
for _ in range(reps):
    kernels.flatip_topk(q, x, k)
torch.cuda.synchronize()
print("done", k, reps)
