#!/usr/bin/env python3
"""C4 shard top-K (65,536 x 125,000 f16, d = 128) under a chosen planner mode,
for rocprofv3 traces / counter passes.
Usage: prof_topk_modes.py MODE K REPS [NX]   (MODE: 1 old kernels, 2 v4)"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "real-time-recommendation-system-with-feature-store_amd")]

import torch  # noqa: E402

from rtrec_amd import kernels  # noqa: E402

mode, k, reps = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
nx = int(sys.argv[4]) if len(sys.argv) > 4 else 125_000
g = torch.Generator(device="cuda").manual_seed(0)
q = torch.nn.functional.normalize(torch.randn(65536, 128, device="cuda", generator=g), dim=1).half()
x = torch.nn.functional.normalize(torch.randn(nx, 128, device="cuda", generator=g), dim=1).half()
kernels.topk_tuning(mode, 0, -1)
for _ in range(reps):
    kernels.flatip_topk(q, x, k)
torch.cuda.synchronize()
print("done", mode, k, reps, nx)
