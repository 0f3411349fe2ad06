#!/usr/bin/env python3
"""rt_gather_rows on the C5 shard shape (bench.py extras.gather_c5: bf16 rows of
256 from a 12.5M-row table, 16,777,216 random ids) for rocprofv3 kernel-trace /
FETCH_SIZE / WRITE_SIZE passes. Usage: prof_gather.py [reps]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "real-time-recommendation-system-with-feature-store_amd")]

import torch  # noqa: E402

from rtrec_amd import kernels  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
g = torch.Generator(device="cuda").manual_seed(7)
rows = 12_500_000
table = torch.empty((rows, 256), dtype=torch.bfloat16, device="cuda")
table.view(torch.int16).random_(-30000, 30000, generator=g)
ids = torch.randint(0, rows, (16_777_216,), device="cuda", generator=g)
out = torch.empty((ids.numel(), 256), dtype=torch.bfloat16, device="cuda")
for _ in range(reps):
    kernels.gather_rows(table, ids, out=out)
torch.cuda.synchronize()
print("done", reps)
