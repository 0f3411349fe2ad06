#!/usr/bin/env python3
"""Micro-benchmark of rt_flatip_topk on the C3 / C4-shard shapes and k sweeps
(GPU box): separates the MFMA scan from the selection cost.
Usage: python tools/microbench_topk.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "real-time-recommendation-system-with-feature-store_amd")]

import torch  # noqa: E402

from rtrec_amd import kernels  # noqa: E402

PEAK = {torch.float32: 157.3e12, torch.float16: 2.5e15, torch.bfloat16: 2.5e15}


def run(nq, nx, d, k, dt, reps=5):
    g = torch.Generator(device="cuda").manual_seed(0)
    q = torch.randn(nq, d, device="cuda", generator=g)
    x = torch.randn(nx, d, device="cuda", generator=g)
    q = torch.nn.functional.normalize(q, dim=1).to(dt)
    x = torch.nn.functional.normalize(x, dim=1).to(dt)
    kernels.flatip_topk(q, x, k)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        kernels.flatip_topk(q, x, k)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    fl = 2.0 * nq * nx * d
    print(f"nq={nq:6d} nx={nx:7d} d={d} k={k:3d} {str(dt):14s} {ms:8.3f} ms  {nq / ms * 1e3:12.0f} QPS  "
          f"{fl / ms / 1e9:8.1f} TF/s  {100 * fl / ms / 1e-3 / PEAK[dt]:5.1f}% peak", flush=True)


if __name__ == "__main__":
    for k in (1, 10, 100):
        run(6040, 3416, 128, k, torch.float32)
    for k in (1, 10, 100):
        run(65536, 125000, 128, k, torch.float16, reps=2)
    run(65536, 125000, 128, 100, torch.bfloat16, reps=2)
    run(8192, 1000000, 128, 100, torch.float16, reps=2)
