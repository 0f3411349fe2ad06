#!/usr/bin/env python3
"""In-batch CE (rt_inbatch_loss_fwd_bwd) on the C5 shape: B=8192 users x 8192
items, D=256, bf16 (and the fp32 / C2 shapes for comparison). Algorithmic
FLOPs: forward 2·B·N·D, forward+backward 6·B·N·D (S, dU, dP).
Usage: python tools/microbench_inbatch.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "real-time-recommendation-system-with-feature-store_amd")]

import torch  # noqa: E402

from rtrec_amd import kernels  # noqa: E402

PEAK = {torch.float32: 157.3e12, torch.float16: 2.5e15, torch.bfloat16: 2.5e15}


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def run(b, nx, d, dt, reps=10):
    g = torch.Generator(device="cuda").manual_seed(0)
    u = (torch.randn(b, d, device="cuda", generator=g) * 0.06).to(dt)
    p = (torch.randn(nx, d, device="cuda", generator=g) * 0.06).to(dt)
    for grad in (False, True):
        ms = timed(lambda: kernels.inbatch_loss(u, p, 0.05, grad=grad), reps)
        fl = (6.0 if grad else 2.0) * b * nx * d
        print(f"b={b:5d} n={nx:5d} d={d} {str(dt):14s} {'fwd+bwd' if grad else 'fwd    '} {ms:8.3f} ms "
              f"{fl / ms / 1e9:8.1f} TF/s  {100 * fl / ms / 1e-3 / PEAK[dt]:5.1f}% peak", flush=True)


if __name__ == "__main__":
    run(8192, 8192, 256, torch.bfloat16)
    if "--c5" in sys.argv:
        sys.exit(0)
    run(8192, 8192, 256, torch.float16)
    run(1024, 8192, 256, torch.bfloat16)
    run(8192, 8192, 256, torch.float32, reps=3)
    run(1024, 1024, 128, torch.float32)
