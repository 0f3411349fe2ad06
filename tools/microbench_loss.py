#!/usr/bin/env python3
"""Micro-benchmark of the fused C2 loss (rt_twotower_loss_fwd_bwd) at the C2
shape (B = 1024, N = 16, D = 128, fp32): the full mixed loss, the in-batch term
alone and the explicit term alone, so the two launches' time splits between the
in-batch scores and the explicit negatives. Per-kernel times: run it under
`rocprofv3 --kernel-trace --stats`.
Usage: python tools/microbench_loss.py"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "real-time-recommendation-system-with-feature-store_amd")]

import torch  # noqa: E402

from rtrec_amd import native  # noqa: E402
from rtrec_amd.native import call  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    lib = native.lib()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    b, n, d = 1024, 16, 128
    g = torch.Generator(device="cuda").manual_seed(0)
    u = torch.nn.functional.normalize(torch.randn(b, d, device=dev, generator=g), dim=1)
    p = torch.nn.functional.normalize(torch.randn(b, d, device=dev, generator=g), dim=1)
    q = torch.nn.functional.normalize(torch.randn(b * n, d, device=dev, generator=g), dim=1)
    loss = torch.zeros(3, dtype=torch.float64, device=dev)
    du, dp = torch.empty(b, d, device=dev), torch.empty(b, d, device=dev)
    dq = torch.empty(b * n, d, device=dev)
    ws = torch.empty(lib.rt_twotower_loss_workspace_bytes(b, d), dtype=torch.uint8, device=dev)
    P = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
    reps = int(os.environ.get("REPS", "200"))
    for label, qq, nn, we, wb in [("full", q, n, 0.7, 0.3), ("in-batch only", None, 0, 0.0, 1.0),
                                  ("explicit only", q, n, 0.7, 0.0)]:
        def fn():
            call("rt_twotower_loss_fwd_bwd", P(u), P(p), P(qq), 0, b, d, nn, 20.0, None, None, we, wb,
                 P(loss), P(du), P(dp), P(dq) if qq is not None else None, None, None, P(ws), ws.numel(), st)
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        print(f"{label:14s} fwd+bwd {e0.elapsed_time(e1) / reps * 1e3:7.1f} us (2 launches)", flush=True)


if __name__ == "__main__":
    main()
