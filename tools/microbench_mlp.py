#!/usr/bin/env python3
"""Micro-benchmark of the fused tower-MLP kernels in isolation (GPU box).

Times rt_linear_fwd_f32 / rt_linear_bwd_f32 for the C2 tower shapes with and
without the BN/dropout prologue, to attribute the per-launch cost.
Usage: python tools/microbench_mlp.py
"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "real-time-recommendation-system-with-feature-store_amd")]

import torch  # noqa: E402

from rtrec_amd import native  # noqa: E402
from rtrec_amd.native import LinearBwdArgs, LinearFwdArgs, call  # noqa: E402


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


def main():
    dev = torch.device("cuda:0")
    native.lib()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    print(f"{'case':44s} {'us':>8s} {'TF/s':>7s}")
    for (m, k, n) in [(1024, 256, 128), (16384, 256, 128), (16384, 20, 256), (16384, 128, 128), (1024, 3, 256)]:
        src = torch.randn(m, k, device=dev)
        w = torch.randn(n, k, device=dev) * 0.05
        b = torch.zeros(n, device=dev)
        z = torch.empty(m, n, device=dev)
        S = 16  # RT_STAT_SLOTS
        stats_prev = torch.zeros(S * 2 * k, dtype=torch.float64, device=dev)
        stats_prev[:k] = 0.1 * m
        stats_prev[k:2 * k] = 1.0 * m
        gam = torch.ones(k, device=dev)
        bet = torch.zeros(k, device=dev)
        rm = torch.zeros(k, device=dev)
        rv = torch.ones(k, device=dev)
        sm = torch.empty(k, device=dev)
        si = torch.empty(k, device=dev)
        stats = torch.zeros(S * 2 * n, dtype=torch.float64, device=dev)
        for label, mode, drop, want_stats in [("raw", 0, 0.0, False), ("raw+stats", 0, 0.0, True),
                                              ("bn-train", 1, 0.0, True), ("bn-train+drop", 1, 0.2, True)]:
            a = LinearFwdArgs()
            a.src, a.src_rows, a.ld_src, a.m, a.k, a.n = src.data_ptr(), m, k, m, k, n
            a.w, a.bias, a.z_out, a.act = w.data_ptr(), b.data_ptr(), z.data_ptr(), 0
            a.prev_mode, a.prev_act = mode, 0
            if mode == 1:
                a.prev_stats, a.bn_gamma, a.bn_beta = stats_prev.data_ptr(), gam.data_ptr(), bet.data_ptr()
                a.running_mean, a.running_var = rm.data_ptr(), rv.data_ptr()
                a.save_mean, a.save_invstd = sm.data_ptr(), si.data_ptr()
                a.bn_eps, a.bn_momentum = 1e-5, 0.1
            a.drop_p, a.drop_seed = drop, 7
            if want_stats:
                a.stats_out = stats.data_ptr()
            us = timeit(lambda: call("rt_linear_fwd_f32", ctypes.byref(a), st))
            print(f"fwd m={m:5d} k={k:3d} n={n:3d} {label:14s} {us:8.1f} {2 * m * k * n / us / 1e6:7.2f}")
        # backward (hidden-layer form: BN-train grad, dA with stats)
        g = torch.randn(m, n, device=dev)
        dz = torch.empty(m, n, device=dev)
        dw = torch.zeros(n, k, device=dev)
        db = torch.zeros(n, device=dev)
        gst = torch.zeros(S * 2 * n, dtype=torch.float64, device=dev)
        gprev = torch.empty(m, k, device=dev)
        gprev_st = torch.zeros(S * 2 * k, dtype=torch.float64, device=dev)
        smn = torch.zeros(n, device=dev)
        sin = torch.ones(n, device=dev)
        gn = torch.ones(n, device=dev)
        dgn = torch.zeros(n, device=dev)
        dbn = torch.zeros(n, device=dev)
        for label, want_da in [("dz+dW", False), ("dz+dA+dW", True)]:
            a = LinearBwdArgs()
            a.m, a.k, a.n, a.w, a.dw, a.dbias, a.dz_ws = m, k, n, w.data_ptr(), dw.data_ptr(), db.data_ptr(), dz.data_ptr()
            a.grad_mode, a.g, a.z, a.act = 1, g.data_ptr(), z.data_ptr(), 0
            a.g_stats, a.save_mean, a.save_invstd, a.bn_gamma = gst.data_ptr(), smn.data_ptr(), sin.data_ptr(), gn.data_ptr()
            a.dgamma, a.dbeta = dgn.data_ptr(), dbn.data_ptr()
            a.src, a.src_rows, a.ld_src = src.data_ptr(), m, k
            a.prev_mode, a.prev_act = 1, 0
            a.prev_mean, a.prev_invstd, a.prev_gamma, a.prev_beta = sm.data_ptr(), si.data_ptr(), gam.data_ptr(), bet.data_ptr()
            if want_da:
                a.g_prev, a.g_prev_stats = gprev.data_ptr(), gprev_st.data_ptr()
            us = timeit(lambda: call("rt_linear_bwd_f32", ctypes.byref(a), st))
            fl = (4 if want_da else 2) * m * k * n
            print(f"bwd m={m:5d} k={k:3d} n={n:3d} {label:14s} {us:8.1f} {fl / us / 1e6:7.2f}")


def fwd_epilogues():
    """The C2 step's forward shapes (m = 18,432, BN-train + dropout prologue,
    two BN segments) with each epilogue: raw z, z + next-BN stats, and the
    final layer's row L2 normalisation."""
    dev = torch.device("cuda:0")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    S = 16
    m, seg = 18432, 1024
    for (k, n) in [(256, 128), (128, 128)]:
        src = torch.randn(m, k, device=dev)
        w = torch.randn(n, k, device=dev) * 0.05
        b = torch.zeros(n, device=dev)
        z = torch.empty(m, n, device=dev)
        out = torch.empty(m, n, device=dev)
        norms = torch.empty(m, device=dev)
        stats_prev = torch.zeros(2 * S * 2 * k, dtype=torch.float64, device=dev)
        stats_prev.view(2, S, 2, k)[:, 0, 0] = 0.1 * m
        stats_prev.view(2, S, 2, k)[:, 0, 1] = 1.0 * m
        gam, bet = torch.ones(k, device=dev), torch.zeros(k, device=dev)
        rm, rv = torch.zeros(k, device=dev), torch.ones(k, device=dev)
        sm, si = torch.empty(2 * k, device=dev), torch.empty(2 * k, device=dev)
        stats = torch.zeros(2 * S * 2 * n, dtype=torch.float64, device=dev)
        for label in ("z", "z+stats", "l2norm", "two-seg z+stats", "two-seg l2norm"):
            a = LinearFwdArgs()
            a.src, a.src_rows, a.ld_src, a.m, a.k, a.n = src.data_ptr(), m, k, m, k, n
            a.w, a.bias, a.act = w.data_ptr(), b.data_ptr(), 0
            a.prev_mode, a.prev_act = 1, 0
            a.prev_stats, a.bn_gamma, a.bn_beta = stats_prev.data_ptr(), gam.data_ptr(), bet.data_ptr()
            a.running_mean, a.running_var = rm.data_ptr(), rv.data_ptr()
            a.save_mean, a.save_invstd = sm.data_ptr(), si.data_ptr()
            a.bn_eps, a.bn_momentum = 1e-5, 0.1
            a.drop_p, a.drop_seed = 0.2, 7
            if label.startswith("two-seg"):
                a.seg_split = seg
            if label.endswith("l2norm"):
                a.l2_out, a.norms_out = out.data_ptr(), norms.data_ptr()
            else:
                a.z_out = z.data_ptr()
                if "stats" in label:
                    a.stats_out = stats.data_ptr()
            us = timeit(lambda: call("rt_linear_fwd_f32", ctypes.byref(a), st))
            print(f"fwd m={m} k={k:3d} n={n:3d} {label:18s} {us:8.1f} us {2 * m * k * n / us / 1e6:7.2f} TF/s")


def fwd_attr():
    """Attribution of the hidden-layer forward (k = 256 -> n = 128): prologue
    mode x epilogue x row count, so the fixed per-launch cost, the BN/dropout
    prologue and the stats epilogue separate."""
    dev = torch.device("cuda:0")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    S = 16
    k, n = 256, 128
    tiny = torch.zeros(64, device=dev)
    print(f"launch floor (64-element fill) {timeit(lambda: tiny.zero_()):8.1f} us")
    for m in (8192, 16384, 18432, 24576):
        src = torch.randn(m, k, device=dev)
        w = torch.randn(n, k, device=dev) * 0.05
        b = torch.zeros(n, device=dev)
        z = torch.empty(m, n, device=dev)
        stats_prev = torch.zeros(2 * S * 2 * k, dtype=torch.float64, device=dev)
        stats_prev.view(2, S, 2, k)[:, 0, 0] = 0.1 * m
        stats_prev.view(2, S, 2, k)[:, 0, 1] = 1.0 * m
        gam, bet = torch.ones(k, device=dev), torch.zeros(k, device=dev)
        rm, rv = torch.zeros(k, device=dev), torch.ones(k, device=dev)
        sm, si = torch.empty(2 * k, device=dev), torch.empty(2 * k, device=dev)
        stats = torch.zeros(2 * S * 2 * n, dtype=torch.float64, device=dev)
        for label, mode, drop, want_stats in [("raw", 0, 0.0, False), ("raw+stats", 0, 0.0, True),
                                              ("bn", 1, 0.0, False), ("bn-eval", 2, 0.0, False),
                                              ("bn+drop", 1, 0.2, False), ("bn+drop+stats", 1, 0.2, True)]:
            a = LinearFwdArgs()
            a.src, a.src_rows, a.ld_src, a.m, a.k, a.n = src.data_ptr(), m, k, m, k, n
            a.w, a.bias, a.z_out, a.act = w.data_ptr(), b.data_ptr(), z.data_ptr(), 0
            a.prev_mode, a.prev_act = mode, 0
            if mode:
                a.prev_stats, a.bn_gamma, a.bn_beta = stats_prev.data_ptr(), gam.data_ptr(), bet.data_ptr()
                a.running_mean, a.running_var = rm.data_ptr(), rv.data_ptr()
                a.save_mean, a.save_invstd = sm.data_ptr(), si.data_ptr()
                a.bn_eps, a.bn_momentum = 1e-5, 0.1
                a.seg_split = 1024
            a.drop_p, a.drop_seed = drop, 7
            if want_stats:
                a.stats_out = stats.data_ptr()
            us = timeit(lambda: call("rt_linear_fwd_f32", ctypes.byref(a), st))
            print(f"fwd m={m:5d} blocks={m // 32:4d} {label:14s} {us:8.1f} us {2 * m * k * n / us / 1e6:7.2f} TF/s")


def split_bwd():
    """dz and dW launches timed separately at the C2 item-tower shapes (17,408
    rows), hidden-layer form, with and without the dropout prologue."""
    dev = torch.device("cuda:0")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    S = 16
    shapes = [(17408, 128, 128), (17408, 256, 128), (17408, 20, 256)]
    if "--k" in sys.argv:
        kk = int(sys.argv[sys.argv.index("--k") + 1])
        shapes = [t for t in shapes if t[1] == kk]
    for (m, k, n) in shapes:
        src = torch.randn(m, k, device=dev)
        w = torch.randn(n, k, device=dev) * 0.05
        g = torch.randn(m, n, device=dev)
        z = torch.randn(m, n, device=dev)
        dz = torch.empty(m, n, device=dev)
        dw = torch.zeros(n, k, device=dev)
        db = torch.zeros(n, device=dev)
        gst = torch.zeros(2 * S * 2 * n, dtype=torch.float64, device=dev)
        gprev = torch.empty(m, k, device=dev)
        gprev_st = torch.zeros(2 * S * 2 * k, dtype=torch.float64, device=dev)
        one_n, zero_n = torch.ones(2 * n, device=dev), torch.zeros(2 * n, device=dev)
        one_k, zero_k = torch.ones(2 * k, device=dev), torch.zeros(2 * k, device=dev)
        for drop in ((0.2,) if "--k" in sys.argv else (0.0, 0.2)):
            a = LinearBwdArgs()
            a.m, a.k, a.n, a.w, a.dw, a.dbias, a.dz_ws = m, k, n, w.data_ptr(), dw.data_ptr(), db.data_ptr(), dz.data_ptr()
            a.grad_mode, a.g, a.z, a.act = 1, g.data_ptr(), z.data_ptr(), 0
            a.g_stats, a.save_mean, a.save_invstd, a.bn_gamma = gst.data_ptr(), zero_n.data_ptr(), one_n.data_ptr(), one_n.data_ptr()
            a.dgamma, a.dbeta = zero_n.data_ptr(), zero_n.data_ptr()
            a.src, a.src_rows, a.ld_src = src.data_ptr(), m, k
            a.seg_split = 1024
            if k != 20:
                a.prev_mode, a.prev_act, a.prev_drop_p, a.prev_drop_seed = 1, 0, drop, 3
                a.prev_mean, a.prev_invstd = zero_k.data_ptr(), one_k.data_ptr()
                a.prev_gamma, a.prev_beta = one_k.data_ptr(), zero_k.data_ptr()
                a.g_prev, a.g_prev_stats = gprev.data_ptr(), gprev_st.data_ptr()
            t_dz = timeit(lambda: call("rt_linear_bwd_dz_f32", ctypes.byref(a), st))
            t_dw = timeit(lambda: call("rt_linear_bwd_dw_f32", ctypes.byref(a), st))
            print(f"m={m} k={k:3d} n={n:3d} drop={drop:.1f}  dz {t_dz:7.1f} us  dw {t_dw:7.1f} us  "
                  f"(dA {2 * m * k * n / t_dz / 1e6:6.2f} TF/s, dW {2 * m * k * n / t_dw / 1e6:6.2f} TF/s)")


if __name__ == "__main__":
    if "--split" in sys.argv:
        native.lib()
        split_bwd()
    elif "--fwd-epi" in sys.argv:
        native.lib()
        fwd_epilogues()
    elif "--fwd-attr" in sys.argv:
        native.lib()
        fwd_attr()
    else:
        main()
