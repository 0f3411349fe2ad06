"""C-ABI boundary checks that need no GPU: librtrec_hip.so loads, exports every
entry point include/rtrec_hip.h declares, the ctypes mirror matches the C
struct layouts (compiled here with gcc from the header), host-only queries
answer, argument errors come back as rt_status codes, and the product path
refuses CPU tensors instead of falling back."""
import ctypes
import re
import subprocess

import pytest
import torch

from conftest import PKG, REPO

HEADER = REPO / "include" / "rtrec_hip.h"


@pytest.fixture(scope="module")
def native():
    from rtrec_amd import native as nat
    if not (PKG / "lib" / "librtrec_hip.so").exists():
        subprocess.run(["make", "-s", "-j8", "-C", str(PKG)], check=True)
    nat.lib()
    return nat


def _declared():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+char\s*\*|int|size_t)\s+(rt_\w+)\s*\(", text, flags=re.M)))


def test_every_declared_symbol_is_exported(native):
    declared = _declared()
    assert len(declared) >= 17, declared
    handle = native.lib()
    missing = [n for n in declared if not hasattr(handle, n)]
    assert not missing, missing
    assert not native.MISSING
    # the ctypes signature table covers the header one-to-one
    assert sorted(native.SIGNATURES) == declared


def test_abi_version_and_status_strings(native):
    assert native.lib().rt_abi_version() >= 1
    for code in (0, -1, -2, -3, -4):
        assert native.lib().rt_status_string(code)
    assert native.lib().rt_last_error() is not None


_LAYOUT_C = r"""
#include <stdio.h>
#include <stddef.h>
#include "rtrec_hip.h"
#define F(T, f) printf(#T " " #f " %zu\n", offsetof(T, f));
int main(void) {
  printf("rt_linear_fwd_args size %zu\n", sizeof(rt_linear_fwd_args));
  printf("rt_linear_bwd_args size %zu\n", sizeof(rt_linear_bwd_args));
  %FIELDS%
  return 0;
}
"""


def test_ctypes_struct_layout_matches_header(native, tmp_path):
    lines = []
    for cname, cls in (("rt_linear_fwd_args", native.LinearFwdArgs), ("rt_linear_bwd_args", native.LinearBwdArgs)):
        for fname, _ in cls._fields_:
            lines.append(f"F({cname}, {fname})")
    src = tmp_path / "layout.c"
    src.write_text(_LAYOUT_C.replace("%FIELDS%", "\n  ".join(lines)))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", str(REPO / "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    got = {}
    for ln in out:
        if ln:
            t, f, v = ln.split()
            got[(t, f)] = int(v)
    assert got[("rt_linear_fwd_args", "size")] == ctypes.sizeof(native.LinearFwdArgs)
    assert got[("rt_linear_bwd_args", "size")] == ctypes.sizeof(native.LinearBwdArgs)
    for cname, cls in (("rt_linear_fwd_args", native.LinearFwdArgs), ("rt_linear_bwd_args", native.LinearBwdArgs)):
        for fname, _ in cls._fields_:
            assert got[(cname, fname)] == getattr(cls, fname).offset, (cname, fname)


def test_host_only_queries(native):
    L = native.lib()
    # workspace sizes are pure host arithmetic: monotone in the problem size
    a = L.rt_flatip_topk_workspace_bytes(1024, 4096, 128, 0, 10)
    b = L.rt_flatip_topk_workspace_bytes(65536, 4096, 128, 0, 100)
    assert 0 < a <= b
    assert L.rt_twotower_loss_workspace_bytes(1024, 128) > 0


def test_argument_errors_are_status_codes(native):
    L = native.lib()
    assert L.rt_linear_fwd_f32(None, None) == -1
    assert L.rt_linear_bwd_f32(None, None) == -1
    args = native.LinearFwdArgs()
    args.m, args.k, args.n = 4, 8, 1024           # n > 512: valid but unsupported
    args.src = args.w = ctypes.c_void_p(16)
    args.ld_src = 8
    assert L.rt_linear_fwd_f32(ctypes.byref(args), None) == -2
    with pytest.raises(native.RTError):
        native.call("rt_linear_fwd_f32", None, None)


def test_product_path_refuses_cpu_tensors(native):
    from rtrec_amd import kernels
    t = torch.zeros(4, 8)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        kernels.gather_rows(t, torch.zeros(2, dtype=torch.int64))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        kernels.flatip_topk(t, t, 2)


def test_ctypes_argument_counts_match_header(native):
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    protos = re.findall(r"^\s*(?:const\s+char\s*\*|int|size_t)\s+(rt_\w+)\s*\(([^;]*?)\)\s*;", text, flags=re.M | re.S)
    assert protos
    for name, params in protos:
        params = params.strip()
        n = 0 if params in ("", "void") else params.count(",") + 1
        assert len(native.SIGNATURES[name][1]) == n, (name, n, len(native.SIGNATURES[name][1]))


def test_sample_rank_matches_binomial_tail(native):
    """rt_topk_sample_rank (host-only) is the least rank r <= 32 with
    P(Bin(k, f) >= r) <= 1e-6 for f = sampled / stages (r > k: safe; 0 when
    none fits) — the failure bound of the v4 sampled threshold
    (topk_api.hip::safe_rank), checked against scipy's binomial tail."""
    from scipy.stats import binom
    L = native.lib()
    for k in (1, 10, 33, 64, 100, 128):
        for stages in (64, 977, 7813):
            for sampled in sorted(x for x in {1, 4, 16, 31, 62, 124, stages // 2, stages} if x <= stages):
                r = ctypes.c_int(-1)
                assert L.rt_topk_sample_rank(k, sampled, stages, ctypes.byref(r)) == 0
                f = sampled / stages
                want = next((rr for rr in range(1, 33) if rr > k or binom.sf(rr - 1, k, f) <= 1e-6), 0)
                assert r.value == want, (k, sampled, stages, r.value, want)


def test_shard_plan_is_cheap_on_the_host(native):
    """The v4 plan runs on the host path of every search call: after the first
    call of a shape its (stride, rank) come from a memo (a per-(stride, rank)
    log-sum-exp tail once cost ~1.7 ms per call)."""
    import time
    L = native.lib()
    counts = (ctypes.c_int64 * 2)()
    args = (ctypes.c_int64(65536), ctypes.c_int64(125000), 128, 1, 100, 64, ctypes.cast(counts, ctypes.c_void_p))
    assert L.rt_flatip_topk_shard_plan(*args) == 0
    assert list(counts) == [16, 977]
    t0 = time.perf_counter()
    for _ in range(200):
        L.rt_flatip_topk_shard_plan(*args)
    assert (time.perf_counter() - t0) / 200 < 1e-3  # loose: CPU-contended runners
