"""ORACLE — test infrastructure only (see oracle/__init__.py).

ctypes front-end of ``oracle/flatip.c``: the CPU restatement of
``faiss.normalize_L2`` + ``faiss.IndexFlatIP.search`` (src/serving/retrieval.py:
70-197) and of the offline masked top-K of scripts/evaluate_model.py:217-232.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Optional, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle_flatip.so")
_lib = None

DTYPE_CODES = {np.dtype(np.float32): 0, np.dtype(np.float16): 1}
BF16 = "bf16"  # numpy has no bfloat16: pass uint16 bit patterns with dtype_code=2


def build() -> str:
    """Compile flatip.c with gcc (no reference sources involved)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = ctypes.CDLL(_LIB_PATH)
        _lib.orc_renorm_l2.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int]
        _lib.orc_renorm_l2.restype = None
        _lib.orc_flatip_search.argtypes = [
            ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
            ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        _lib.orc_flatip_search.restype = ctypes.c_int
        _lib.orc_topk_merge.argtypes = [
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
            ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        _lib.orc_topk_merge.restype = ctypes.c_int
        _lib.orc_flatl2_search.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                                           ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_int]
        _lib.orc_flatl2_search.restype = ctypes.c_int
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def normalize_L2(x: np.ndarray) -> None:
    """In-place ``faiss.normalize_L2`` restatement (retrieval.py:86,167,214)."""
    assert x.dtype == np.float32 and x.flags.c_contiguous and x.ndim == 2
    lib().orc_renorm_l2(_ptr(x), x.shape[0], x.shape[1])


def flat_ip_search(queries: np.ndarray, items: np.ndarray, k: int,
                   exclude_bits: Optional[np.ndarray] = None, id_offset: int = 0,
                   dtype_code: Optional[int] = None,
                   nthreads: int = 1) -> Tuple[np.ndarray, np.ndarray]:
    """Exact IndexFlatIP search (retrieval.py:171). Returns (scores [nq,k] f32,
    ids [nq,k] int64) ordered by (score desc, id asc); unfilled = (-FLT_MAX, -1).
    ``exclude_bits``: optional uint32 [nq, words] bitmap of items to skip
    (scripts/evaluate_model.py:225-228)."""
    q = np.ascontiguousarray(queries)
    x = np.ascontiguousarray(items)
    if dtype_code is None:
        dtype_code = DTYPE_CODES[q.dtype]
    nq, d = q.shape
    nx = x.shape[0]
    out_s = np.empty((nq, k), np.float32)
    out_i = np.empty((nq, k), np.int64)
    words = 0
    eb = None
    if exclude_bits is not None:
        eb = np.ascontiguousarray(exclude_bits, dtype=np.uint32)
        words = eb.shape[1]
    rc = lib().orc_flatip_search(_ptr(q), nq, _ptr(x), nx, d, dtype_code, k,
                                 _ptr(eb) if eb is not None else None, words, id_offset,
                                 _ptr(out_s), _ptr(out_i), nthreads)
    if rc != 0:
        raise RuntimeError(f"orc_flatip_search failed: {rc}")
    return out_s, out_i


def flat_l2_search(queries: np.ndarray, items: np.ndarray, k: int, nthreads: int = 1
                   ) -> Tuple[np.ndarray, np.ndarray]:
    """IndexFlatL2 search (retrieval.py:99-100, metric != "cosine"): squared L2
    distances ascending, ties by id ascending; unfilled = (FLT_MAX, -1)."""
    q = np.ascontiguousarray(queries, dtype=np.float32)
    x = np.ascontiguousarray(items, dtype=np.float32)
    nq, d = q.shape
    out_s = np.empty((nq, k), np.float32)
    out_i = np.empty((nq, k), np.int64)
    rc = lib().orc_flatl2_search(_ptr(q), nq, _ptr(x), x.shape[0], d, k, _ptr(out_s), _ptr(out_i), nthreads)
    if rc != 0:
        raise RuntimeError(f"orc_flatl2_search failed: {rc}")
    return out_s, out_i


def topk_merge(scores: np.ndarray, ids: np.ndarray, k_out: int) -> Tuple[np.ndarray, np.ndarray]:
    """Merge [n_lists, nq, k_in] candidate lists into the (score desc, id asc) top k_out."""
    s = np.ascontiguousarray(scores, dtype=np.float32)
    i = np.ascontiguousarray(ids, dtype=np.int64)
    n_lists, nq, k_in = s.shape
    out_s = np.empty((nq, k_out), np.float32)
    out_i = np.empty((nq, k_out), np.int64)
    rc = lib().orc_topk_merge(_ptr(s), _ptr(i), nq, n_lists, k_in, k_out, _ptr(out_s), _ptr(out_i))
    if rc != 0:
        raise RuntimeError(f"orc_topk_merge failed: {rc}")
    return out_s, out_i


def exclusion_bitmap(n_queries: int, n_items: int, excluded) -> np.ndarray:
    """Build the uint32 bitmap from per-query excluded item lists."""
    words = (n_items + 31) // 32
    bm = np.zeros((n_queries, words), np.uint32)
    for q, items in enumerate(excluded):
        for it in items:
            if 0 <= it < n_items:
                bm[q, it >> 5] |= np.uint32(1 << (it & 31))
    return bm


def argsort_topk(scores: np.ndarray, k: int, exclude=None) -> np.ndarray:
    """scripts/evaluate_model.py:221-232 restated: train items → -inf, then
    descending order, first k. Uses a stable (score desc, id asc) order instead
    of numpy's unstable quicksort so ties are deterministic."""
    s = scores.astype(np.float32, copy=True)
    if exclude is not None:
        for q, items in enumerate(exclude):
            s[q, [it for it in items if it < s.shape[1]]] = -np.inf
    order = np.lexsort((np.broadcast_to(np.arange(s.shape[1]), s.shape), -s), axis=1)
    return order[:, :k]


def dot_fma(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Sequential fmaf-chain dot products of rows (float64 emulation is exact for
    dyadic inputs only; general bit-exact scores come from flatip.c)."""
    return (a.astype(np.float64) @ b.astype(np.float64).T).astype(np.float32)


def sample_rank(k: int, sampled: int, stages: int) -> int:
    """Restatement of rt_topk_sample_rank (csrc/topk_api.hip): the smallest
    rank r <= 32 with P(Bin(k, f) >= r) <= 1e-6 for f = sampled / stages
    (0 when none), the failure bound of a threshold taken as the r-th largest
    sampled group maximum."""
    import math
    f = sampled / stages

    def log_tail(r):
        if r > k:
            return -1e300
        terms = [math.lgamma(k + 1) - math.lgamma(i + 1) - math.lgamma(k - i + 1) + i * math.log(f) +
                 ((k - i) * math.log1p(-f) if f < 1 else (0.0 if i == k else -1e300)) for i in range(r, k + 1)]
        mx = max(terms)
        return mx + math.log(sum(math.exp(t - mx) for t in terms))
    for r in range(1, 33):
        if log_tail(r) <= math.log(1e-6):
            return r
    return 0


def shard_sample(queries: np.ndarray, shard: np.ndarray, stride: int, nt: int = 128, group: int = 16):
    """CPU stand-in of rt_flatip_topk_shard_sample for the orchestration tests:
    per query the 32 largest maxima of 16-row groups over every stride-th
    nt-row stage of the shard (exact float64 scores of dyadic data), -inf
    padded, and the (sampled, total) stage counts. Any grouping gives the
    same failure bound (a group maximum above the k-th score needs a top-k
    row in the group)."""
    n = shard.shape[0]
    stages = -(-n // nt)
    rows = np.concatenate([np.arange(v * nt, min(n, (v + 1) * nt)) for v in range(0, stages, stride)]) \
        if n else np.zeros(0, np.int64)
    sc = queries.astype(np.float64) @ shard[rows].astype(np.float64).T  # [nq, m]
    m = sc.shape[1]
    pad = (-m) % group
    sc = np.concatenate([sc, np.full((sc.shape[0], pad), -np.inf)], axis=1)
    gmax = sc.reshape(sc.shape[0], -1, group).max(axis=2)
    top = -np.sort(-gmax, axis=1)[:, :32]
    if top.shape[1] < 32:
        top = np.concatenate([top, np.full((top.shape[0], 32 - top.shape[1]), -np.inf)], axis=1)
    return top.astype(np.float32), (len(range(0, stages, stride)), stages)
