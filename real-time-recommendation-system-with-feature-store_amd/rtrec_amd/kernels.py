"""Torch-facing wrappers of the HIP C ABI (include/rtrec_hip.h).

Every function here launches hand-written gfx950 kernels from
librtrec_hip.so on torch's current stream; none has a CPU path (CPU tensors
raise). Shapes/dtypes are validated on the host before any launch so a bad
call never reaches the GPU.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import torch

from . import native
from .native import call, ptr, stream_of
from .profiling import TIMER

# ---------------------------------------------------------------------------
# workspace cache (grow-only, per device): no allocation inside hot calls
# ---------------------------------------------------------------------------
_WS = {}


def workspace(device: torch.device, nbytes: int, tag: str = "ws") -> torch.Tensor:
    key = (device.index if device.index is not None else torch.cuda.current_device(), tag)
    buf = _WS.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(max(nbytes, 256), dtype=torch.uint8, device=device)
        _WS[key] = buf
    return buf


# ---------------------------------------------------------------------------
# row gather (src/training/datasets/movielens.py:108-116; nn.Embedding lookup)
# ---------------------------------------------------------------------------

def gather_rows(table: torch.Tensor, ids: torch.Tensor, row_begin: int = 0,
                out: Optional[torch.Tensor] = None, oob: Optional[torch.Tensor] = None,
                check: bool = False) -> torch.Tensor:
    """``out[r] = table[ids[r] - row_begin]``; ids outside the table give zero rows
    (counted in ``oob`` if given). ``check=True`` raises IndexError on any
    out-of-range id like numpy fancy indexing (costs a device sync)."""
    native.require_device(table, ids, what="gather_rows")
    if ids.dtype != torch.int64:
        ids = ids.to(torch.int64)
    ids = ids.contiguous()
    table = table.contiguous()
    row_shape = table.shape[1:]
    row_bytes = table[0].numel() * table.element_size() if table.shape[0] > 0 else \
        int(torch.tensor(row_shape).prod()) * table.element_size()
    if out is None:
        out = torch.empty((ids.numel(),) + tuple(row_shape), dtype=table.dtype, device=table.device)
    if check and oob is None:
        oob = torch.zeros(1, dtype=torch.int32, device=table.device)
    with TIMER.region("gather_rows", bytes_=2.0 * ids.numel() * row_bytes + 8.0 * ids.numel()):
        call("rt_gather_rows", ptr(table), row_begin, table.shape[0], row_bytes, ptr(ids), ids.numel(),
             ptr(out), ptr(oob), stream_of(table))
    if check and int(oob.item()) != 0:
        raise IndexError(f"{int(oob.item())} ids out of range for table of {table.shape[0]} rows")
    return out.view(tuple(ids.shape) + tuple(row_shape))


def scatter_add_rows(grad_table: torch.Tensor, ids: torch.Tensor, grad_out: torch.Tensor,
                     padding_idx: int = -1) -> torch.Tensor:
    """nn.Embedding backward: grad_table[ids[r]] += grad_out[r] (padding_idx skipped)."""
    native.require_device(grad_table, ids, grad_out, what="scatter_add_rows")
    ids = ids.contiguous().to(torch.int64)
    grad_out = grad_out.contiguous().float()
    call("rt_scatter_add_rows_f32", ptr(grad_table), grad_table.shape[0], grad_table.shape[1], ptr(ids),
         ids.numel(), ptr(grad_out), padding_idx, stream_of(grad_table))
    return grad_table


# ---------------------------------------------------------------------------
# Faiss normalize_L2 + IndexFlatIP search (src/serving/retrieval.py:86,167,171)
# ---------------------------------------------------------------------------

def l2_renorm_(x: torch.Tensor) -> torch.Tensor:
    """In-place ``faiss.normalize_L2`` on fp32 rows."""
    native.require_device(x, what="l2_renorm_")
    if x.dtype != torch.float32 or not x.is_contiguous() or x.dim() != 2:
        raise ValueError("l2_renorm_ expects a contiguous fp32 [n, d] tensor")
    call("rt_l2_renorm_f32", ptr(x), x.shape[0], x.shape[1], stream_of(x))
    return x


def flatip_topk(queries: torch.Tensor, items: torch.Tensor, k: int,
                exclude_bits: Optional[torch.Tensor] = None, id_offset: int = 0,
                out: Optional[Tuple[torch.Tensor, torch.Tensor]] = None
                ) -> Tuple[torch.Tensor, torch.Tensor]:
    """Exact inner-product top-k: (scores [nq,k] f32, ids [nq,k] int64), ordered by
    (score desc, id asc); unfilled slots are (-FLT_MAX, -1)."""
    native.require_device(queries, items, what="flatip_topk")
    if queries.dim() != 2 or items.dim() != 2 or queries.shape[1] != items.shape[1]:
        raise ValueError(f"shape mismatch: queries {tuple(queries.shape)} items {tuple(items.shape)}")
    if queries.dtype != items.dtype:
        raise TypeError("queries and items must share a dtype")
    if k <= 0:
        raise ValueError("k must be positive")
    if k > TOPK_MAX_K:
        return _flatip_topk_wide(queries, items, k, exclude_bits, id_offset, out)
    queries = queries.contiguous()
    items = items.contiguous()
    nq, d = queries.shape
    nx = items.shape[0]
    dt = native.dtype_code(queries.dtype)
    if out is None:
        scores = torch.empty((nq, k), dtype=torch.float32, device=queries.device)
        ids = torch.empty((nq, k), dtype=torch.int64, device=queries.device)
    else:
        scores, ids = out
    if nq == 0:
        return scores, ids
    words = 0
    if exclude_bits is not None:
        exclude_bits = exclude_bits.contiguous()
        if exclude_bits.dtype not in (torch.int32, torch.uint32) or exclude_bits.shape[0] != nq:
            raise ValueError("exclude_bits must be int32/uint32 [nq, words]")
        words = exclude_bits.shape[1]
    nbytes = native.lib().rt_flatip_topk_workspace_bytes(nq, nx, d, dt, k)
    ws = workspace(queries.device, nbytes, "topk")
    with TIMER.region("flatip_topk", flops=2.0 * nq * nx * d,
                      bytes_=float((nq + nx) * d * queries.element_size() + nq * k * 12)):
        call("rt_flatip_topk", ptr(queries), nq, ptr(items) if nx else None, nx, d, dt, k, ptr(exclude_bits),
             words, id_offset, ptr(scores), ptr(ids), ptr(ws), ws.numel(), stream_of(queries))
    return scores, ids


TOPK_MAX_K = 512  # rt_flatip_topk: k <= 512 per launch (include/rtrec_hip.h)


def _flatip_topk_wide(queries, items, k, exclude_bits, id_offset, out):
    """k > 512 (faiss.IndexFlatIP.search takes any k, src/serving/retrieval.py:
    170-171): ceil(k/512) exact passes of rt_flatip_topk, each excluding every
    row the earlier passes returned (rt_exclusion_bitmap over their sorted ids,
    OR-ed with the caller's bitmap). Each pass returns the best remaining rows
    in (score desc, id asc) order, so the concatenation is the exact top-k in
    that order; slots past the corpus are (-FLT_MAX, -1)."""
    nq, nx = queries.shape[0], items.shape[0]
    dev = queries.device
    words = (nx + 31) // 32
    if exclude_bits is not None:
        exclude_bits = exclude_bits.contiguous()
        if exclude_bits.dtype not in (torch.int32, torch.uint32) or exclude_bits.shape[0] != nq:
            raise ValueError("exclude_bits must be int32/uint32 [nq, words]")
        if exclude_bits.shape[1] < words:
            raise ValueError("exclude_bits has fewer words than ceil(n_items / 32)")
    parts_s, parts_i = [], []
    found = None  # [nq, m] local row ids returned so far (-1 = none)
    left = k
    bits = exclude_bits
    while left > 0:
        kk = min(TOPK_MAX_K, left)
        ps, pi = flatip_topk(queries, items, kk, exclude_bits=bits, id_offset=id_offset)
        parts_s.append(ps)
        parts_i.append(pi)
        left -= kk
        if left <= 0:
            break
        loc = torch.where(pi >= 0, pi - id_offset, torch.full_like(pi, -1))
        found = loc if found is None else torch.cat([found, loc], dim=1)
        srt = found.sort(dim=1).values.to(torch.int32).contiguous()
        offs = torch.arange(nq + 1, dtype=torch.int64, device=dev) * srt.shape[1]
        new = exclusion_bitmap_csr(offs, srt.reshape(-1), nx)
        bits = new if exclude_bits is None else torch.bitwise_or(new, exclude_bits[:, :words].to(new.dtype))
    scores, ids = torch.cat(parts_s, dim=1), torch.cat(parts_i, dim=1)
    if out is not None:
        out[0].copy_(scores)
        out[1].copy_(ids)
        return out
    return scores, ids


# ---- corpus-sharded search with one corpus-wide threshold per query -------
def shard_sample_stride(n_total: int, nt: int = 128, max_stride: int = 64) -> int:
    """Sampling stride (in 128-row stages) for a corpus of ``n_total`` rows
    spread over shards: the planner's 64 when the corpus holds >= 32 x 64
    stages, else fewer, so that >= 32 stages are sampled in all."""
    stages = max(1, -(-int(n_total) // nt))
    return int(max(1, min(max_stride, stages // 32)))


def flatip_topk_shard_plan(nq: int, n_rows: int, d: int, dtype: torch.dtype, k: int, stride: int):
    """Host-only plan of a shard of ``n_rows`` rows (rt_flatip_topk_shard_plan):
    the (sampled, total) 128-row stage counts rt_flatip_topk_shard_sample would
    report, or None when the shape has no v4 plan. No device work, no sync."""
    counts = (ctypes.c_int64 * 2)()
    rc = native.lib().rt_flatip_topk_shard_plan(int(nq), int(n_rows), int(d), native.dtype_code(dtype), int(k),
                                                int(stride), ctypes.cast(counts, ctypes.c_void_p))
    if rc != 0:
        return None
    return int(counts[0]), int(counts[1])


def flatip_topk_shard_sample(queries: torch.Tensor, items: torch.Tensor, k: int, stride: int):
    """This shard's sample (rt_flatip_topk_shard_sample): per query the union
    of each lane half's 16 largest sampled group maxima [nq, 32] f32
    (descending; a subset of the 32 largest, so thresholds drawn from it are
    at or below the exact ones) and the (sampled, total) 128-row stage counts
    of the shard. None when the shape has no v4 plan (f16/bf16, d <= 128,
    k <= 128, >= 65,536 rows or forced)."""
    native.require_device(queries, items, what="flatip_topk_shard_sample")
    queries, items = queries.contiguous(), items.contiguous()
    nq, d = queries.shape
    dt = native.dtype_code(queries.dtype)
    lib = native.lib()
    nbytes = lib.rt_flatip_topk_shard_workspace_bytes(nq, items.shape[0], d, dt, k)
    if nbytes == 0:
        return None
    ws = workspace(queries.device, nbytes, "topk_shard")
    top = torch.empty((nq, 32), dtype=torch.float32, device=queries.device)
    counts = (ctypes.c_int64 * 2)()
    call("rt_flatip_topk_shard_sample", ptr(queries), nq, ptr(items), items.shape[0], d, dt, k, int(stride), ptr(top),
         ctypes.cast(counts, ctypes.c_void_p), ptr(ws), ws.numel(), stream_of(queries))
    return top, (int(counts[0]), int(counts[1]))


def topk_sample_rank(k: int, sampled: int, stages: int) -> int:
    """Failure-safe rank of a corpus-wide sample (rt_topk_sample_rank): P(the
    rank-th largest sampled group maximum exceeds the k-th score) < 1e-6;
    0 when no rank <= 32 is safe (search from -inf)."""
    r = ctypes.c_int(0)
    call("rt_topk_sample_rank", int(k), int(sampled), int(stages), ctypes.byref(r))
    return int(r.value)


def topk_sample_threshold(lists: torch.Tensor, rank: int) -> torch.Tensor:
    """thr [nq] = the rank-th largest of the union of lists [n_lists, nq, 32]
    (rt_topk_sample_threshold); -FLT_MAX when fewer finite entries."""
    native.require_device(lists, what="topk_sample_threshold")
    lists = lists.contiguous()
    n_lists, nq = lists.shape[0], lists.shape[1]
    thr = torch.empty(nq, dtype=torch.float32, device=lists.device)
    call("rt_topk_sample_threshold", ptr(lists), n_lists, nq, int(rank), ptr(thr), stream_of(lists))
    return thr


def flatip_topk_shard_search(queries: torch.Tensor, items: torch.Tensor, k: int, thr: torch.Tensor,
                             id_offset: int = 0) -> Tuple[torch.Tensor, torch.Tensor]:
    """This shard's rows scoring >= thr[q], the best k per query in (score desc,
    id asc) order, (-FLT_MAX, -1) padded (rt_flatip_topk_shard_search)."""
    native.require_device(queries, items, thr, what="flatip_topk_shard_search")
    queries, items, thr = queries.contiguous(), items.contiguous(), thr.contiguous().float()
    nq, d = queries.shape
    dt = native.dtype_code(queries.dtype)
    nbytes = native.lib().rt_flatip_topk_shard_workspace_bytes(nq, items.shape[0], d, dt, k)
    if nbytes == 0:
        raise native.RTError("rt_flatip_topk_shard_search", -2, "no v4 plan for this shape")
    ws = workspace(queries.device, nbytes, "topk_shard")
    scores = torch.empty((nq, k), dtype=torch.float32, device=queries.device)
    ids = torch.empty((nq, k), dtype=torch.int64, device=queries.device)
    with TIMER.region("flatip_topk", flops=2.0 * nq * items.shape[0] * d,
                      bytes_=float((nq + items.shape[0]) * d * queries.element_size() + nq * k * 12)):
        call("rt_flatip_topk_shard_search", ptr(queries), nq, ptr(items), items.shape[0], d, dt, k, ptr(thr),
             int(id_offset), ptr(scores), ptr(ids), ptr(ws), ws.numel(), stream_of(queries))
    return scores, ids


def topk_tuning(v4_mode: int = 0, v4_stride: int = 0, v4_rank: int = -1) -> None:
    """Planner override of flatip_topk (rt_flatip_topk_tuning; process-wide,
    results unchanged): v4_mode 0 automatic / 1 never / 2 wherever legal the
    sampled-threshold kernel pair (+4: per-split thresholds instead of one
    corpus-wide threshold per query; +8: small fp32 corpora keep the fused
    register-list scan instead of the score-slab GEMM + select); v4_stride the sample stride in 128-row stages
    (0 = planner); v4_rank the sampled rank (-1 = planner, 0 = no sample)."""
    call("rt_flatip_topk_tuning", int(v4_mode), int(v4_stride), int(v4_rank))


def l2_augment(x: torch.Tensor, role: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """[n, d] fp32 → [n, d+4] augmented rows for the L2 mode (rt_l2_augment_f32):
    role 0 (queries) appends 1, role 1 (items) appends -||x||^2/2."""
    native.require_device(x, what="l2_augment")
    if x.dtype != torch.float32 or x.dim() != 2:
        raise ValueError("l2_augment expects fp32 [n, d]")
    x = x.contiguous()
    n, d = x.shape
    if out is None:
        out = torch.empty((n, d + 4), dtype=torch.float32, device=x.device)
    call("rt_l2_augment_f32", ptr(x), n, d, ptr(out), out.shape[1], role, stream_of(x))
    return out


def flatl2_topk(q_aug: torch.Tensor, x_aug: torch.Tensor, d: int, k: int,
                exclude_bits: Optional[torch.Tensor] = None, id_offset: int = 0, verify: bool = True
                ) -> Tuple[torch.Tensor, torch.Tensor]:
    """Exact squared-L2 k-NN on augmented rows (IndexFlatL2.search): (distances
    [nq, k] ascending, ids [nq, k]); unfilled slots (FLT_MAX, -1). k + 32
    candidates are selected on the augmented inner product and re-ranked on
    Faiss's distance (rt_l2_finish_f32), which certifies every query: a query
    whose k-th distance is within a rounding bound of what an unselected item
    could reach (near-duplicate or clustered corpora) is re-selected with 512
    candidates. ``verify`` costs one device→host read (the flagged count);
    ``L2_STATS`` counts re-selected queries and any left uncertified (only
    possible when more than 512 - k items tie within rounding of the k-th)."""
    nq, nx = q_aug.shape[0], x_aug.shape[0]
    k_sel = min(k + L2_MARGIN, 512)
    s = torch.empty((nq, k), dtype=torch.float32, device=q_aug.device)
    i = torch.empty((nq, k), dtype=torch.int64, device=q_aug.device)
    if nq == 0:
        return s, i
    verify = verify and k_sel < nx  # a selection of the whole corpus is exact by construction
    flags = torch.empty(nq, dtype=torch.int32, device=q_aug.device) if verify else None

    def select_finish(q, bits, ksel, out_s, out_i, out_f):
        sel_s, sel = flatip_topk(q, x_aug, ksel, exclude_bits=bits, id_offset=id_offset)
        call("rt_l2_finish_f32", ptr(q), q.shape[1], ptr(x_aug), x_aug.shape[1], d, q.shape[0], ksel,
             ptr(sel), ptr(sel_s) if out_f is not None else None, k, ptr(out_s), ptr(out_i), ptr(out_f),
             id_offset, stream_of(q))

    select_finish(q_aug, exclude_bits, k_sel, s, i, flags)
    if verify:
        bad = torch.nonzero(flags).flatten()
        nb = bad.numel()
        left = 0
        if nb and k_sel < min(512, nx):
            qb = q_aug.index_select(0, bad).contiguous()
            bb = exclude_bits.index_select(0, bad).contiguous() if exclude_bits is not None else None
            s2 = torch.empty((nb, k), dtype=torch.float32, device=q_aug.device)
            i2 = torch.empty((nb, k), dtype=torch.int64, device=q_aug.device)
            k2 = min(512, nx)
            # a re-selection of the whole corpus is exact by construction: no certificate
            f2 = torch.empty(nb, dtype=torch.int32, device=q_aug.device) if k2 < nx else None
            select_finish(qb, bb, k2, s2, i2, f2)
            s.index_copy_(0, bad, s2)
            i.index_copy_(0, bad, i2)
            left = int(f2.sum().item()) if f2 is not None else 0
        elif nb:
            left = nb
        L2_STATS["reselected"] += nb if k_sel < min(512, nx) else 0
        L2_STATS["uncertified"] += left
    return s, i


L2_MARGIN = 32  # over-selected candidates per query in the L2 mode
L2_STATS = {"reselected": 0, "uncertified": 0}  # flatl2_topk certificate outcomes (process-wide)


def topk_merge(scores: torch.Tensor, ids: torch.Tensor, k_out: int
               ) -> Tuple[torch.Tensor, torch.Tensor]:
    """Merge candidate lists [n_lists, nq, k_in] into the (score desc, id asc) top k_out."""
    native.require_device(scores, ids, what="topk_merge")
    scores = scores.contiguous().float()
    ids = ids.contiguous().to(torch.int64)
    n_lists, nq, k_in = scores.shape
    os_ = torch.empty((nq, k_out), dtype=torch.float32, device=scores.device)
    oi = torch.empty((nq, k_out), dtype=torch.int64, device=scores.device)
    call("rt_topk_merge", ptr(scores), ptr(ids), nq, n_lists, k_in, k_out, ptr(os_), ptr(oi),
         stream_of(scores))
    return os_, oi


def exclusion_bitmap(n_queries: int, n_items: int, excluded, device) -> torch.Tensor:
    """int32 bitmap [nq, ceil(n_items/32)] (bit j of row q set ⇒ item j skipped for
    query q) from per-query excluded item lists — the train-item mask of
    scripts/evaluate_model.py:225-228. Host-side construction."""
    import numpy as np
    words = (n_items + 31) // 32
    mask = np.zeros((n_queries, words * 32), dtype=bool)
    for q, items in enumerate(excluded):
        sel = [int(i) for i in items if 0 <= int(i) < n_items]
        if sel:
            mask[q, sel] = True
    packed = np.packbits(mask, axis=1, bitorder="little")  # little-endian words: bit j = item j
    return torch.from_numpy(np.ascontiguousarray(packed).view(np.int32).copy()).to(device)


def exclusion_bitmap_csr(offsets: torch.Tensor, items: torch.Tensor, n_items: int,
                         rows: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Device exclusion bitmap (rt_exclusion_bitmap): row r masks the items of CSR
    row ``rows[r]`` (or r) — the train-item -inf mask of generate_recommendations
    (scripts/evaluate_model.py:224-228). int32 [n_rows, ceil(n_items/32)]."""
    native.require_device(offsets, items, what="exclusion_bitmap_csr")
    if offsets.dtype != torch.int64 or items.dtype != torch.int32:
        raise TypeError("CSR must be int64 offsets and int32 sorted items")
    n_csr = offsets.numel() - 1
    if rows is not None:
        rows = rows.contiguous().to(torch.int64)
    n_rows = rows.numel() if rows is not None else n_csr
    words = (n_items + 31) // 32
    if out is None:
        out = torch.empty((n_rows, words), dtype=torch.int32, device=offsets.device)
    call("rt_exclusion_bitmap", ptr(offsets), ptr(items), n_csr, ptr(rows), n_rows, n_items, ptr(out), words,
         stream_of(offsets))
    return out


def rank_metrics(preds: torch.Tensor, gt_offsets: torch.Tensor, gt_items: torch.Tensor, k_values,
                 gt_rows: Optional[torch.Tensor] = None, ex_offsets: Optional[torch.Tensor] = None,
                 ex_items: Optional[torch.Tensor] = None, ex_rows: Optional[torch.Tensor] = None,
                 num_items: int = 0):
    """Ranking metrics of Evaluator.evaluate (src/evaluation/metrics.py:248-319) on
    the device (rt_rank_metrics + rt_rank_metrics_reduce). Returns (per_row fp64
    [n, 4·n_k+2], valid int32 [n], summary fp64 [4·n_k+4] = column means over
    valid rows, n_valid, coverage)."""
    native.require_device(preds, gt_offsets, gt_items, what="rank_metrics")
    preds = preds.contiguous().to(torch.int64)
    if preds.dim() != 2:
        raise ValueError("preds must be [n_rows, list_len]")
    ks = [int(k) for k in k_values]
    if not ks or len(ks) > native.RT_METRICS_MAX_K or sorted(set(ks)) != ks or ks[0] <= 0:
        raise ValueError(f"k_values must be 1..{native.RT_METRICS_MAX_K} ascending positive ints")
    for t, dt in ((gt_offsets, torch.int64), (gt_items, torch.int32), (ex_offsets, torch.int64),
                  (ex_items, torch.int32)):
        if t is not None and t.dtype != dt:
            raise TypeError("CSR must be int64 offsets and int32 sorted items")
    n, L = preds.shape
    nk = len(ks)
    dev = preds.device
    per_row = torch.empty((n, 4 * nk + 2), dtype=torch.float64, device=dev)
    valid = torch.empty(n, dtype=torch.int32, device=dev)
    cov = torch.zeros((num_items + 31) // 32, dtype=torch.int32, device=dev) if num_items > 0 else None
    karr = (ctypes.c_int32 * nk)(*ks)
    st = stream_of(preds)
    rows = lambda t: None if t is None else t.contiguous().to(torch.int64)  # noqa: E731
    gt_rows, ex_rows = rows(gt_rows), rows(ex_rows)
    call("rt_rank_metrics", ptr(preds), n, L, ptr(gt_offsets), ptr(gt_items), ptr(gt_rows), gt_offsets.numel() - 1,
         ptr(ex_offsets), ptr(ex_items), ptr(ex_rows), (ex_offsets.numel() - 1) if ex_offsets is not None else 0,
         karr, nk, num_items, ptr(per_row), ptr(valid), ptr(cov), st)
    summary = torch.empty(4 * nk + 4, dtype=torch.float64, device=dev)
    call("rt_rank_metrics_reduce", ptr(per_row), ptr(valid), n, 4 * nk + 2, ptr(cov), num_items, ptr(summary), st)
    return per_row, valid, summary


def sample_negatives(pos_offsets: torch.Tensor, pos_items: torch.Tensor, users: torch.Tensor, num_items: int,
                     num_neg: int, seed: int, seed_offset: Optional[torch.Tensor] = None,
                     out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """[n, num_neg] int64 negatives per row (rt_sample_negatives): distinct, uniform
    over the items user ``users[r]`` has not interacted with (CSR positives)."""
    native.require_device(pos_offsets, pos_items, users, what="sample_negatives")
    if pos_offsets.dtype != torch.int64 or pos_items.dtype != torch.int32:
        raise TypeError("CSR must be int64 offsets and int32 sorted items")
    users = users.contiguous().to(torch.int64)
    n = users.numel()
    if out is None:
        out = torch.empty((n, num_neg), dtype=torch.int64, device=users.device)
    with TIMER.region("sample_negatives", bytes_=8.0 * n * (num_neg + 1)):
        call("rt_sample_negatives", ptr(pos_offsets), ptr(pos_items), pos_offsets.numel() - 1, ptr(users), n,
             num_items, num_neg, seed & 0xFFFFFFFFFFFFFFFF, ptr(seed_offset), ptr(out), stream_of(users))
    return out


def twotower_loss(u: torch.Tensor, p: torch.Tensor, q: Optional[torch.Tensor], temperature: float,
                  user_bias: Optional[torch.Tensor] = None, item_bias: Optional[torch.Tensor] = None,
                  explicit_weight: float = 0.7, in_batch_weight: float = 0.3, grad: bool = True):
    """Fused mixed loss (rt_twotower_loss_fwd_bwd / _fwd) on fp32, fp16 or bf16
    embeddings (widened to fp32 on load). Returns (loss fp64 [3] = (mixed,
    explicit, in-batch), du, dp, dq, d_user_bias, d_item_bias) — grads fp32 (None
    without ``grad``). q: [B*N, D] negatives (row i*N+j belongs to user i) or None."""
    native.require_device(u, p, what="twotower_loss")
    b, d = u.shape
    dt = native.dtype_code(u.dtype)
    if p.dtype != u.dtype or (q is not None and q.dtype != u.dtype):
        raise TypeError("u, p, q must share a dtype")
    u, p = u.contiguous(), p.contiguous()
    q = q.contiguous().reshape(-1, d) if q is not None else None
    n_neg = q.shape[0] // b if q is not None else 0
    dev = u.device
    loss = torch.zeros(3, dtype=torch.float64, device=dev)
    ws = workspace(dev, native.lib().rt_twotower_loss_workspace_bytes(b, d), "loss_k")
    f32 = dict(dtype=torch.float32, device=dev)
    st = stream_of(u)
    with TIMER.region("loss_fwd_bwd" if grad else "loss_fwd", flops=(6.0 if grad else 2.0) * b * b * d):
        if grad:
            du, dp = torch.empty((b, d), **f32), torch.empty((b, d), **f32)
            dq = torch.empty((q.shape[0], d), **f32) if q is not None else None
            dub = torch.zeros(1, **f32) if user_bias is not None else None
            dib = torch.zeros(1, **f32) if item_bias is not None else None
            call("rt_twotower_loss_fwd_bwd", ptr(u), ptr(p), ptr(q), dt, b, d, n_neg, 1.0 / temperature,
                 ptr(user_bias), ptr(item_bias), explicit_weight, in_batch_weight, ptr(loss), ptr(du), ptr(dp),
                 ptr(dq), ptr(dub), ptr(dib), ptr(ws), ws.numel(), st)
            return loss, du, dp, dq, dub, dib
        call("rt_twotower_loss_fwd", ptr(u), ptr(p), ptr(q), dt, b, d, n_neg, 1.0 / temperature, ptr(user_bias),
             ptr(item_bias), explicit_weight, in_batch_weight, ptr(loss), ptr(ws), ws.numel(), st)
        return loss, None, None, None, None, None


def inbatch_loss(u: torch.Tensor, p: torch.Tensor, temperature: float, label_offset: int = 0,
                 grad: bool = True):
    """In-batch CE of b local users against n_items in-batch items (label of user
    i = item label_offset + i) — rt_inbatch_loss_fwd_bwd. Returns (loss fp64 [3],
    du [b, D] fp32, dp [n_items, D] fp32); grads None without ``grad``."""
    native.require_device(u, p, what="inbatch_loss")
    if u.dtype != p.dtype:
        raise TypeError("u and p must share a dtype")
    u, p = u.contiguous(), p.contiguous()
    b, d = u.shape
    nx = p.shape[0]
    dev = u.device
    loss = torch.zeros(3, dtype=torch.float64, device=dev)
    ws = workspace(dev, native.lib().rt_inbatch_loss_workspace_bytes(b, nx, d), "inb")
    du = torch.empty((b, d), dtype=torch.float32, device=dev) if grad else None
    dp = torch.empty((nx, d), dtype=torch.float32, device=dev) if grad else None
    with TIMER.region("inbatch_loss", flops=(6.0 if grad else 2.0) * b * nx * d):
        call("rt_inbatch_loss_fwd_bwd", ptr(u), ptr(p), native.dtype_code(u.dtype), b, nx, d, label_offset,
             1.0 / temperature, ptr(loss), ptr(du), ptr(dp), ptr(ws), ws.numel(), stream_of(u))
    return loss, du, dp
