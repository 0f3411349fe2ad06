"""GPU parity of the 16-bit Flat-IP top-K path (f16/bf16, k <= 128: the
radix-compacted candidate-buffer kernel, csrc/topk_v2.h) against the CPU oracle
(oracle/flatip.c = faiss.IndexFlatIP.search semantics, src/serving/retrieval.py:
141-197).

Inputs are dyadic (entries j/64, |j| <= 64): exactly representable in f16 and
bf16, and every partial sum of a d <= 256 dot product is exact in fp32, so the
MFMA summation order cannot change a score and the comparison is bit-exact —
indices included, with the lower id winning exact ties as in Faiss. Corpora
are large enough that every query's candidate buffer is compacted several
times (> 480 items per split), and the tie-heavy cases drive the exact-sort
fallback of the compaction."""
import numpy as np
import pytest
import torch

from oracle import flat_ip as orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def K():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from rtrec_amd import kernels, native
    native.lib()
    return kernels


def _dyadic(rng, n, d, lo=-64, hi=64):
    return (rng.integers(lo, hi + 1, size=(n, d)) / 64.0).astype(np.float32)


def _check(K, q, x, k, dtype, exclude=None, id_offset=0):
    bm_np = None
    bm = None
    if exclude is not None:
        bm_np = orc.exclusion_bitmap(q.shape[0], x.shape[0], exclude)
        bm = K.exclusion_bitmap(q.shape[0], x.shape[0], exclude, "cuda")
    rs, ri = orc.flat_ip_search(q, x, k, exclude_bits=bm_np, id_offset=id_offset, nthreads=8)
    gs, gi = K.flatip_topk(torch.from_numpy(q).to(dtype).cuda(), torch.from_numpy(x).to(dtype).cuda(), k,
                           exclude_bits=bm, id_offset=id_offset)
    gi = gi.cpu().numpy()
    gs = gs.cpu().numpy()
    bad = np.nonzero((gi != ri).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} rows differ, first {bad[:5]}: got {gi[bad[0]][:8]} want {ri[bad[0]][:8]}"
    assert np.array_equal(gs, rs)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("nq,nx,d,k", [(300, 20000, 128, 100), (257, 9001, 128, 10), (64, 30000, 128, 128),
                                       (33, 5000, 128, 1), (100, 12345, 64, 50), (70, 7000, 256, 100),
                                       (1, 3000, 128, 100), (40, 2500, 96, 64)])
def test_topk16_dyadic_bit_exact(K, dtype, nq, nx, d, k):
    rng = np.random.default_rng(nq * 7 + nx + d + k)
    _check(K, _dyadic(rng, nq, d), _dyadic(rng, nx, d), k, dtype)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_topk16_fewer_items_than_k(K, dtype):
    rng = np.random.default_rng(1)
    _check(K, _dyadic(rng, 45, 128), _dyadic(rng, 37, 128), 100, dtype)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_topk16_massive_exact_ties(K, dtype):
    """40 distinct rows repeated over 12,000 items: thousands of exact ties per
    score, so the radix prefix cannot shrink a buffer and the exact-sort
    fallback (strict threshold, lower id wins) must reproduce Faiss order."""
    rng = np.random.default_rng(2)
    base = _dyadic(rng, 40, 128)
    x = base[rng.integers(0, 40, size=12000)]
    _check(K, _dyadic(rng, 96, 128), x, 100, dtype)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_topk16_coarse_scores(K, dtype):
    """Small-integer entries: scores take few distinct values (heavy ties at
    every rank)."""
    rng = np.random.default_rng(3)
    q = _dyadic(rng, 80, 64, -1, 1)
    x = _dyadic(rng, 8000, 64, -1, 1)
    _check(K, q, x, 128, dtype)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_topk16_exclusion_and_offset(K, dtype):
    rng = np.random.default_rng(4)
    q = _dyadic(rng, 130, 128)
    x = _dyadic(rng, 6000, 128)
    excl = [rng.choice(6000, int(rng.integers(0, 2000)), replace=False) for _ in range(130)]
    _check(K, q, x, 100, dtype, exclude=excl, id_offset=1_000_000)


@pytest.mark.parametrize("k", [100, 10])
def test_topk16_c4_shard_properties(K, k):
    """C4 shard shape at full size (65,536 queries x 125,000 fp16 rows; k=100
    runs the v4 sampled-threshold pair — presample, threshold, scan, finish —
    k=10 the v3 scan): size-independent checks — sorted
    (score desc, id asc), ids distinct and in range, scores equal to the fp32
    dot of the returned rows (recomputed on the device), and a 512-query sample
    bit-exact against the oracle."""
    g = torch.Generator(device="cuda").manual_seed(11)
    nq, nx, d = 65536, 125000, 128
    q = torch.randint(-64, 65, (nq, d), device="cuda", generator=g).half() / 64
    x = torch.randint(-64, 65, (nx, d), device="cuda", generator=g).half() / 64
    gs, gi = K.flatip_topk(q, x, k)
    torch.cuda.synchronize()
    assert (gi >= 0).all() and (gi < nx).all()
    assert (gs[:, :-1] >= gs[:, 1:]).all()
    tie = gs[:, :-1] == gs[:, 1:]
    assert (gi[:, :-1][tie] < gi[:, 1:][tie]).all()
    srt = gi.sort(dim=1).values
    assert (srt[:, 1:] != srt[:, :-1]).all()
    rows = x.float()[gi[:4096]]                       # [4096, k, d]
    dots = torch.einsum("qkd,qd->qk", rows, q[:4096].float())
    assert torch.equal(dots, gs[:4096])
    sel = torch.randperm(nq, generator=torch.Generator().manual_seed(0))[:512].numpy()
    qs = q.float().cpu().numpy()[sel]
    rs, ri = orc.flat_ip_search(np.ascontiguousarray(qs), x.float().cpu().numpy(), k, nthreads=16)
    assert np.array_equal(gi.cpu().numpy()[sel], ri)
    assert np.array_equal(gs.cpu().numpy()[sel], rs)


# ---- the sampled-threshold kernel pair (csrc/topk_v4.h) --------------------
@pytest.fixture
def V4(K):
    """Force the v4 scan + finish pair on shapes the planner would give to
    v2/v3 (small corpora, any k <= 128), with the given sample; restored after."""
    def set_(stride=0, rank=-1, mode=2):
        K.topk_tuning(mode, stride, rank)
    yield set_
    K.topk_tuning(0, 0, -1)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("nq,nx,d,k", [(700, 40000, 128, 100), (300, 20000, 64, 40), (129, 30011, 128, 128),
                                       (600, 25000, 96, 10), (64, 9000, 128, 1)])
def test_topk16_v4_dyadic_bit_exact(K, V4, dtype, nq, nx, d, k):
    """Planner's (stride, rank) for the split; several splits merged by the
    finish pass; ragged last stage (nx not a multiple of 128)."""
    V4()
    rng = np.random.default_rng(nq + nx + d + k)
    _check(K, _dyadic(rng, nq, d), _dyadic(rng, nx, d), k, dtype)


@pytest.mark.parametrize("stride,rank", [(4, 1), (32, 32), (16, 0), (1, 3)])
def test_topk16_v4_forced_rescans_and_compactions(K, V4, stride, rank):
    """rank 1 and stride 1 (rank 3): estimates far above the k-th score, so most queries
    fail verification and their blocks rescan; rank 32 of a 1/32 sample: a low
    threshold that overflows buffers (streamed compactions); rank 0: no sample,
    a running threshold from -inf (compaction-driven). All bit-exact."""
    V4(stride, rank)
    rng = np.random.default_rng(stride * 100 + rank)
    _check(K, _dyadic(rng, 520, 128), _dyadic(rng, 24000, 128), 100, torch.float16)


def test_topk16_v4_massive_ties_and_exclusion(K, V4):
    """Thousands of exact ties per score (compactions resolved into the ids,
    strict thresholds) with an exclusion bitmap and an id offset."""
    V4(8, 0)
    rng = np.random.default_rng(5)
    base = _dyadic(rng, 40, 128)
    x = base[rng.integers(0, 40, size=20000)]
    q = _dyadic(rng, 300, 128)
    excl = [rng.choice(20000, int(rng.integers(0, 3000)), replace=False) for _ in range(300)]
    _check(K, q, x, 100, torch.float16, exclude=excl, id_offset=7_000_000)
    V4()
    _check(K, q, x, 64, torch.bfloat16, exclude=excl)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_topk16_v4_full_query_chunk_vs_v2(K, dtype):
    """A full 65,536-query chunk (the C4 query count; v4 forced below its
    65,536-row corpus bound): compared bit for bit with the v2 kernel on the
    same inputs (both exact), with an exclusion bitmap, an id offset and a
    ragged last stage."""
    g = torch.Generator(device="cuda").manual_seed(3)
    nq, nx, d, k = 65536, 20011, 128, 100
    q = (torch.randint(-64, 65, (nq, d), device="cuda", generator=g) / 64).to(dtype)
    x = (torch.randint(-64, 65, (nx, d), device="cuda", generator=g) / 64).to(dtype)
    words = (nx + 31) // 32
    bits = torch.randint(-2**31, 2**31 - 1, (nq, words), device="cuda", generator=g, dtype=torch.int64)
    bits = (bits & torch.randint(-2**31, 2**31 - 1, (nq, words), device="cuda", generator=g, dtype=torch.int64))
    bits = (bits & 0x11111111).to(torch.int32)  # ~1 in 16 items excluded per query
    try:
        K.topk_tuning(1, 0, -1)  # v2 / v3 only
        rs, ri = K.flatip_topk(q, x, k, exclude_bits=bits, id_offset=123_456)
        K.topk_tuning(2, 0, -1)  # v4 (forced below its 65,536-row bound)
        gs, gi = K.flatip_topk(q, x, k, exclude_bits=bits, id_offset=123_456)
        torch.cuda.synchronize()
    finally:
        K.topk_tuning(0, 0, -1)
    assert torch.equal(gi, ri)
    assert torch.equal(gs, rs)


def test_topk16_v4_sixteen_splits_presampled(K, V4):
    """8,192 queries (16 query tiles) over a 200K-row corpus: the planner
    spreads the items over 16 splits (256 blocks), the joint threshold comes
    from the presample launch (every split sampled once, then one threshold
    per query), the finish merges 32 split segments per query. Whole-result
    properties plus a 512-query sample bit-exact against the oracle."""
    V4(mode=2)
    g = torch.Generator(device="cuda").manual_seed(21)
    nq, nx, d, k = 8192, 200_000, 64, 100
    q = (torch.randint(-64, 65, (nq, d), device="cuda", generator=g) / 64).half()
    x = (torch.randint(-64, 65, (nx, d), device="cuda", generator=g) / 64).half()
    gs, gi = K.flatip_topk(q, x, k)
    torch.cuda.synchronize()
    assert (gi >= 0).all() and (gi < nx).all()
    assert (gs[:, :-1] >= gs[:, 1:]).all()
    sel = torch.randperm(nq, generator=torch.Generator().manual_seed(1))[:512].numpy()
    rs, ri = orc.flat_ip_search(np.ascontiguousarray(q.float().cpu().numpy()[sel]), x.float().cpu().numpy(), k,
                                nthreads=16)
    assert np.array_equal(gi.cpu().numpy()[sel], ri)
    assert np.array_equal(gs.cpu().numpy()[sel], rs)


@pytest.mark.parametrize("n_shards,nx,k", [(8, 400_000, 100), (4, 300_000, 64), (2, 140_000, 128)])
def test_shard_global_threshold_emulated(K, V4, n_shards, nx, k):
    """rt_flatip_topk_shard_* as N ranks would run them, all on one GPU: each
    shard sampled (shard_sample), the lists combined into one threshold per
    query (topk_sample_threshold with the failure-safe rank of the
    corpus-wide sampled fraction), each shard searched against it
    (shard_search), the lists merged (topk_merge): bit-exact against the
    oracle on dyadic data (scores exact in fp32), every query's merged list
    full (no rescue needed at this rank), and each shard's candidates far
    fewer than its own k."""
    from rtrec_amd.dist.sharded import shard_range
    V4(mode=2)  # shards below the planner's 65,536-row bound keep the v4 plan
    g = torch.Generator(device="cuda").manual_seed(5 + n_shards)
    nq, d = 65536, 128
    q = (torch.randint(-64, 65, (nq, d), device="cuda", generator=g) / 64).half()
    x = (torch.randint(-64, 65, (nx, d), device="cuda", generator=g) / 64).half()
    stride = K.shard_sample_stride(nx)
    tops, sampled, stages, spans = [], 0, 0, []
    for r in range(n_shards):
        b, c = shard_range(nx, n_shards, r)
        spans.append((b, c))
        top, (sa, st) = K.flatip_topk_shard_sample(q, x[b:b + c], k, stride)
        assert top.shape == (nq, 32) and (top[:, :-1] >= top[:, 1:]).all()
        tops.append(top)
        sampled += sa
        stages += st
    rank = K.topk_sample_rank(k, sampled, stages)
    assert rank > 0
    thr = K.topk_sample_threshold(torch.stack(tops), rank)
    ss, ii = [], []
    for b, c in spans:
        s, i = K.flatip_topk_shard_search(q, x[b:b + c], k, thr, id_offset=b)
        ss.append(s)
        ii.append(i)
        valid = i >= 0
        assert (s[valid] >= thr.unsqueeze(1).expand_as(s)[valid]).all()
    ms, mi = K.topk_merge(torch.stack(ss), torch.stack(ii), k)
    torch.cuda.synchronize()
    assert (mi >= 0).all(), "a threshold above a query's k-th score (needs the rescue)"
    per_shard = torch.stack([(i >= 0).sum(dim=1).float().mean() for i in ii]).mean().item()
    assert per_shard < k, per_shard  # candidates per shard shrink below k
    sel = torch.randperm(nq, generator=torch.Generator().manual_seed(2))[:256].numpy()
    rs, ri = orc.flat_ip_search(np.ascontiguousarray(q.float().cpu().numpy()[sel]), x.float().cpu().numpy(), k,
                                nthreads=16)
    assert np.array_equal(mi.cpu().numpy()[sel], ri)
    assert np.array_equal(ms.cpu().numpy()[sel], rs)


@pytest.mark.parametrize("n_lists", [1, 3, 8, 16, 17, 64])
@pytest.mark.parametrize("rank", [1, 7, 32])
def test_sample_threshold_kway_merge(K, n_lists, rank):
    """rt_topk_sample_threshold's k-way merge (16- and 64-lane groups) equals
    the rank-th largest of the sorted union: ragged lists (-inf tails), exact
    ties across lists, empty queries (-FLT_MAX), nq not a multiple of the
    block's query count."""
    g = torch.Generator().manual_seed(100 * n_lists + rank)
    nq = 1001
    vals = torch.randint(-20, 21, (n_lists, nq, 32), generator=g).float() / 4
    fill = torch.randint(0, 33, (n_lists, nq), generator=g)
    fill[:, 5] = 0  # query 5: every list empty
    mask = torch.arange(32).view(1, 1, 32) >= fill.unsqueeze(2)
    vals = vals.masked_fill(mask, float("-inf"))
    lists = vals.sort(dim=2, descending=True).values
    union = lists.permute(1, 0, 2).reshape(nq, -1).sort(dim=1, descending=True).values
    want = union[:, rank - 1].clamp(min=-torch.finfo(torch.float32).max)
    thr = K.topk_sample_threshold(lists.cuda(), rank)
    torch.cuda.synchronize()
    assert torch.equal(thr.cpu(), want)
    assert thr[5].item() == -torch.finfo(torch.float32).max
