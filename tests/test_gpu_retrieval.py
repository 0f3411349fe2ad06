"""GPU parity: gather / renorm / Flat-IP top-K / merge kernels and the
HipFlatIPIndex + RetrievalEngine surface vs the CPU oracle (oracle/flatip.c)."""
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


def _bf16_bits(x: torch.Tensor) -> np.ndarray:
    return x.contiguous().view(torch.int16).cpu().numpy().view(np.uint16)


def _tie_aware(ref_s, ref_i, got_s, got_i, tol):
    assert got_i.shape == ref_i.shape
    np.testing.assert_allclose(got_s, ref_s, rtol=0, atol=tol)
    for r in range(ref_i.shape[0]):
        if np.array_equal(ref_i[r], got_i[r]):
            continue
        kth = ref_s[r, -1]
        a = set(ref_i[r][ref_s[r] > kth + 2 * tol].tolist())
        b = set(got_i[r][got_s[r] > kth + 2 * tol].tolist())
        assert a == b, f"row {r}: confident sets differ"


# ---------------------------------------------------------------- gather
@pytest.mark.parametrize("rows,dim,dtype", [(6040, 3, torch.float32), (3416, 20, torch.float32),
                                            (1000, 128, torch.float32), (5000, 256, torch.bfloat16),
                                            (777, 6, torch.float16)])
def test_gather_rows_bit_exact(K, rows, dim, dtype):
    g = torch.Generator().manual_seed(rows + dim)
    table = torch.randn(rows, dim, generator=g).to(dtype)
    ids = torch.randint(0, rows, (4099,), generator=g)
    out = K.gather_rows(table.cuda(), ids.cuda(), check=True)
    ref = table.numpy() if dtype != torch.bfloat16 else None
    if ref is not None:
        assert np.array_equal(out.cpu().numpy(), ref[ids.numpy()])
    else:
        assert np.array_equal(_bf16_bits(out), _bf16_bits(table)[ids.numpy()])


def test_gather_rows_oob_and_sharded(K):
    table = torch.arange(40, dtype=torch.float32).view(10, 4).cuda()
    ids = torch.tensor([0, 9, 10, -1, 3], dtype=torch.int64).cuda()
    with pytest.raises(IndexError):
        K.gather_rows(table, ids, check=True)
    oob = torch.zeros(1, dtype=torch.int32, device="cuda")
    out = K.gather_rows(table, ids, oob=oob)
    assert int(oob.item()) == 2
    assert torch.equal(out[2], torch.zeros(4, device="cuda")) and torch.equal(out[1], table[9])
    # shard owning global rows [100, 110): ids outside read as zero rows
    out = K.gather_rows(table, torch.tensor([100, 105, 3, 109]).cuda(), row_begin=100)
    assert torch.equal(out[1], table[5]) and torch.equal(out[2], torch.zeros(4, device="cuda"))
    assert torch.equal(out[3], table[9])


def test_gather_empty(K):
    table = torch.randn(5, 8).cuda()
    out = K.gather_rows(table, torch.empty(0, dtype=torch.int64).cuda())
    assert out.shape == (0, 8)


def test_scatter_add_rows(K):
    g = torch.Generator().manual_seed(3)
    grad_out = torch.randn(64, 16, generator=g)
    ids = torch.randint(0, 11, (64,), generator=g)
    ref = torch.zeros(11, 16).index_add_(0, ids, grad_out)
    ref[0] = 0  # padding_idx row gets no gradient
    got = K.scatter_add_rows(torch.zeros(11, 16).cuda(), ids.cuda(), grad_out.cuda(), padding_idx=0)
    np.testing.assert_allclose(got.cpu().numpy(), ref.numpy(), rtol=1e-6, atol=1e-6)


# ---------------------------------------------------------------- renorm
@pytest.mark.parametrize("n,d", [(1000, 128), (65, 64), (3, 32), (100, 20)])
def test_l2_renorm_bit_exact(K, n, d):
    x = np.random.default_rng(n).standard_normal((n, d)).astype(np.float32)
    x[0] = 0.0  # zero row stays zero (sum == 0 → untouched)
    ref = x.copy()
    orc.normalize_L2(ref)
    got = K.l2_renorm_(torch.from_numpy(x).cuda()).cpu().numpy()
    assert np.array_equal(got, ref)


# ---------------------------------------------------------------- top-K
@pytest.mark.parametrize("nq,nx,d,k", [(300, 3000, 128, 10), (300, 3000, 128, 100), (257, 1999, 64, 256),
                                       (5, 1000, 32, 50), (1, 1000, 128, 50), (130, 70, 128, 100),
                                       (64, 5000, 128, 512)])
def test_flatip_fp32_bit_exact_vs_oracle(K, nq, nx, d, k):
    """fp32 scores are the sequential fmaf chain (f32 MFMA k-order) → identical
    ids AND scores to oracle/flatip.c on random data."""
    rng = np.random.default_rng(nq * 7 + nx)
    q = rng.standard_normal((nq, d)).astype(np.float32)
    x = rng.standard_normal((nx, d)).astype(np.float32)
    rs, ri = orc.flat_ip_search(q, x, k, nthreads=8)
    gs, gi = K.flatip_topk(torch.from_numpy(q).cuda(), torch.from_numpy(x).cuda(), k)
    assert np.array_equal(gi.cpu().numpy(), ri)
    assert np.array_equal(gs.cpu().numpy(), rs)


@pytest.mark.parametrize("name,k", [("flatip_dyadic_raw", 10), ("flatip_dyadic_raw", 100),
                                    ("flatip_dyadic_raw", 256), ("flatip_dyadic_unit", 1),
                                    ("flatip_dyadic_unit", 100), ("flatip_dyadic_small", 10)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
def test_flatip_dyadic_all_dtypes(K, golden, name, k, dtype):
    """Exactly summable inputs: every dtype and summation order give the same bits,
    including planted exact ties (lower id wins)."""
    g = golden(name)
    q = torch.from_numpy(g["queries"]).to(dtype).cuda()
    x = torch.from_numpy(g["items"]).to(dtype).cuda()
    gs, gi = K.flatip_topk(q, x, k)
    assert np.array_equal(gi.cpu().numpy(), g[f"k{k}_ids"])
    assert np.array_equal(gs.cpu().numpy(), g[f"k{k}_scores"])


def test_flatip_dyadic_exclusion(K, golden):
    g = golden("flatip_dyadic_raw")
    bm = torch.from_numpy(g["exclude_bits"].view(np.int32)).cuda()
    gs, gi = K.flatip_topk(torch.from_numpy(g["queries"]).cuda(), torch.from_numpy(g["items"]).cuda(), 100,
                           exclude_bits=bm)
    assert np.array_equal(gi.cpu().numpy(), g["excl_k100_ids"])
    assert np.array_equal(gs.cpu().numpy(), g["excl_k100_scores"])


@pytest.mark.parametrize("dtype,code", [(torch.float16, 1), (torch.bfloat16, 2)])
def test_flatip_half_types_tie_aware(K, dtype, code):
    rng = np.random.default_rng(5)
    q = torch.nn.functional.normalize(torch.from_numpy(rng.standard_normal((200, 128)).astype(np.float32)), dim=1)
    x = torch.nn.functional.normalize(torch.from_numpy(rng.standard_normal((4000, 128)).astype(np.float32)), dim=1)
    qh, xh = q.to(dtype), x.to(dtype)
    rs, ri = orc.flat_ip_search(qh.view(torch.int16).numpy(), xh.view(torch.int16).numpy(), 100,
                                dtype_code=code, nthreads=8)
    gs, gi = K.flatip_topk(qh.cuda(), xh.cuda(), 100)
    _tie_aware(rs, ri, gs.cpu().numpy(), gi.cpu().numpy(), tol=2e-6)


def test_flatip_exclusion_random_and_id_offset(K):
    rng = np.random.default_rng(9)
    q = rng.standard_normal((100, 64)).astype(np.float32)
    x = rng.standard_normal((2000, 64)).astype(np.float32)
    excl = [rng.choice(2000, 300, replace=False) for _ in range(100)]
    bm_np = orc.exclusion_bitmap(100, 2000, excl)
    rs, ri = orc.flat_ip_search(q, x, 100, exclude_bits=bm_np, id_offset=5000, nthreads=8)
    bm = K.exclusion_bitmap(100, 2000, excl, "cuda")
    gs, gi = K.flatip_topk(torch.from_numpy(q).cuda(), torch.from_numpy(x).cuda(), 100, exclude_bits=bm,
                           id_offset=5000)
    assert np.array_equal(gi.cpu().numpy(), ri)
    assert np.array_equal(gs.cpu().numpy(), rs)


def test_flatip_c3_shape(K):
    """Config 3: 6040 users x 3416 items, d=128 fp32, top-10 (exact vs oracle)."""
    rng = np.random.default_rng(3)
    q = rng.standard_normal((6040, 128)).astype(np.float32)
    x = rng.standard_normal((3416, 128)).astype(np.float32)
    orc.normalize_L2(q)
    orc.normalize_L2(x)
    rs, ri = orc.flat_ip_search(q, x, 10, nthreads=16)
    gs, gi = K.flatip_topk(torch.from_numpy(q).cuda(), torch.from_numpy(x).cuda(), 10)
    assert np.array_equal(gi.cpu().numpy(), ri)
    assert np.array_equal(gs.cpu().numpy(), rs)


def test_flatip_errors(K):
    from rtrec_amd.native import RTError
    with pytest.raises(RTError):  # fp32 rows must be 16-byte multiples (d % 4 == 0)
        K.flatip_topk(torch.randn(4, 10).cuda(), torch.randn(10, 10).cuda(), 5)
    with pytest.raises(ValueError):
        K.flatip_topk(torch.randn(4, 16).cuda(), torch.randn(10, 32).cuda(), 5)
    with pytest.raises(RuntimeError):
        K.flatip_topk(torch.randn(4, 16), torch.randn(10, 16), 5)  # CPU tensors: no fallback


@pytest.mark.parametrize("nq,nx,d,k,dtype", [(64, 3000, 128, 1100, torch.float32), (20, 600, 64, 700, torch.float32),
                                             (33, 2500, 128, 513, torch.float16), (40, 9000, 96, 1024, torch.bfloat16)])
def test_flatip_wide_k_vs_oracle(K, nq, nx, d, k, dtype):
    """k > 512 (Faiss takes any k, src/serving/retrieval.py:170-171): exact
    512-wide passes, each excluding the rows the earlier ones returned —
    bit-exact against the oracle (fp32 on random data, 16-bit on dyadic
    data), k > N padded, with an exclusion bitmap and an id offset."""
    rng = np.random.default_rng(nq + nx + k)
    if dtype == torch.float32:
        q = rng.standard_normal((nq, d)).astype(np.float32)
        x = rng.standard_normal((nx, d)).astype(np.float32)
    else:
        q = (rng.integers(-64, 65, size=(nq, d)) / 64.0).astype(np.float32)
        x = (rng.integers(-64, 65, size=(nx, d)) / 64.0).astype(np.float32)
    excl = [rng.choice(nx, int(rng.integers(0, nx // 3)), replace=False) for _ in range(nq)]
    bm_np = orc.exclusion_bitmap(nq, nx, excl)
    bm = K.exclusion_bitmap(nq, nx, excl, "cuda")
    for bits, bits_np, off in ((None, None, 0), (bm, bm_np, 777)):
        rs, ri = orc.flat_ip_search(q, x, k, exclude_bits=bits_np, id_offset=off, nthreads=8)
        gs, gi = K.flatip_topk(torch.from_numpy(q).to(dtype).cuda(), torch.from_numpy(x).to(dtype).cuda(), k,
                               exclude_bits=bits, id_offset=off)
        assert np.array_equal(gi.cpu().numpy(), ri)
        assert np.array_equal(gs.cpu().numpy(), rs)


def test_index_search_wide_k_and_filter(K):
    """HipFlatIPIndex.search with k > 512 and with filter_ids at k = 300
    (k_search = 600 > 512), as faiss-backed FaissIndex.search allows."""
    from rtrec_amd.serving.retrieval import HipFlatIPIndex
    rng = np.random.default_rng(12)
    emb = rng.standard_normal((2000, 64)).astype(np.float32)
    ids = [f"m{i}" for i in range(2000)]
    idx = HipFlatIPIndex({"dimension": 64})
    idx.build(emb, ids)
    q = rng.standard_normal((3, 64)).astype(np.float32)
    got, sc = idx.search(q, 900)
    e, qn = emb.copy(), q.copy()
    orc.normalize_L2(e)  # faiss.normalize_L2, bit-exact with the index's rt_l2_renorm_f32
    orc.normalize_L2(qn)
    rs, ri = orc.flat_ip_search(qn, e, 900, nthreads=4)
    assert [len(g) for g in got] == [900, 900, 900]
    for row, want in zip(got, ri):
        assert row == [ids[j] for j in want]
    allowed = ids[::3]
    fgot, _ = idx.search(q, 300, filter_ids=allowed)
    aset = set(allowed)
    for row, want in zip(fgot, ri):
        exp = [ids[j] for j in want[:600] if ids[j] in aset][:300]
        assert row == exp


def test_topk_merge(K):
    rng = np.random.default_rng(11)
    s = rng.standard_normal((8, 500, 100)).astype(np.float32)
    s[:, :, 50:] = np.round(s[:, :, 50:], 1)  # ties across lists
    i = rng.choice(10**6, (8, 500, 100)).astype(np.int64)
    for l in range(8):
        i[l] = i[l] // 8 * 8 + l  # disjoint id sets per list (like corpus shards)
    i[0, :, -3:] = -1
    rs, ri = orc.topk_merge(s, i, 100)
    gs, gi = K.topk_merge(torch.from_numpy(s).cuda(), torch.from_numpy(i).cuda(), 100)
    assert np.array_equal(gi.cpu().numpy(), ri)
    assert np.array_equal(gs.cpu().numpy(), rs)


# ---------------------------------------------------------------- index / engine
def test_hip_flat_index_semantics(K):
    from rtrec_amd.serving.retrieval import HipFlatIPIndex, RetrievalEngine
    rng = np.random.default_rng(0)
    emb = rng.standard_normal((1000, 128)).astype(np.float32)
    ids = [f"item_{i}" for i in range(1000)]
    idx = HipFlatIPIndex({"dimension": 128, "metric": "cosine"})
    with pytest.raises(ValueError, match="Index not built yet"):
        idx.search(emb[:1], 5)
    idx.build(emb, ids)
    q = rng.standard_normal((3, 128)).astype(np.float32)
    got_ids, got_s = idx.search(q, 50)
    xn, qn = emb.copy(), q.copy()
    orc.normalize_L2(xn)
    orc.normalize_L2(qn)
    rs, ri = orc.flat_ip_search(qn, xn, 50)
    assert got_ids == [[ids[j] for j in row] for row in ri]
    assert np.array_equal(np.array(got_s, np.float32), rs)
    # 1-D query, filter_ids over-fetch (k_search = 2k), add
    one_ids, _ = idx.search(q[0], 5)
    assert one_ids[0] == got_ids[0][:5]
    allow = got_ids[0][1::2]
    f_ids, _ = idx.search(q[:1], 5, filter_ids=allow)
    assert f_ids[0] == [i for i in got_ids[0][:10] if i in set(allow)][:5]
    idx.add(qn[:1] * 3.0, ["new_item"])
    a_ids, a_s = idx.search(q[:1], 1)
    assert a_ids[0] == ["new_item"] and abs(a_s[0][0] - 1.0) < 1e-6
    eng = RetrievalEngine({"index_type": "hip_flat", "embedding_dim": 128, "top_k": 10})
    eng.build_index(emb, ids)
    r1 = eng.retrieve(q[:1])
    r2 = eng.retrieve(q[:1])
    assert r1[0] == r2[0] and r2[2]["cache_hit"] and not r1[2]["cache_hit"]
    m = eng.get_metrics()
    assert m["total_queries"] == 2 and m["cache_hit_rate"] == 0.5 and m["index_size"] == 1000


def test_index_save_load_roundtrip(K, tmp_path):
    from rtrec_amd.serving.retrieval import HipFlatIPIndex
    rng = np.random.default_rng(1)
    emb = rng.standard_normal((300, 64)).astype(np.float32)
    idx = HipFlatIPIndex({"dimension": 64})
    idx.build(emb, [str(i) for i in range(300)])
    q = rng.standard_normal((4, 64)).astype(np.float32)
    before = idx.search(q, 20)
    idx.save(str(tmp_path / "idx"))
    idx2 = HipFlatIPIndex({"dimension": 64})
    idx2.load(str(tmp_path / "idx"))
    assert idx2.current_size == 300
    assert idx2.search(q, 20) == before


# ---------------------------------------------------------------- fp32 d in (128, 256]
@pytest.mark.parametrize("nq,nx,d,k", [(300, 3000, 256, 10), (200, 2500, 256, 32), (130, 2000, 256, 100),
                                       (64, 1500, 192, 300), (33, 700, 160, 7)])
def test_flatip_fp32_wide_rows_bit_exact(K, nq, nx, d, k):
    """emb-256 fp32 corpora (FaissIndex has no dimension cap): register-list
    kernel for k <= 32, candidate-buffer kernel above; bit-exact vs the oracle."""
    rng = np.random.default_rng(nq + nx + d)
    q = rng.standard_normal((nq, d)).astype(np.float32)
    x = rng.standard_normal((nx, d)).astype(np.float32)
    rs, ri = orc.flat_ip_search(q, x, k, nthreads=8)
    gs, gi = K.flatip_topk(torch.from_numpy(q).cuda(), torch.from_numpy(x).cuda(), k)
    assert np.array_equal(gi.cpu().numpy(), ri)
    assert np.array_equal(gs.cpu().numpy(), rs)


# ---------------------------------------------------------------- IndexFlatL2 mode
def _l2_check(ref_s, ref_i, got_s, got_i):
    """Bit-exact against the oracle's IndexFlatL2: the k + 32 candidates selected
    on the augmented inner product are re-ranked on the oracle's own distance
    (same fmaf order), so near-ties at the k-th distance resolve as Faiss's."""
    assert np.array_equal(ref_i, got_i), np.nonzero((ref_i != got_i).any(axis=1))[0][:5]
    assert np.array_equal(ref_s, got_s)


@pytest.mark.parametrize("d,k,nx", [(128, 10, 3000), (128, 100, 3000), (64, 50, 70), (252, 20, 1000),
                                    (32, 10, 6)])
def test_flat_l2_index_vs_oracle(K, d, k, nx):
    from rtrec_amd.serving.retrieval import HipFlatIPIndex
    rng = np.random.default_rng(d * 1000 + k)
    emb = rng.standard_normal((nx, d)).astype(np.float32)
    q = rng.standard_normal((64, d)).astype(np.float32)
    q[:3] = emb[:3]                     # exact self-matches: distance 0 (clamped)
    idx = HipFlatIPIndex({"dimension": d, "metric": "l2"})
    idx.build(emb, [f"i{j}" for j in range(nx)])
    gs, gi = idx.search_tensors(q, k)
    rs, ri = orc.flat_l2_search(q, emb, k, nthreads=8)
    _l2_check(rs, ri, gs.cpu().numpy(), gi.cpu().numpy())
    assert gi[0, 0].item() == 0 and gs[0, 0].item() == 0.0
    ids, dist = idx.search(q[:2], k)
    assert ids[0][0] == "i0" and dist[0] == sorted(dist[0])


@pytest.mark.parametrize("k,n_clus", [(10, 300), (100, 300)])
def test_flat_l2_clustered_near_ties(K, k, n_clus):
    """A cluster of near-duplicates around the queries: their distances differ
    far below fp32 rounding of ||q||^2 + ||x||^2 - 2 q.x, so the augmented
    selection score cannot rank them and k + 32 candidates miss Faiss's own
    choice. The finish's certificate flags those queries, they are re-selected
    with 512 candidates, and the result is bit-exact vs the oracle again."""
    from rtrec_amd import kernels as KK
    from rtrec_amd.serving.retrieval import HipFlatIPIndex
    rng = np.random.default_rng(77 + k)
    d = 64
    base = rng.standard_normal(d).astype(np.float32)
    clus = (base + rng.standard_normal((n_clus, d)).astype(np.float32) * 1e-4).astype(np.float32)
    far = (rng.standard_normal((2000, d)) * 3).astype(np.float32)
    emb = np.concatenate([far[:1000], clus, far[1000:]])
    q = (base + rng.standard_normal((16, d)).astype(np.float32) * 1e-4).astype(np.float32)
    idx = HipFlatIPIndex({"dimension": d, "metric": "l2"})
    idx.build(emb, [str(j) for j in range(len(emb))])
    before = dict(KK.L2_STATS)
    gs, gi = idx.search_tensors(q, k)
    rs, ri = orc.flat_l2_search(q, emb, k, nthreads=8)
    _l2_check(rs, ri, gs.cpu().numpy(), gi.cpu().numpy())
    assert KK.L2_STATS["reselected"] > before["reselected"]   # the certificate fired
    assert KK.L2_STATS["uncertified"] == before["uncertified"]


def test_flat_l2_save_load_and_errors(K, tmp_path):
    from rtrec_amd.serving.retrieval import HipFlatIPIndex, read_flat_index
    rng = np.random.default_rng(9)
    emb = rng.standard_normal((500, 64)).astype(np.float32)
    idx = HipFlatIPIndex({"dimension": 64, "metric": "euclidean"})
    idx.build(emb[:400], [str(i) for i in range(400)])
    idx.add(emb[400:], [str(i) for i in range(400, 500)])
    q = rng.standard_normal((5, 64)).astype(np.float32)
    before = idx.search(q, 30)
    idx.save(str(tmp_path / "l2idx"))
    vecs, is_ip = read_flat_index(tmp_path / "l2idx.faiss")
    assert not is_ip and np.array_equal(vecs, emb)   # IxF2 layout, raw rows
    idx2 = HipFlatIPIndex({"dimension": 64})
    idx2.load(str(tmp_path / "l2idx"))
    assert idx2.search(q, 30) == before
    with pytest.raises(ValueError, match="dimension"):
        HipFlatIPIndex({"dimension": 256, "metric": "l2"})
    with pytest.raises(ValueError, match="dimension"):
        HipFlatIPIndex({"dimension": 384})
    with pytest.raises(ValueError, match="float32"):
        HipFlatIPIndex({"dimension": 64, "metric": "l2", "storage_dtype": "float16"})
    with pytest.raises(ValueError, match="k="):
        idx.search(q, 513)


@pytest.mark.parametrize("n_lists,k_in,k_out,dup", [(8, 100, 100, False), (4, 100, 100, False), (3, 37, 50, False),
                                                    (8, 100, 64, True), (2, 128, 128, True)])
def test_topk_merge_sorted_lists(K, n_lists, k_in, k_out, dup):
    """Lists in (score desc, id asc) order with their -1 padding last — the
    per-shard top-K the multi-GPU owner merge receives — through
    rt_topk_merge's register select (<= 1,024 candidates into <= 128): score
    ties across lists, short (padded) lists, k_out below and above k_in, and
    (dup) the same (score, id) in two lists. Equal to the oracle's full sort."""
    rng = np.random.default_rng(100 * n_lists + k_in)
    nq = 700
    s = np.round(rng.standard_normal((n_lists, nq, k_in)), 1).astype(np.float32)  # many exact ties
    i = rng.choice(10**6, (n_lists, nq, k_in)).astype(np.int64)
    for l in range(n_lists):
        i[l] = i[l] // n_lists * n_lists + l
    if dup:  # list 1 repeats some entries of list 0
        i[1, :, :10] = i[0, :, :10]
        s[1, :, :10] = s[0, :, :10]
    nvalid = rng.integers(0, k_in + 1, (n_lists, nq))
    for l in range(n_lists):
        for q in range(nq):
            o = np.lexsort((i[l, q], -s[l, q]))  # score desc, id asc
            s[l, q], i[l, q] = s[l, q][o], i[l, q][o]
            i[l, q, nvalid[l, q]:] = -1
            s[l, q, nvalid[l, q]:] = -np.finfo(np.float32).max
    rs, ri = orc.topk_merge(s, i, k_out)
    gs, gi = K.topk_merge(torch.from_numpy(s).cuda(), torch.from_numpy(i).cuda(), k_out)
    assert np.array_equal(gi.cpu().numpy(), ri)
    assert np.array_equal(gs.cpu().numpy(), rs)
