"""N>1 paths on CPU: world_size-2 gloo process groups driving
the same orchestration code the GPU ranks run (rtrec_amd/dist/sharded.py), with the
per-rank compute bound to the oracle (tests may use the oracle as checker).

* corpus-sharded exact top-K: merged result == one index over the whole corpus,
  bit-exact on dyadic data (ties resolved by the lower global id);
* table-sharded gather + all-reduce == one gather from the unsharded table;
* C5 data-parallel in-batch step (each rank's users vs the gathered global
  batch, label offset rank·b) == the reference loss and grads of the whole batch;
* data-parallel gradient average.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import flat_ip as orc
from rtrec_amd.dist import sharded as sharded_mod
from rtrec_amd.dist.sharded import (allreduce_mean_, owner_of, segment_capacity, shard_range, sharded_gather_rows,
                                    sharded_inbatch_step, sharded_scatter_add_rows, sharded_topk, sharded_topk_owner)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(world, fn, *args):
    port = _free_port()
    mp.spawn(_entry, args=(world, port, fn, args), nprocs=world, join=True)


def _entry(rank, world, port, fn, args):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fn(rank, world, *args)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _dyadic(rng, n, d):
    # multiples of 2^-6 in [-1, 1]: every partial sum is exact in fp32, so any
    # summation order gives the same bits (SURVEY §8(c) parity contract 1)
    return (rng.integers(-64, 65, size=(n, d)) / 64.0).astype(np.float32)


# ---------------------------------------------------------------------------
def test_shard_range_partitions_contiguously():
    for n in (0, 1, 7, 1000, 1001, 12_500_000 * 8 + 3):
        for world in (1, 2, 3, 8):
            spans = [shard_range(n, world, r) for r in range(world)]
            assert spans[0][0] == 0
            for (b0, c0), (b1, _) in zip(spans, spans[1:]):
                assert b0 + c0 == b1
            assert sum(c for _, c in spans) == n
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1
    ids = torch.arange(1001)
    own = owner_of(ids, 1001, 3)
    for r in range(3):
        b, c = shard_range(1001, 3, r)
        assert torch.all(own[b:b + c] == r)


def _topk_worker(rank, world, n, d, nq, k, seed, with_ties):
    rng = np.random.default_rng(seed)
    corpus = _dyadic(rng, n, d)
    queries = _dyadic(rng, nq, d)
    if with_ties:  # duplicate rows across the shard boundary: equal scores, lower id must win
        corpus[n - 1] = corpus[0]
        corpus[n // 2] = corpus[1]
    b, c = shard_range(n, world, rank)
    shard = corpus[b:b + c]

    def local(q, kk):
        s, i = orc.flat_ip_search(q.numpy(), shard, kk, id_offset=b)
        return torch.from_numpy(s), torch.from_numpy(i)

    def merge(s, i, kk):
        ms, mi = orc.topk_merge(s.numpy(), i.numpy(), kk)
        return torch.from_numpy(ms), torch.from_numpy(mi)

    got_s, got_i = sharded_topk(torch.from_numpy(queries), k, local, merge)
    ref_s, ref_i = orc.flat_ip_search(queries, corpus, k)
    np.testing.assert_array_equal(got_i.numpy(), ref_i)
    np.testing.assert_array_equal(got_s.numpy(), ref_s)


@pytest.mark.parametrize("n,k,ties", [(1001, 10, False), (300, 100, True), (37, 50, False)])
def test_sharded_topk_matches_single_index_gloo(n, k, ties):
    _run(2, _topk_worker, n, 32, 19, k, 7, ties)


def _topk_owner_worker(rank, world, n, d, nq, k, seed):
    rng = np.random.default_rng(seed)
    corpus = _dyadic(rng, n, d)
    corpus[n - 1] = corpus[0]  # a tie across the shard boundary
    queries = _dyadic(rng, nq, d)
    b, c = shard_range(n, world, rank)

    def local(q, kk):
        s, i = orc.flat_ip_search(q.numpy(), corpus[b:b + c], kk, id_offset=b)
        return torch.from_numpy(s), torch.from_numpy(i)

    def merge(s, i, kk):
        ms, mi = orc.topk_merge(s.numpy(), i.numpy(), kk)
        return torch.from_numpy(ms), torch.from_numpy(mi)

    got_s, got_i = sharded_topk_owner(torch.from_numpy(queries), k, local, merge)
    qb, qc = shard_range(nq, world, rank)
    ref_s, ref_i = orc.flat_ip_search(queries[qb:qb + qc], corpus, k)
    np.testing.assert_array_equal(got_i.numpy(), ref_i)
    np.testing.assert_array_equal(got_s.numpy(), ref_s)


@pytest.mark.parametrize("world,n,k", [(2, 1001, 10), (4, 500, 100)])
def test_sharded_topk_query_owner_gloo(world, n, k):
    """C4 at N GPUs: all-to-all of per-slice candidate lists, the query owner
    merges — equal to one index over the whole corpus for the owned queries."""
    _run(world, _topk_owner_worker, n, 32, 24, k, 11)


def _gather_worker(rank, world, n, d, seed, counts, skew):
    rng = np.random.default_rng(seed)
    table = rng.standard_normal((n, d)).astype(np.float32)
    # skew: every id in the first shard's window, so the other owners' segments are empty
    hi = shard_range(n, world, 0)[1] if skew else n
    all_ids = [rng.integers(0, hi, size=c) for c in counts]
    b, c = shard_range(n, world, rank)
    shard = torch.from_numpy(table[b:b + c])

    def window_gather(t, ids, begin):  # rt_gather_rows semantics: rows outside the window are zero
        loc = ids - begin
        ok = (loc >= 0) & (loc < t.shape[0])
        out = torch.zeros((ids.numel(), t.shape[1]), dtype=t.dtype)
        out[ok] = t[loc[ok]]
        return out

    status = torch.zeros(2, dtype=torch.int64)
    rows = sharded_gather_rows(shard, b, torch.from_numpy(all_ids[rank]), gather=window_gather,
                               counts=counts if len(set(counts)) > 1 else None, status=status)
    ref = table[np.concatenate(all_ids)]
    np.testing.assert_array_equal(rows.numpy(), ref)
    assert status[0] == status[1] == sum(counts)  # every id owned by exactly one rank
    # owner segments unless a skewed batch overflowed one (then the byte-MAX exchange)
    P = world * max(counts)
    cap = segment_capacity(P, world)
    overflow = skew and cap < P and max(counts) > 0 and sum(counts) > cap
    want = "byte-MAX all-reduce" if overflow else "owner segments"
    assert sharded_mod.LAST_EXCHANGE["mode"] == want, (sharded_mod.LAST_EXCHANGE, cap, P)
    for mode in ("max", "segments"):  # both exchanges, forced, give the same rows
        r = sharded_gather_rows(shard, b, torch.from_numpy(all_ids[rank]), gather=window_gather,
                                counts=counts if len(set(counts)) > 1 else None, exchange=mode)
        np.testing.assert_array_equal(r.numpy(), ref)
    # bit-exact through the byte-wise exchange: -0.0 and NaN payloads survive
    special = table.copy()
    special[::7, 0] = -0.0
    special[1::7, 1] = np.float32("nan")
    shard2 = torch.from_numpy(special[b:b + c])
    rows2 = sharded_gather_rows(shard2, b, torch.from_numpy(all_ids[rank]), gather=window_gather,
                                counts=counts if len(set(counts)) > 1 else None)
    assert rows2.numpy().tobytes() == special[np.concatenate(all_ids)].tobytes()
    # an id outside every window: counted (no sync) or raised with check=True
    bad = torch.from_numpy(all_ids[rank]).clone()
    if bad.numel():
        bad[0] = n + 5
    st = torch.zeros(2, dtype=torch.int64)
    sharded_gather_rows(shard, b, bad, gather=window_gather, counts=counts if len(set(counts)) > 1 else None,
                        status=st)
    assert int(st[1]) == sum(counts) - sum(1 for cc in counts if cc)
    with pytest.raises(IndexError):  # every rank with ids planted one bad id
        sharded_gather_rows(shard, b, bad, gather=window_gather, counts=counts if len(set(counts)) > 1 else None,
                            check=True)
    # ragged batches WITHOUT counts: the sizes are all-gathered (no hang, same rows)
    rows3 = sharded_gather_rows(shard, b, torch.from_numpy(all_ids[rank]), gather=window_gather)
    np.testing.assert_array_equal(rows3.numpy(), ref)
    # ranks passing different status/check arguments: the owned-count all-reduce
    # runs on every rank regardless, so nothing deadlocks
    st2 = torch.zeros(2, dtype=torch.int64)
    sharded_gather_rows(shard, b, torch.from_numpy(all_ids[rank]), gather=window_gather,
                        status=st2 if rank == 0 else None)
    if rank == 0:
        assert st2[0] == st2[1] == sum(counts)

    # a gather that returns a NON-contiguous tensor: the exchanged rows are kept
    def strided_gather(t, ids, begin):
        out = window_gather(t, ids, begin)
        wide = torch.zeros((out.shape[1], out.shape[0]), dtype=out.dtype)
        wide.copy_(out.t())
        return wide.t()  # same values, column-major storage
    rows4 = sharded_gather_rows(shard, b, torch.from_numpy(all_ids[rank]), gather=strided_gather)
    np.testing.assert_array_equal(rows4.numpy(), ref)


@pytest.mark.parametrize("world,counts,skew", [(2, [13, 29], False), (4, [7, 0, 31, 16], False),
                                               (2, [40, 9], True), (3, [5, 5, 5], True),
                                               (4, [512] * 4, False), (4, [512] * 4, True),
                                               (3, [300, 0, 417], False), (8, [1024] * 8, False),
                                               (8, [1024] * 8, True), (8, [100, 0, 57, 300, 1, 2, 3, 64], False)])
def test_sharded_gather_rows_gloo(world, counts, skew):
    """C5 exchange: ragged per-rank batches (one empty), ids skewed onto one
    owner (the other windows own nothing; at 4 x 512 positions that overflows
    the owner segments and re-runs as the byte-MAX all-reduce): rows in batch
    order, bit-exact (-0.0 and NaN payloads included); out-of-window ids
    counted."""
    _run(world, _gather_worker, 997, 16, 3, counts, skew)


def _scatter_worker(rank, world, n, d, b, seed, skew=False):
    rng = np.random.default_rng(seed)
    ids = rng.integers(0, shard_range(n, world, 0)[1] if skew else n, size=b)
    ids[: b // 16] = ids[0]                      # repeated ids accumulate
    grads = [rng.standard_normal((b, d)).astype(np.float32) for _ in range(world)]  # every rank's contribution
    ref = np.zeros((n, d), np.float64)
    for g in grads:
        np.add.at(ref, ids, g)
    rb, rc = shard_range(n, world, rank)
    shard_grad = torch.zeros((rc, d))

    def scatter_add(t, loc, g):  # rt_scatter_add_rows_f32 semantics on CPU: ids outside [0, rows) skipped
        ok = (loc >= 0) & (loc < t.shape[0])
        t.index_add_(0, loc[ok], g[ok])
        return t

    status = torch.zeros(2, dtype=torch.int64)
    sharded_scatter_add_rows(shard_grad, rb, torch.from_numpy(ids), torch.from_numpy(grads[rank]),
                             scatter_add=scatter_add, status=status)
    np.testing.assert_allclose(shard_grad.numpy(), ref[rb:rb + rc], rtol=1e-5, atol=1e-5)
    assert status[0] == status[1] == b
    cap = segment_capacity(b, world)
    per_owner = np.bincount(owner_of(torch.from_numpy(ids), n, world).numpy(), minlength=world)
    want = "all-reduce" if per_owner.max() > cap else "owner reduce-scatter"
    assert sharded_mod.LAST_EXCHANGE["mode"] == want, (sharded_mod.LAST_EXCHANGE, cap)
    for mode in ("allreduce", "segments"):
        t = torch.zeros((rc, d))
        sharded_scatter_add_rows(t, rb, torch.from_numpy(ids), torch.from_numpy(grads[rank]),
                                 scatter_add=scatter_add, exchange=mode)
        np.testing.assert_allclose(t.numpy(), ref[rb:rb + rc], rtol=1e-5, atol=1e-5)
    # an id outside every window is counted (sync-free) and raised with check=True
    bad = torch.from_numpy(ids).clone()
    bad[1] = n + 3
    st = torch.zeros(2, dtype=torch.int64)
    sharded_scatter_add_rows(torch.zeros((rc, d)), rb, bad, torch.from_numpy(grads[rank]),
                             scatter_add=scatter_add, status=st)
    assert int(st[0]) == b and int(st[1]) == b - 1
    with pytest.raises(IndexError):
        sharded_scatter_add_rows(torch.zeros((rc, d)), rb, bad, torch.from_numpy(grads[rank]),
                                 scatter_add=scatter_add, check=True)


@pytest.mark.parametrize("world,b,skew", [(2, 64, False), (3, 64, False), (4, 2048, False), (4, 2048, True),
                                          (8, 2048, False), (8, 2048, True)])
def test_sharded_scatter_add_rows_gloo(world, b, skew):
    """Trainable C5 table: row gradients of the global batch summed over ranks
    and added by their owners into their shards — by one reduce-scatter of
    owner segments, or (a skewed batch overflowing a segment) one all-reduce."""
    _run(world, _scatter_worker, 301, 8, b, 13, skew)


def _dp_worker(rank, world):
    g = torch.full((5,), float(rank + 1))
    allreduce_mean_(g)
    assert torch.all(g == 1.5)


def test_allreduce_mean_gloo():
    _run(2, _dp_worker)


def _c5_worker(rank, world, n, d, b, seed):
    from oracle import two_tower as orc
    rng = np.random.default_rng(seed)
    table = rng.standard_normal((n, d)).astype(np.float32)
    users = rng.standard_normal((world * b, d)).astype(np.float32)
    ids = rng.integers(0, n, size=world * b)
    beg, cnt = shard_range(n, world, rank)
    shard = torch.from_numpy(table[beg:beg + cnt])

    def window_gather(t, i, begin):
        loc = i - begin
        ok = (loc >= 0) & (loc < t.shape[0])
        out = torch.zeros((i.numel(), t.shape[1]), dtype=t.dtype)
        out[ok] = t[loc[ok]]
        return out

    def cpu_loss(u, p, off):  # the reference CE on the local rows, rectangular S, torch autograd
        uu, pp = u.clone().requires_grad_(), p.clone().requires_grad_()
        s = uu @ pp.t() / 0.1
        loss = torch.nn.functional.cross_entropy(s, torch.arange(off, off + u.shape[0]))
        loss.backward()
        return torch.stack([loss.detach(), torch.tensor(0.0), loss.detach()]).double(), uu.grad, pp.grad

    def scatter_add(t, loc, g):
        ok = (loc >= 0) & (loc < t.shape[0])
        t.index_add_(0, loc[ok], g[ok])
        return t

    u_loc = torch.from_numpy(users[rank * b:(rank + 1) * b])
    grad_shard = torch.zeros((cnt, d))
    status = torch.zeros(2, dtype=torch.int64)
    loss, du, dp = sharded_inbatch_step(shard, beg, u_loc, torch.from_numpy(ids[rank * b:(rank + 1) * b]), 0.1,
                                        gather=window_gather, loss_fn=cpu_loss, grad_shard=grad_shard,
                                        scatter_add=scatter_add, status=status)
    assert status[0] == status[1] == world * b  # the owned count rode in the loss all-reduce
    dp_sum = dp.clone()
    torch.distributed.all_reduce(dp_sum)  # the frozen path exchanges nothing: sum here to compare
    # equals the single-process reference loss over the whole global batch
    U = torch.from_numpy(users).requires_grad_()
    P = torch.from_numpy(table[ids]).requires_grad_()
    ref = orc.in_batch_negative_loss(U, P, 0.1)
    ref.backward()
    np.testing.assert_allclose(float(loss), float(ref), rtol=1e-6)
    np.testing.assert_allclose(du.numpy(), U.grad[rank * b:(rank + 1) * b].numpy(), rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(dp_sum.numpy(), P.grad.numpy(), rtol=1e-5, atol=1e-7)
    # trainable table: the owners' shard gradients
    ref_g = np.zeros((n, d), np.float64)
    np.add.at(ref_g, ids, P.grad.numpy())
    np.testing.assert_allclose(grad_shard.numpy(), ref_g[beg:beg + cnt], rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("world", [2, 8])
def test_sharded_inbatch_step_gloo(world):
    _run(world, _c5_worker, 401, 16, 24, 5)


class CpuShardOps:
    """CPU restatements of the six per-rank calls of sharded_topk_global
    (tests may use the oracle): scores are the oracle's fmaf chains
    (flat_ip_search over the whole shard), ids are global positions
    (``begin + row`` or ``gpos[row]``), the plan always applies to a
    non-empty shard, ``force_rescue`` picks an unsafe rank of 1."""

    def __init__(self, shard, begin=0, gpos=None, force_rescue=False):
        self.shard = shard
        self.begin, self.gpos, self.force = int(begin), gpos, force_rescue

    def _glob(self, i):
        if self.gpos is None:
            return np.where(i >= 0, i + self.begin, -1)
        return np.where(i >= 0, self.gpos[np.maximum(i, 0)], -1)

    def plan(self, nq, rows, kk, stride):
        if rows <= 0:
            return None
        stages = -(-rows // 128)
        return len(range(0, stages, stride)), stages

    def sample(self, q, kk, stride):
        top, cnt = orc.shard_sample(q.numpy(), self.shard.numpy(), stride)
        return torch.from_numpy(top), cnt

    def rank(self, kk, sampled, stages):
        return 1 if self.force else orc.sample_rank(kk, sampled, stages)

    def threshold(self, lists, r):
        u = -np.sort(-lists.numpy().transpose(1, 0, 2).reshape(lists.shape[1], -1), axis=1)
        t = u[:, r - 1]
        return torch.from_numpy(np.where(np.isfinite(t), t, -np.finfo(np.float32).max).astype(np.float32))

    def search(self, q, kk, thr):
        n = self.shard.shape[0]
        s, i = orc.flat_ip_search(q.numpy(), self.shard.numpy(), n)  # every row, (score desc, id asc)
        out_s = np.full((q.shape[0], kk), -np.finfo(np.float32).max, np.float32)
        out_i = np.full((q.shape[0], kk), -1, np.int64)
        for r in range(q.shape[0]):
            m = min(kk, int(np.sum(s[r] >= thr[r].item())))
            out_s[r, :m] = s[r, :m]
            out_i[r, :m] = self._glob(i[r, :m])
        return torch.from_numpy(out_s), torch.from_numpy(out_i)

    def topk(self, q, kk):
        s, i = orc.flat_ip_search(q.numpy(), self.shard.numpy(), kk)
        return torch.from_numpy(s), torch.from_numpy(self._glob(i))


def _cpu_merge(s, i, kk):
    ms, mi = orc.topk_merge(s.numpy(), i.numpy(), kk)
    return torch.from_numpy(ms), torch.from_numpy(mi)


def _global_thr_worker(rank, world, n, d, nq, k, seed, owner, force_rescue, pass_rows=True):
    from rtrec_amd.dist.sharded import LAST_TOPK, sharded_topk_global
    from rtrec_amd import kernels as K
    rng = np.random.default_rng(seed)
    corpus = _dyadic(rng, n, d)
    corpus[n - 1] = corpus[0]  # a tie across the shard boundary
    queries = _dyadic(rng, nq, d)
    b, c = shard_range(n, world, rank)
    ops = CpuShardOps(torch.from_numpy(corpus[b:b + c]), b, force_rescue=force_rescue)
    rows = [shard_range(n, world, r)[1] for r in range(world)] if pass_rows else None
    got_s, got_i = sharded_topk_global(torch.from_numpy(queries), k, n, ops, _cpu_merge, owner=owner,
                                       shard_rows=rows)
    if owner:
        qb, qc = shard_range(nq, world, rank)
        ref_s, ref_i = orc.flat_ip_search(queries[qb:qb + qc], corpus, k)
    else:
        ref_s, ref_i = orc.flat_ip_search(queries, corpus, k)
    np.testing.assert_array_equal(got_i.numpy(), ref_i)
    np.testing.assert_array_equal(got_s.numpy(), ref_s)
    assert LAST_TOPK["path"] == "global threshold"
    assert LAST_TOPK["stride"] == K.shard_sample_stride(n)
    # host reads: the rescue count only (plus the shard-size all-gather without shard_rows)
    assert LAST_TOPK["host_reads"] == (1 if pass_rows else 2)
    if force_rescue:
        assert LAST_TOPK["rescued_queries"] > 0


@pytest.mark.parametrize("world,n,nq,k,owner,force,rows", [
    (2, 16384, 24, 10, True, False, True), (3, 16384, 24, 100, False, False, True),
    (4, 9000, 24, 50, True, False, False), (2, 16384, 24, 100, True, True, True),
    (8, 20000, 24, 100, True, False, True), (8, 20000, 21, 100, False, False, True),
    (8, 20000, 24, 100, True, True, True), (8, 20000, 13, 10, False, True, False)])
def test_sharded_topk_global_threshold_gloo(world, n, nq, k, owner, force, rows):
    """C4 at N GPUs with ONE corpus-wide threshold per query (ranks' shard
    samples all-gathered, the failure-safe rank of the corpus-wide sampled
    fraction): exact against one index over the whole corpus, owner and
    all-gather layouts (queries padded to a multiple of the world), up to the
    machine's 8 ranks; forcing an unsafe rank (threshold above the k-th)
    exercises the rescue of the short queries from -inf."""
    _run(world, _global_thr_worker, n, 32, nq, k, 13, owner, force, rows)


def test_sample_rank_matches_library():
    """oracle.sample_rank restates rt_topk_sample_rank (host code of the library)."""
    from rtrec_amd import kernels as K
    for k, s, t in [(100, 122, 7813), (10, 16, 977), (100, 2, 977), (50, 40, 40), (128, 31, 1000)]:
        assert K.topk_sample_rank(k, s, t) == orc.sample_rank(k, s, t), (k, s, t)


def test_bf16_floor_bits_round_down():
    """The sample-list exchange of sharded_topk_global sends bf16 patterns
    rounded toward -inf: every value comes back <= the original (so the
    derived threshold can only drop), bf16-representable values exactly,
    -FLT_MAX as -inf, and the patterns survive a float16 view (the wire type)."""
    from rtrec_amd.dist.sharded import _bf16_bits_to_f32, _bf16_floor_bits
    g = torch.Generator().manual_seed(0)
    fmax = float(np.finfo(np.float32).max)
    x = torch.cat([torch.randn(20000, generator=g) * 30,
                   torch.tensor([0.0, -0.0, 1.0, -1.0, float("inf"), float("-inf"), fmax, -fmax, 1e-40, -1e-40])])
    bits = _bf16_floor_bits(x)
    y = _bf16_bits_to_f32(bits.view(torch.float16).view(torch.int16))
    assert bool((y <= x).all())
    assert float(_bf16_bits_to_f32(_bf16_floor_bits(torch.tensor([-fmax])))[0]) == float("-inf")
    sel = torch.isfinite(x) & torch.isfinite(y) & (x.abs() > 1e-30)
    gap = (x - y)[sel] / x[sel].abs()
    assert float(gap.max()) <= 2.0 ** -7  # one bf16 ulp at most
    z = torch.randn(1000, generator=g).to(torch.bfloat16).float()
    assert torch.equal(_bf16_bits_to_f32(_bf16_floor_bits(z)), z)


# ---------------------------------------------------------------------------
# HipShardedFlatIPIndex behind the reference plugin API (RetrievalEngine
# index_type "hip_flat_sharded"), per-rank compute on the CPU oracle
def _cpu_index_cls(force_rescue=False):
    from rtrec_amd.serving.retrieval import HipShardedFlatIPIndex

    class CpuShardedIndex(HipShardedFlatIPIndex):
        """The product class with its three device hooks on the CPU oracle:
        storage on the CPU, oracle renorm (Faiss rule), oracle ops/merge. The
        id maps, layout, add, filter, tiling, save/load and every collective
        are the product code."""

        def _dev(self):
            return torch.device("cpu")

        def _renorm_(self, t):
            a = t.numpy()
            orc.normalize_L2(a)
            return t

        def _ops(self, rows):
            gpos = self.gpos.numpy() if self.gpos is not None else None
            return CpuShardOps(rows.float(), self.begin, gpos, force_rescue=force_rescue)

        def _merge(self, s, i, k):
            return _cpu_merge(s, i, k)
    return CpuShardedIndex


def _ref_lists(corpus, queries, k, metric, ids, filter_ids=None):
    """One whole-corpus index (the HipFlatIPIndex / FaissIndex contract) on the oracle."""
    from rtrec_amd.serving.retrieval import _lists_from_positions
    x, q = corpus.copy(), queries.copy()
    if metric == "cosine":
        orc.normalize_L2(x)
        orc.normalize_L2(q)
    ks = min(2 * k, len(x)) if filter_ids else k
    s, i = orc.flat_ip_search(q, x, ks)
    return _lists_from_positions(s, i, {p: v for p, v in enumerate(ids)}, k, filter_ids)


def _index_worker(rank, world, n, d, nq, k, metric, tile, tmp, force_rescue):
    from rtrec_amd.dist import sharded as sh
    from rtrec_amd.serving.retrieval import RetrievalEngine, register_index
    register_index("hip_flat_sharded", _cpu_index_cls(force_rescue))
    rng = np.random.default_rng(21)
    corpus = _dyadic(rng, n, d) if metric == "inner_product" else rng.standard_normal((n, d)).astype(np.float32)
    corpus[n - 1] = corpus[3]          # an exact tie across shards: the lower position wins
    queries = _dyadic(rng, nq, d) if metric == "inner_product" else rng.standard_normal((nq, d)).astype(np.float32)
    ids = [f"item_{p}" for p in range(n)]
    cfg = {"index_type": "hip_flat_sharded", "embedding_dim": d, "top_k": k,
           "hip_flat_sharded": {"metric": metric, "query_tile": tile}}
    eng = RetrievalEngine(cfg)
    assert eng.index.world == world and eng.index.rank == rank
    eng.build_index(corpus, ids)
    got_i, got_s, met = eng.retrieve(queries, k)
    ref_i, ref_s = _ref_lists(corpus, queries, k, metric, ids)
    assert got_i == ref_i and got_s == ref_s
    assert met["num_results"] == nq * min(k, n)
    assert sh.LAST_TOPK["path"] == "global threshold"
    if force_rescue:
        assert sh.LAST_TOPK["rescued_queries"] > 0
    # a 1-D query is reshaped; the md5 cache answers the repeat
    one_i, _, _ = eng.retrieve(queries[0], k)
    assert one_i == [ref_i[0]]
    _, _, m2 = eng.retrieve(queries[0], k)
    assert m2["cache_hit"]
    # filter_ids: k_search = min(2k, N) over-fetch, then the filter
    allow = [ids[p] for p in range(0, n, 3)]
    f_i, f_s, _ = eng.retrieve(queries, k, allow)
    r_i, r_s = _ref_lists(corpus, queries, k, metric, ids, allow)
    assert f_i == r_i and f_s == r_s
    # owner layout: this rank's slice of each query tile
    nq_own = nq - nq % world
    s_own, p_own = eng.index.search_tensors(queries[:nq_own], k, layout="owner")
    s_all, p_all = eng.index.search_tensors(queries[:nq_own], k)
    tile_eff = max(tile - tile % world, world)  # the index's tiles hold a multiple of the world
    rows = []
    for t0 in range(0, nq_own, tile_eff):
        qb, qc = shard_range(min(tile_eff, nq_own - t0), world, rank)
        rows.extend(range(t0 + qb, t0 + qb + qc))
    np.testing.assert_array_equal(p_own.numpy(), p_all.numpy()[rows])
    np.testing.assert_array_equal(s_own.numpy(), s_all.numpy()[rows])
    # incremental add (Kafka item_update path): new global rows spread over the ranks
    extra = _dyadic(rng, 37, d) if metric == "inner_product" else rng.standard_normal((37, d)).astype(np.float32)
    extra[5] = corpus[3]               # ties the earlier row: the older (lower) position wins
    new_ids = [f"new_{j}" for j in range(37)]
    eng.update_index(extra, new_ids)
    assert eng.get_metrics()["index_size"] == n + 37
    assert sum(eng.index.shard_sizes) == n + 37
    assert max(eng.index.shard_sizes) - min(eng.index.shard_sizes) <= 2
    all_x, all_ids = np.concatenate([corpus, extra]), ids + new_ids
    a_i, a_s, _ = eng.retrieve(queries, k)
    r_i, r_s = _ref_lists(all_x, queries, k, metric, all_ids)
    assert a_i == r_i and a_s == r_s
    # per-shard save, same-world load
    path = os.path.join(tmp, "idx")
    eng.save(path)
    eng2 = RetrievalEngine(cfg)
    eng2.load(path)
    b_i, b_s, _ = eng2.retrieve(queries, k)
    assert b_i == r_i and b_s == r_s
    assert eng2.index.current_size == n + 37
    # errors of the FaissIndex contract
    fresh = RetrievalEngine(cfg).index
    with pytest.raises(ValueError, match="Index not built yet"):
        fresh.search(queries, k)
    with pytest.raises(ValueError, match="No index to save"):
        fresh.save(path + "_none")


@pytest.mark.parametrize("world,n,nq,k,metric,tile,force", [
    (2, 3001, 19, 10, "cosine", 65536, False), (4, 2500, 23, 50, "inner_product", 8, False),
    (8, 4099, 29, 100, "inner_product", 65536, False), (8, 3000, 17, 20, "cosine", 8, True)])
def test_sharded_index_through_retrieval_engine_gloo(tmp_path, world, n, nq, k, metric, tile, force):
    """the multi-GPU index behind the reference plugin API —
    RetrievalEngine({"index_type": "hip_flat_sharded"}) at world 2/4/8 equals
    one whole-corpus index id for id (string ids, scores, exact ties, 1-D
    queries, the cache, filter_ids over-fetch, add, per-shard save/load,
    query tiles, owner layout, forced rescues)."""
    _run(world, _index_worker, n, 32, nq, k, metric, tile, str(tmp_path), force)


def _reshard_save_worker(rank, world, n, d, tmp):
    from rtrec_amd.serving.retrieval import RetrievalEngine, register_index
    register_index("hip_flat_sharded", _cpu_index_cls())
    rng = np.random.default_rng(8)
    corpus = _dyadic(rng, n, d)
    eng = RetrievalEngine({"index_type": "hip_flat_sharded", "embedding_dim": d,
                           "hip_flat_sharded": {"metric": "inner_product"}})
    eng.build_index(corpus, [f"i{p}" for p in range(n)])
    eng.update_index(_dyadic(rng, 11, d), [f"n{j}" for j in range(11)])
    eng.save(os.path.join(tmp, "w"))


def _reshard_load_worker(rank, world, n, d, tmp):
    from rtrec_amd.serving.retrieval import RetrievalEngine, register_index
    register_index("hip_flat_sharded", _cpu_index_cls())
    rng = np.random.default_rng(8)
    corpus = np.concatenate([_dyadic(rng, n, d), _dyadic(rng, 11, d)])
    ids = [f"i{p}" for p in range(n)] + [f"n{j}" for j in range(11)]
    q = _dyadic(np.random.default_rng(9), 9, d)
    cfg = {"index_type": "hip_flat_sharded", "embedding_dim": d, "hip_flat_sharded": {"metric": "inner_product"}}
    eng = RetrievalEngine(cfg)
    eng.load(os.path.join(tmp, "w"))        # saved by 2 ranks, loaded by `world`: re-sharded
    got = eng.retrieve(q, 15)[:2]
    assert got == _ref_lists(corpus, q, 15, "inner_product", ids)
    assert eng.index.shard_sizes == [shard_range(n + 11, world, r)[1] for r in range(world)]
    eng2 = RetrievalEngine(cfg)
    eng2.load(os.path.join(tmp, "single"))  # a single-GPU HipFlatIPIndex save
    assert eng2.retrieve(q, 15)[:2] == got


def test_sharded_index_reshards_on_load_gloo(tmp_path):
    """A per-shard save from 2 ranks loads on 4 (rows re-sharded by global
    position), and a single-GPU index save (one .faiss + .pkl) loads sharded."""
    import pickle

    from rtrec_amd.serving.retrieval import write_flat_index
    n, d = 203, 16
    _run(2, _reshard_save_worker, n, d, str(tmp_path))
    rng = np.random.default_rng(8)
    corpus = np.concatenate([_dyadic(rng, n, d), _dyadic(rng, 11, d)])
    ids = [f"i{p}" for p in range(n)] + [f"n{j}" for j in range(11)]
    write_flat_index(tmp_path / "single.faiss", corpus, True)
    with open(tmp_path / "single.pkl", "wb") as f:
        pickle.dump({"id_map": dict(enumerate(ids)), "reverse_id_map": {v: p for p, v in enumerate(ids)},
                     "current_size": len(ids), "config": {"metric": "inner_product"}}, f)
    _run(4, _reshard_load_worker, n, d, str(tmp_path))
