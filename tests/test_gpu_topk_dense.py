"""fp32 small-corpus top-K (topk_dense.h: score-slab GEMM + per-query select)
against the oracle (oracle/flatip.c, Faiss IndexFlatIP semantics): bit-exact
ids and scores, including the select's radix fallback, ties, exclusion,
id offsets, short corpora and query chunks that span several slabs; and the
same answers as the fused register-list kernel it replaces for these shapes
(rt_flatip_topk_tuning +8)."""
import numpy as np
import pytest
import torch

from oracle import flat_ip as orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def K():
    from rtrec_amd import kernels
    yield kernels
    kernels.topk_tuning(0, 0, -1)


def _run(K, q, x, k, bits=None, id_offset=0):
    dev = torch.device("cuda")
    tb = torch.from_numpy(bits.view(np.int32)).to(dev) if bits is not None else None
    s, i = K.flatip_topk(torch.from_numpy(q).to(dev), torch.from_numpy(x).to(dev), k, exclude_bits=tb,
                         id_offset=id_offset)
    return s.cpu().numpy(), i.cpu().numpy()


def _check(K, q, x, k, bits=None, id_offset=0):
    rs, ri = orc.flat_ip_search(q, x, k, exclude_bits=bits, id_offset=id_offset, nthreads=8)
    gs, gi = _run(K, q, x, k, bits, id_offset)
    assert np.array_equal(gi, ri), np.nonzero((gi != ri).any(axis=1))[0][:5]
    assert np.array_equal(gs.view(np.uint32), rs.view(np.uint32))  # bit patterns (-0.0 included)
    return gs, gi


@pytest.mark.parametrize("k", [1, 10, 32, 64, 65, 100, 128])
def test_dense_random_bit_exact(K, k):
    rng = np.random.default_rng(k)
    q = rng.standard_normal((300, 128)).astype(np.float32)
    x = rng.standard_normal((3416, 128)).astype(np.float32)
    _check(K, q, x, k)


@pytest.mark.parametrize("d", [8, 136, 256])
def test_dense_dims(K, d):
    rng = np.random.default_rng(d)
    q = rng.standard_normal((77, d)).astype(np.float32)
    x = rng.standard_normal((1000, d)).astype(np.float32)
    _check(K, q, x, 20)


def test_dense_one_lane_holds_the_top(K):
    """Items whose id % 256 < 4 (all in select lane 0) score far above the
    rest: the k-th lane maximum is a weak bound, more than 128 keys pass it and
    the radix select narrows them."""
    rng = np.random.default_rng(5)
    d = 64
    q = np.abs(rng.standard_normal((64, d))).astype(np.float32)
    x = rng.standard_normal((4096, d)).astype(np.float32) * 0.01
    ids = np.arange(4096)
    x[(ids % 256) < 4] = np.abs(x[(ids % 256) < 4]) + 1.0
    for k in (16, 64):
        _check(K, q, x, k)


def test_dense_ties_and_negative_zero(K):
    """Dyadic entries: many exactly equal scores (lower id first) and exact
    zero scores of both signs."""
    rng = np.random.default_rng(7)
    d = 16
    q = (rng.integers(-2, 3, (50, d)) / 4).astype(np.float32)
    x = (rng.integers(-2, 3, (2000, d)) / 4).astype(np.float32)
    q[0] = 0.0
    q[1] = -0.0
    x[:10] = 0.0
    for k in (5, 50, 128):
        _check(K, q, x, k)


def test_dense_exclusion_offset_short_corpus(K):
    rng = np.random.default_rng(11)
    q = rng.standard_normal((40, 64)).astype(np.float32)
    x = rng.standard_normal((900, 64)).astype(np.float32)
    words = (900 + 31) // 32
    bits = np.zeros((40, words), np.uint32)
    for r in range(40):
        for j in rng.choice(900, size=rng.integers(0, 600), replace=False):
            bits[r, j >> 5] |= np.uint32(1) << np.uint32(j & 31)
    bits[0, :] = 0xFFFFFFFF  # every item excluded: (-FLT_MAX, -1) throughout
    gs, gi = _check(K, q, x, 50, bits=bits, id_offset=1000)
    assert (gi[0] == -1).all() and (gs[0] == -np.finfo(np.float32).max).all()
    # fewer items than k
    _check(K, q, x[:7], 10)


def test_dense_several_slabs(K):
    """nq beyond one 256 MB score slab (nx = 4096: 16,384 queries per slab)."""
    rng = np.random.default_rng(13)
    q = rng.standard_normal((20000, 8)).astype(np.float32)
    x = rng.standard_normal((4096, 8)).astype(np.float32)
    _check(K, q, x, 10)


def test_dense_matches_register_list_kernel(K):
    """The C3 shape on both fp32 paths: identical lists."""
    rng = np.random.default_rng(17)
    q = rng.standard_normal((6040, 128)).astype(np.float32)
    x = rng.standard_normal((3416, 128)).astype(np.float32)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    a_s, a_i = _run(K, q, x, 10)
    K.topk_tuning(8, 0, -1)
    try:
        b_s, b_i = _run(K, q, x, 10)
    finally:
        K.topk_tuning(0, 0, -1)
    assert np.array_equal(a_i, b_i) and np.array_equal(a_s, b_s)
