"""C4 top-K parity on the benchmark's own distribution (normalized Gaussian
rows rounded to f16, as bench.py generates them), at full size:

* the 125,000-row shard leg of ``bench.topk_extras`` (65,536 queries, k=100),
* the 1M-row corpus of ``bench.topk_c4_scaling`` at N=1 (one GPU: 2 item
  splits, the joint corpus-wide threshold, the rescue pair).

Both run the sampled-threshold pair of csrc/topk_v4.h. Reference semantics:
faiss.IndexFlatIP.search (src/serving/retrieval.py:141-197), restated by
oracle/flatip.c, which is fed the same rounded f16 inputs.

Random f16 products are exact in fp32, but the MFMA and the oracle's sequential
fmaf chain sum them in different orders, so scores may differ in the last
bits. The bars, per sampled query (512 of them):

* every returned score is within ``tol`` of the exact (float64) dot product of
  its row, with tol = (d - 1) * 2^-24 * sum|q_i x_i| bounded by Cauchy-Schwarz
  (the fp32 summation bound); the oracle's scores satisfy the same bound;
* the returned set is the exact top-k up to near ties: every returned row
  scores >= kth - 2 tol, every row scoring > kth + 2 tol is returned;
* ids are bit-exact at every position whose oracle score is separated from
  both neighbours (and, at the last position, from the (k+1)-th row) by more
  than 4 tol — there the order is determined whatever the summation order;
  at least 80 % of the positions must be of that kind.
"""
import numpy as np
import pytest
import torch

from oracle import flat_ip as orc

pytestmark = pytest.mark.gpu

K_TOP = 100
D = 128
SAMPLE = 512


@pytest.fixture(scope="module")
def K():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from rtrec_amd import kernels, native
    native.lib()
    return kernels


def _bench_shard_inputs(dev):
    """bench.topk_extras: generator seed 7, the C3 draws first, then the shard."""
    g = torch.Generator(device=dev).manual_seed(7)
    torch.randn(6040, D, device=dev, generator=g)
    torch.randn(3416, D, device=dev, generator=g)
    q = torch.nn.functional.normalize(torch.randn(65536, D, device=dev, generator=g), dim=1).half()
    x = torch.nn.functional.normalize(torch.randn(125000, D, device=dev, generator=g), dim=1).half()
    return q, x


def _bench_1m_inputs(dev):
    """bench.topk_c4_scaling at N=1 (rank 0 holds the whole 1M-row corpus)."""
    g = torch.Generator(device=dev).manual_seed(1000)
    x = torch.nn.functional.normalize(torch.randn(1_000_000, D, device=dev, generator=g), dim=1).half()
    gq = torch.Generator(device=dev).manual_seed(99)
    q = torch.nn.functional.normalize(torch.randn(65536, D, device=dev, generator=gq), dim=1).half()
    return q, x


def _check_sample(q, x, gs, gi, k, seed):
    nq, nx = q.shape[0], x.shape[0]
    # whole-result properties
    assert (gi >= 0).all() and (gi < nx).all()
    assert (gs[:, :-1] >= gs[:, 1:]).all()
    tie = gs[:, :-1] == gs[:, 1:]
    assert (gi[:, :-1][tie] < gi[:, 1:][tie]).all()
    srt = gi.sort(dim=1).values
    assert (srt[:, 1:] != srt[:, :-1]).all()

    sel = torch.randperm(nq, generator=torch.Generator().manual_seed(seed))[:SAMPLE]
    qs = q[sel.to(q.device)]
    # exact scores (f16 products are exact in float64; the float64 sum's error is far below tol)
    ex = qs.double() @ x.double().T                                   # [S, nx]
    absdot = qs.double().abs() @ x.double().abs().T if nx <= 200_000 else None
    qn = qs.double().norm(dim=1)
    xn = x.double().norm(dim=1).max()
    bound = (absdot.max(dim=1).values if absdot is not None else qn * xn)  # >= sum|q_i x_i| of any row
    tol = ((D - 1) * 2.0 ** -24 * bound).unsqueeze(1)                # [S, 1]
    del absdot

    ord_ = ex.topk(k + 1, dim=1)
    kth = ord_.values[:, k - 1:k]
    kp1 = ord_.values[:, k:k + 1]

    gsel, isel = gs[sel.to(gs.device)].double(), gi[sel.to(gi.device)]
    gex = ex.gather(1, isel)
    assert ((gsel - gex).abs() <= tol).all(), "device score outside the fp32 summation bound"
    assert (gex >= kth - 2 * tol).all(), "a returned row is below the exact k-th by more than 2 tol"
    must = ex > kth + 2 * tol                                          # [S, nx]
    cnt_must = must.sum(dim=1)
    hit = must.gather(1, isel).sum(dim=1)
    assert torch.equal(hit, cnt_must), "a row clearly inside the top-k is missing"
    del must

    rs, ri = orc.flat_ip_search(np.ascontiguousarray(qs.cpu().numpy()), x.cpu().numpy(), k, nthreads=16)
    rs_t = torch.from_numpy(rs).to(ex.device).double()
    ri_t = torch.from_numpy(ri).to(ex.device)
    assert ((rs_t - ex.gather(1, ri_t)).abs() <= tol).all(), "oracle outside the bound (test premise)"
    # positions whose order is determined: gaps > 4 tol to both neighbours
    up = torch.full_like(rs_t, float("inf"))
    up[:, 1:] = rs_t[:, :-1] - rs_t[:, 1:]
    dn = torch.empty_like(rs_t)
    dn[:, :-1] = rs_t[:, :-1] - rs_t[:, 1:]
    dn[:, -1] = (rs_t[:, -1] - kp1[:, 0])
    clear = (up > 4 * tol) & (dn > 4 * tol)
    frac = clear.double().mean().item()
    assert frac >= 0.8, f"only {frac:.2%} of positions are separated: the sample does not test the order"
    mism = clear & (isel != ri_t)
    assert not mism.any(), f"{int(mism.sum())} separated positions differ from the oracle"
    same_bits = (gs[sel.to(gs.device)].cpu().numpy() == rs).mean()
    return frac, float(same_bits)


def test_c4_shard_bench_distribution(K):
    q, x = _bench_shard_inputs("cuda")
    gs, gi = K.flatip_topk(q, x, K_TOP)
    torch.cuda.synchronize()
    frac, same = _check_sample(q, x, gs, gi, K_TOP, seed=5)
    print(f"shard: {frac:.1%} positions separated, {same:.1%} scores bit-identical to the oracle")


def test_c4_1m_bench_distribution(K):
    """The 1M-row single-GPU plan: 2 splits, joint threshold, rescue pair."""
    q, x = _bench_1m_inputs("cuda")
    gs, gi = K.flatip_topk(q, x, K_TOP)
    torch.cuda.synchronize()
    frac, same = _check_sample(q, x, gs, gi, K_TOP, seed=6)
    print(f"1M: {frac:.1%} positions separated, {same:.1%} scores bit-identical to the oracle")
