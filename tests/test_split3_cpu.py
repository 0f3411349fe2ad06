"""The three-piece bf16 split behind the tower kernels' fp32 products
(csrc/mlp.hip split3 / mfma3, DESIGN.md §5 note i), restated in numpy:
x = hi + mid + lo with each piece the round-to-nearest-even bf16 of the
previous residual, and a product taken as the 6 piece products of order
<= 2^-16. These checks pin the error bounds the kernels rely on — each
residual exact in fp32, |x - hi - mid - lo| <= 2^-24 |x| (|x| >= 2^-100, where
the pieces stay normal), and a dropped-term
error below 2^-22 |x·y| per product, i.e. fp32-class — on the host, so they
run without a GPU."""
import numpy as np


def _bf16_rne(x: np.ndarray) -> np.ndarray:
    """fp32 → nearest bf16 (ties to even), returned as fp32 (v_cvt_pk_bf16_f32)."""
    u = x.astype(np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return r.astype(np.uint32).view(np.float32)


def _split3(x: np.ndarray):
    x = x.astype(np.float32)
    hi = _bf16_rne(x)
    r1 = (x - hi).astype(np.float32)
    mid = _bf16_rne(r1)
    r2 = (r1 - mid).astype(np.float32)
    lo = _bf16_rne(r2)
    return hi, mid, lo, r1, r2


def test_pieces_exact_residuals_and_bound():
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.standard_normal(200_000).astype(np.float32) * 10.0 ** rng.integers(-20, 20, 200_000),
                        np.array([0.0, -0.0, 1.0, -1.5, 3.0e-38, 6.5e4], np.float32)]).astype(np.float32)
    hi, mid, lo, r1, r2 = _split3(x)
    x64 = x.astype(np.float64)
    # every residual is exact in fp32
    assert np.array_equal(r1.astype(np.float64), x64 - hi.astype(np.float64))
    assert np.array_equal(r2.astype(np.float64), r1.astype(np.float64) - mid.astype(np.float64))
    # each piece is a bf16 value
    for p in (hi, mid, lo):
        assert not np.any(p.view(np.uint32) & 0xFFFF)
    err = np.abs(x64 - hi.astype(np.float64) - mid.astype(np.float64) - lo.astype(np.float64))
    # relative bound while the pieces stay normal (|x| >= 2^-100); below that the
    # lo piece is subnormal and the error is absolute, under 2^-125
    big = np.abs(x64) >= 2.0 ** -100
    assert np.all(err[big] <= 2.0 ** -24 * np.abs(x64[big]))
    assert np.all(err[~big] <= 2.0 ** -125)


def test_six_piece_products_are_fp32_class():
    rng = np.random.default_rng(1)
    n = 100_000
    x = (rng.standard_normal(n) * 3).astype(np.float32)
    y = (rng.standard_normal(n) * 0.2).astype(np.float32)
    xh, xm, xl, _, _ = (a.astype(np.float64) for a in _split3(x))
    yh, ym, yl, _, _ = (a.astype(np.float64) for a in _split3(y))
    six = xl * yh + xh * yl + xm * ym + xm * yh + xh * ym + xh * yh  # each term exact (8 x 8 bits)
    exact = x.astype(np.float64) * y.astype(np.float64)
    rel = np.abs(six - exact) / np.maximum(np.abs(exact), 1e-300)
    assert rel.max() <= 2.0 ** -22
    # a 256-deep dot product: within a few fp32 roundings of the exact sum,
    # no worse than a sequential fp32 fma chain
    k = 256
    a = (rng.standard_normal((64, k))).astype(np.float32)
    b = (rng.standard_normal((k, 64))).astype(np.float32)
    ah, am, al, _, _ = (t.astype(np.float64) for t in _split3(a))
    bh, bm, bl, _, _ = (t.astype(np.float64) for t in _split3(b))
    approx = al @ bh + ah @ bl + am @ bm + am @ bh + ah @ bm + ah @ bh
    exact = a.astype(np.float64) @ b.astype(np.float64)
    scale = np.abs(a.astype(np.float64)) @ np.abs(b.astype(np.float64))
    assert (np.abs(approx - exact) / scale).max() <= 2.0 ** -21
    seq = np.zeros((64, 64), np.float32)
    for t in range(k):
        seq = (seq + np.outer(a[:, t], b[t, :]).astype(np.float32)).astype(np.float32)
    seq_err = (np.abs(seq.astype(np.float64) - exact) / scale).max()
    assert (np.abs(approx - exact) / scale).max() <= seq_err
