"""Pin the CPU oracle to the reference: golden vectors produced by importing the
reference (tools/make_goldens.py) and dyadic Flat-IP fixtures. CPU only."""
import numpy as np
import pytest
import torch

from oracle import flat_ip
from oracle import two_tower as orc


def _state(g, prefix):
    out = {}
    for k, v in g.items():
        if k.startswith(prefix + "/"):
            t = torch.from_numpy(np.array(v))
            out[k[len(prefix) + 1:]] = t.clone()
    return out


TOWER_CASES = ["tower_user_c2", "tower_item_c2", "tower_user_cat", "tower_item_content",
               "tower_act_gelu", "tower_act_leaky_relu", "tower_act_tanh", "tower_act_sigmoid"]


@pytest.mark.parametrize("name", TOWER_CASES)
def test_tower_forward_backward(golden, name):
    g = golden(name)
    act = name.split("tower_act_")[1] if name.startswith("tower_act_") else "relu"
    st = _state(g, "state")
    x = torch.from_numpy(g["x"])
    cat = {k[4:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("cat/")} or None
    content = torch.from_numpy(g["content"]) if "content" in g else None
    y = orc.tower_forward(st, x, cat, content, train=False, activation=act)
    np.testing.assert_allclose(y.numpy(), g["out_eval"], rtol=1e-5, atol=1e-6)
    st = _state(g, "state")
    params = {k: v.requires_grad_(True) for k, v in st.items()
              if not ("running" in k or "num_batches" in k)}
    xg = x.clone().requires_grad_(True)
    y = orc.tower_forward(st, xg, cat, content, train=True, activation=act)
    np.testing.assert_allclose(y.detach().numpy(), g["out_train"], rtol=1e-5, atol=1e-6)
    (y * torch.from_numpy(g["r"])).sum().backward()
    np.testing.assert_allclose(xg.grad.numpy(), g["grad_x"], rtol=1e-4, atol=1e-5)
    for k, p in params.items():
        if f"grad/{k}" in g:
            np.testing.assert_allclose(p.grad.numpy(), g[f"grad/{k}"], rtol=1e-4, atol=1e-5, err_msg=k)
    for k, v in g.items():
        if k.startswith("post/"):
            np.testing.assert_allclose(st[k[5:]].detach().numpy(), v, rtol=1e-5, atol=1e-6, err_msg=k)


@pytest.mark.parametrize("b,d", [(8, 64), (8, 128), (256, 64), (256, 128), (1024, 128)])
def test_in_batch_loss(golden, b, d):
    g = golden(f"loss_inbatch_B{b}_D{d}")
    u = torch.from_numpy(g["u"]).requires_grad_(True)
    i = torch.from_numpy(g["i"]).requires_grad_(True)
    loss = orc.in_batch_negative_loss(u, i, float(g["tau"]))
    loss.backward()
    np.testing.assert_allclose(loss.item(), g["loss"], rtol=1e-6)
    np.testing.assert_allclose(u.grad.numpy(), g["grad_u"], rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(i.grad.numpy(), g["grad_i"], rtol=1e-5, atol=1e-7)


def test_contrastive_loss(golden):
    g = golden("loss_contrastive")
    u = torch.from_numpy(g["u"]).requires_grad_(True)
    p = torch.from_numpy(g["p"]).requires_grad_(True)
    n = torch.from_numpy(g["n"]).requires_grad_(True)
    ub = torch.tensor([float(g["user_bias"])], requires_grad=True)
    ib = torch.tensor([float(g["item_bias"])], requires_grad=True)
    loss = orc.contrastive_loss(u, p, n, float(g["tau"]), ub, ib)
    loss.backward()
    np.testing.assert_allclose(loss.item(), g["loss"], rtol=1e-6)
    for t, k in [(u, "grad_u"), (p, "grad_p"), (n, "grad_n"), (ub, "grad_user_bias"), (ib, "grad_item_bias")]:
        np.testing.assert_allclose(t.grad.numpy(), g[k], rtol=1e-5, atol=1e-7, err_msg=k)


def test_similarity(golden):
    g = golden("similarity")
    s = orc.compute_similarity(torch.from_numpy(g["u"]), torch.from_numpy(g["i"]), float(g["tau"]),
                               torch.tensor([float(g["user_bias"])]), torch.tensor([float(g["item_bias"])]))
    np.testing.assert_allclose(s.numpy(), g["sim"], rtol=1e-6, atol=1e-6)


def test_train_step_two_steps(golden):
    g = golden("train_step_c2")
    us, its = _state(g, "user"), _state(g, "item")
    biases = {"user_bias": torch.zeros(1), "item_bias": torch.zeros(1)}
    opt = {}
    losses = []
    for j in range(2):
        r = orc.train_step(us, its, biases, opt, torch.from_numpy(g[f"b{j}_user_features"]),
                           torch.from_numpy(g[f"b{j}_pos_item_features"]),
                           torch.from_numpy(g[f"b{j}_neg_item_features"]), temperature=0.05)
        losses.append(r["loss"])
        pre = "mid" if j == 0 else "final"
        for k, v in us.items():
            np.testing.assert_allclose(v.numpy(), g[f"{pre}_user/{k}"], rtol=1e-4, atol=1e-6, err_msg=k)
        for k, v in its.items():
            np.testing.assert_allclose(v.numpy(), g[f"{pre}_item/{k}"], rtol=1e-4, atol=1e-6, err_msg=k)
        np.testing.assert_allclose(biases["user_bias"].numpy(), g[f"{pre}_user_bias"], rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose(losses, g["losses"], rtol=1e-5)


def test_param_counts(golden):
    g = golden("param_counts")
    assert int(g["c2"]) == 106754  # README.md:140


def _tie_aware_equal(ref_ids, got_ids, scores, tol):
    """Lists agree except for permutations inside groups of near-equal scores."""
    for r in range(ref_ids.shape[0]):
        a, b = ref_ids[r], got_ids[r]
        if np.array_equal(a, b):
            continue
        sa, sb = scores[r, a], scores[r, b]
        assert np.allclose(sa, sb, atol=tol), (r, a[:5], b[:5])
        kth = sa[-1]
        strict_a = set(a[sa > kth + tol].tolist())
        strict_b = set(b[sb > kth + tol].tolist())
        assert strict_a == strict_b, r


def test_eval_topk_masked(golden):
    g = golden("eval_topk")
    us, its = _state(g, "user"), _state(g, "item")
    ue = orc.tower_forward(us, torch.from_numpy(g["user_features"]), train=False).numpy()
    ie = orc.tower_forward(its, torch.from_numpy(g["movie_features"]), train=False).numpy()
    np.testing.assert_allclose(ue, g["user_emb"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(ie, g["item_emb"], rtol=1e-5, atol=1e-6)
    q = ue[g["test_users"]]
    excl = [row[row >= 0].tolist() for row in g["exclude"]]
    bm = flat_ip.exclusion_bitmap(len(q), ie.shape[0], excl)
    s, ids = flat_ip.flat_ip_search(np.ascontiguousarray(q), ie, 100, exclude_bits=bm)
    full = q.astype(np.float64) @ ie.astype(np.float64).T
    _tie_aware_equal(g["recs"], ids, full, 1e-5)


@pytest.mark.parametrize("k", [1, 10, 100])
def test_dyadic_unit_with_renorm(golden, k):
    g = golden("flatip_dyadic_unit")
    x = g["items"].copy()
    q = g["queries"].copy()
    flat_ip.normalize_L2(x)
    flat_ip.normalize_L2(q)
    assert np.array_equal(x, g["items"]) and np.array_equal(q, g["queries"])  # exact unit rows
    s, i = flat_ip.flat_ip_search(q, x, k)
    assert np.array_equal(i, g[f"k{k}_ids"])
    assert np.array_equal(s, g[f"k{k}_scores"])


@pytest.mark.parametrize("k", [10, 100, 256])
def test_dyadic_raw(golden, k):
    g = golden("flatip_dyadic_raw")
    s, i = flat_ip.flat_ip_search(g["queries"], g["items"], k, nthreads=4)
    assert np.array_equal(i, g[f"k{k}_ids"])
    assert np.array_equal(s, g[f"k{k}_scores"])


def test_dyadic_raw_excluded(golden):
    g = golden("flatip_dyadic_raw")
    s, i = flat_ip.flat_ip_search(g["queries"], g["items"], 100, exclude_bits=g["exclude_bits"], nthreads=4)
    assert np.array_equal(i, g["excl_k100_ids"])
    assert np.array_equal(s, g["excl_k100_scores"])


def test_dyadic_k_gt_n(golden):
    g = golden("flatip_dyadic_small")
    s, i = flat_ip.flat_ip_search(g["queries"], g["items"], 10)
    assert np.array_equal(i, g["k10_ids"])
    assert np.array_equal(s, g["k10_scores"])
    assert (i[:, 7:] == -1).all()


def test_topk_merge_matches_single_search(golden):
    g = golden("flatip_dyadic_raw")
    q, x = g["queries"], g["items"]
    parts_s, parts_i = [], []
    for r in range(4):  # row-shard the corpus like the multi-GPU path
        lo, hi = r * 750, (r + 1) * 750
        s, i = flat_ip.flat_ip_search(q, x[lo:hi], 100, id_offset=lo)
        parts_s.append(s)
        parts_i.append(i)
    ms, mi = flat_ip.topk_merge(np.stack(parts_s), np.stack(parts_i), 100)
    assert np.array_equal(mi, g["k100_ids"])
    assert np.array_equal(ms, g["k100_scores"])


# ---------------------------------------------------------------------------
# ranking metrics (src/evaluation/metrics.py) — oracle pinned by the reference's
# own known answers and by its Evaluator output (eval_metrics.npz)
# ---------------------------------------------------------------------------
def test_metrics_oracle_known_answers():
    import math
    from oracle import metrics as om
    from _metric_cases import CASES, EVALUATOR, NDCG_REVERSED
    for fn, pred, gt, k, want in CASES:
        f = getattr(om, fn)
        got = f(pred, gt, k) if k is not None else f(pred, gt)
        assert math.isclose(got, want, rel_tol=1e-12, abs_tol=0.0), (fn, pred, gt, k, got, want)
    p, g, k = NDCG_REVERSED
    assert 0.0 < om.ndcg_at_k(p, g, k) < 1.0
    for preds, gts, ex, ks, ni, want in EVALUATOR:
        out = om.evaluate(preds, gts, ks, num_items=ni, exclude_items=ex)
        for key, v in want.items():
            assert math.isclose(out[key], v, rel_tol=1e-12), (key, out[key], v)


def _eval_metrics_inputs(g):
    users = [int(u) for u in g["test_users"]]
    preds = {u: [int(x) for x in g["recs"][r]] for r, u in enumerate(users)}
    for u in range(1000, 1010):
        preds[u] = list(range(100))
    gt = {u: set(int(x) for x in g["ground_truth"][r] if x >= 0) for r, u in enumerate(users)}
    ex = {u: set(int(x) for x in g["exclude"][r] if x >= 0) for r, u in enumerate(users)}
    preds2 = {u: [int(x) for x in g["preds_with_excluded"][r] if x >= 0] for r, u in enumerate(users)}
    return preds, preds2, gt, ex


def test_metrics_oracle_vs_reference_evaluator(golden):
    from oracle import metrics as om
    g = golden("eval_metrics")
    preds, preds2, gt, ex = _eval_metrics_inputs(g)
    ks = [int(k) for k in g["k_values"]]
    for tag, p in (("plain", preds), ("filtered", preds2)):
        out = om.evaluate(p, gt, ks, num_items=int(g["num_items"]), exclude_items=ex)
        for key in [f"{m}@{k}" for m in ("recall", "precision", "ndcg", "hit_rate") for k in ks] + \
                ["mrr", "map", "coverage"]:
            np.testing.assert_allclose(out[key], g[f"{tag}/{key}"], rtol=1e-13, err_msg=f"{tag} {key}")
        for k in ks:
            np.testing.assert_allclose(out[f"per_user_recall@{k}"], g[f"{tag}/per_user_recall@{k}"], rtol=1e-13)
            np.testing.assert_allclose(out[f"per_user_ndcg@{k}"], g[f"{tag}/per_user_ndcg@{k}"], rtol=1e-13)
