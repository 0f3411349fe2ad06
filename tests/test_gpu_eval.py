"""Offline evaluation on the GPU (SURVEY §8 a11 + f1): generate_recommendations
(scripts/evaluate_model.py:162-234) and the ranking metrics of
src/evaluation/metrics.py through rt_exclusion_bitmap / rt_flatip_topk /
rt_rank_metrics, against

* the reference's own generate_recommendations output (eval_topk.npz, written
  by importing the reference) — tie-aware, since the reference orders exact
  ties by numpy's unstable argsort;
* the reference's Evaluator output on those recommendations (eval_metrics.npz),
  including predictions that contain excluded items;
* the reference's known-answer metric tests (tests/_metric_cases.py);
* the oracle (oracle/metrics.py, pinned by the above) at the C3 shape: 6,040
  users x 3,416 items, top-100, Zipf-sized train/test sets.
"""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _model_from_golden(g, dev):
    from rtrec_amd.training.utils import create_two_tower_model_for_training
    m = create_two_tower_model_for_training(3, 20, {"embedding_dim": 64, "hidden_layers": [128, 64],
                                                    "dropout_rate": 0.2, "temperature": 0.05})
    for tname, tower in (("user", m.user_tower), ("item", m.item_tower)):
        sd = {k[len(tname) + 1:]: torch.from_numpy(np.array(v)) for k, v in g.items() if k.startswith(tname + "/")}
        tower.load_state_dict(sd)
    return m.to(dev).eval()


def test_generate_recommendations_vs_reference(device, golden):
    from rtrec_amd.evaluation import generate_recommendations
    g = golden("eval_topk")
    m = _model_from_golden(g, device)
    users = [int(u) for u in g["test_users"]]
    train = {u: [int(x) for x in g["exclude"][r] if x >= 0] for r, u in enumerate(users)}
    recs = generate_recommendations(m, users, train, g["user_features"], g["movie_features"], top_k=100,
                                    batch_size=256, device="cuda")
    # the embeddings the HIP towers produce match the reference's
    with torch.no_grad():
        ue = m.get_user_embeddings({"numerical": torch.from_numpy(g["user_features"]).to(device),
                                    "categorical": {}}).cpu().numpy()
        ie = m.get_item_embeddings({"numerical": torch.from_numpy(g["movie_features"]).to(device),
                                    "categorical": {}}).cpu().numpy()
    np.testing.assert_allclose(ue, g["user_emb"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(ie, g["item_emb"], rtol=1e-5, atol=1e-6)
    full = g["user_emb"][g["test_users"]].astype(np.float64) @ g["item_emb"].astype(np.float64).T
    n_exact = n_near = 0
    for r, u in enumerate(users):
        got, want = np.array(recs[u]), g["recs"][r]
        assert len(got) == len(want) == 100
        assert not (set(got.tolist()) & set(train[u]))
        # smallest gap between consecutive reference scores over the list and the
        # first item past it (excluded items out): the scores are ~0.3, where one
        # fp32 ulp is 3e-8, so a list whose gaps all exceed 1e-7 cannot reorder
        # under last-bit differences of the embeddings and must match exactly
        s = full[r].copy()
        s[[x for x in train[u]]] = -np.inf
        gap = (-np.diff(np.sort(s)[::-1][:101])).min()
        n_near += gap <= 3e-8
        if np.array_equal(got, want):
            n_exact += 1
            continue
        assert gap <= 1e-7, (r, gap)
        # tie-aware: positions may differ only inside groups of (near-)equal scores
        sg, sw = full[r, got], full[r, want]
        np.testing.assert_allclose(sg, sw, rtol=0, atol=1e-5)
        kth = sw[-1]
        assert set(got[sg > kth + 1e-5].tolist()) == set(want[sw > kth + 1e-5].tolist()), r
    print(f"generate_recommendations: {n_exact}/{len(users)} lists identical to the reference's "
          f"({n_near} lists hold two scores within one fp32 ulp)")
    # the reference data has no exact score ties; 4 of its 300 lists hold a pair
    # of scores within 3e-8 (one ulp). Observed 298/300 identical with the fp32
    # MFMA towers (round 3) and 297/300 with the split-bf16 towers (round 4):
    # every other list identical
    assert n_exact >= len(users) - n_near, (n_exact, n_near)


def test_generate_recommendations_pad_excluded_vs_reference(device, golden):
    """Heavy users (up to 150 of 160 items in train): the reference pads each
    list to top_k with -inf train items in numpy argsort order
    (scripts/evaluate_model.py:224-232); pad_excluded=True returns those
    full-length lists (tests/golden/eval_topk_heavy.npz, reference-generated)."""
    from rtrec_amd.evaluation import generate_recommendations
    g = golden("eval_topk_heavy")
    m = _model_from_golden(g, device)
    users = [int(u) for u in g["test_users"]]
    train = {u: [int(x) for x in g["exclude"][r] if x >= 0] for r, u in enumerate(users)}
    recs = generate_recommendations(m, users, train, g["user_features"], g["movie_features"], top_k=100,
                                    batch_size=256, device="cuda", pad_excluded=True)
    short = generate_recommendations(m, users, train, g["user_features"], g["movie_features"], top_k=100,
                                     batch_size=256, device="cuda")
    n_items = g["movie_features"].shape[0]
    n_exact = n_heavy = 0
    for r, u in enumerate(users):
        got, want = recs[u], [int(x) for x in g["recs"][r]]
        eligible = n_items - len(train[u])
        assert len(got) == len(want) == 100
        assert len(set(got)) == 100
        if eligible < 100:
            n_heavy += 1
            assert short[u] == got[:eligible]            # the eligible items first, GPU order
            assert set(got[eligible:]) <= set(train[u])  # then excluded items only
        n_exact += got == want
    print(f"pad_excluded: {n_exact}/{len(users)} lists identical ({n_heavy} heavy users)")
    assert n_heavy >= 20
    assert n_exact == len(users), n_exact


def test_evaluator_vs_reference_evaluator(device, golden):
    from rtrec_amd.evaluation import Evaluator
    g = golden("eval_metrics")
    users = [int(u) for u in g["test_users"]]
    preds = {u: [int(x) for x in g["recs"][r]] for r, u in enumerate(users)}
    for u in range(1000, 1010):
        preds[u] = list(range(100))
    gt = {u: set(int(x) for x in g["ground_truth"][r] if x >= 0) for r, u in enumerate(users)}
    ex = {u: set(int(x) for x in g["exclude"][r] if x >= 0) for r, u in enumerate(users)}
    preds2 = {u: [int(x) for x in g["preds_with_excluded"][r] if x >= 0] for r, u in enumerate(users)}
    ks = [int(k) for k in g["k_values"]]
    ev = Evaluator(k_values=ks, num_items=int(g["num_items"]))
    for tag, p in (("plain", preds), ("filtered", preds2)):
        m = ev.evaluate(p, gt, ex)
        d = m.to_dict()
        for key in [f"{n}@{k}" for n in ("recall", "precision", "ndcg", "hit_rate") for k in ks] + \
                ["mrr", "map", "coverage"]:
            np.testing.assert_allclose(d[key], g[f"{tag}/{key}"], rtol=1e-12, err_msg=f"{tag} {key}")
        for k in ks:
            np.testing.assert_allclose(m.per_user_recall[k], g[f"{tag}/per_user_recall@{k}"], rtol=1e-12)
            np.testing.assert_allclose(m.per_user_ndcg[k], g[f"{tag}/per_user_ndcg@{k}"], rtol=1e-12)


def test_metric_known_answers_on_gpu(device):
    from _metric_cases import CASES, EVALUATOR, NDCG_REVERSED
    from rtrec_amd.evaluation import metrics as gm
    for fn, pred, gt, k, want in CASES:
        f = getattr(gm, fn)
        got = f(pred, gt, k) if k is not None else f(pred, gt)
        assert math.isclose(got, want, rel_tol=1e-12, abs_tol=0.0), (fn, pred, gt, k, got, want)
    p, g, k = NDCG_REVERSED
    assert 0.0 < gm.ndcg_at_k(p, g, k) < 1.0
    for preds, gts, ex, ks, ni, want in EVALUATOR:
        d = gm.Evaluator(k_values=ks, num_items=ni).evaluate(preds, gts, ex).to_dict()
        for key, v in want.items():
            assert math.isclose(d[key], v, rel_tol=1e-12), (key, d[key], v)
    # a repeated ground-truth item is refused, not silently miscounted
    with pytest.raises(ValueError):
        gm.recall_at_k([1, 1, 2], {1}, 3)


def test_exclusion_bitmap_device_equals_host(device):
    from rtrec_amd import kernels
    from rtrec_amd.evaluation.metrics import csr_from_sets
    rng = np.random.default_rng(3)
    n_items = 3416
    rows = [sorted(rng.choice(n_items + 40, int(rng.integers(0, 300)), replace=False).tolist()) for _ in range(500)]
    off, items = csr_from_sets(rows, device)
    sel = torch.tensor(rng.integers(-3, 503, 700), dtype=torch.int64, device=device)  # incl. out-of-range rows
    got = kernels.exclusion_bitmap_csr(off, items, n_items, rows=sel)
    host_rows = [rows[u] if 0 <= u < 500 else [] for u in sel.cpu().tolist()]
    want = kernels.exclusion_bitmap(len(host_rows), n_items, host_rows, device)
    assert torch.equal(got, want)


def test_c3_scale_metrics_vs_oracle(device):
    """C3 shape: masked top-100 for 6,040 users over 3,416 items, then the
    metrics of every user, GPU vs oracle (exact same recommendation lists)."""
    from oracle import metrics as om
    from rtrec_amd import kernels
    from rtrec_amd.evaluation import evaluate_tensors
    from rtrec_amd.evaluation.metrics import csr_from_sets
    rng = np.random.default_rng(5)
    nu, ni, d = 6040, 3416, 128
    g = torch.Generator(device=device).manual_seed(5)
    q = torch.nn.functional.normalize(torch.randn(nu, d, device=device, generator=g), dim=1)
    x = torch.nn.functional.normalize(torch.randn(ni, d, device=device, generator=g), dim=1)
    train = [sorted(rng.choice(ni, min(ni - 1, 20 + int(rng.zipf(1.6))), replace=False).tolist()) for _ in range(nu)]
    test = [sorted(rng.choice(ni, int(rng.integers(0, 30)), replace=False).tolist()) for _ in range(nu)]
    t_off, t_items = csr_from_sets(train, device)
    bits = kernels.exclusion_bitmap_csr(t_off, t_items, ni)
    _, ids = kernels.flatip_topk(q, x, 100, exclude_bits=bits)
    g_off, g_items = csr_from_sets(test, device)
    ks = [5, 10, 20, 50, 100]
    got = evaluate_tensors(ids, g_off, g_items, ks, ex_offsets=t_off, ex_items=t_items, num_items=ni)
    host = ids.cpu().numpy()
    preds = {u: [x for x in host[u].tolist() if x >= 0] for u in range(nu)}  # -1: fewer eligible items than k
    gt = {u: set(test[u]) for u in range(nu)}
    ref = om.evaluate(preds, gt, ks, num_items=ni, exclude_items={u: set(train[u]) for u in range(nu)})
    d = got.to_dict()
    for key in [f"{n}@{k}" for n in ("recall", "precision", "ndcg", "hit_rate") for k in ks] + ["mrr", "map",
                                                                                                 "coverage"]:
        np.testing.assert_allclose(d[key], ref[key], rtol=1e-12, err_msg=key)
    for k in ks:
        np.testing.assert_allclose(got.per_user_ndcg[k], ref[f"per_user_ndcg@{k}"], rtol=1e-12)
