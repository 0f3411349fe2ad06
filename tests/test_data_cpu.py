"""Host-side data path (SURVEY §8 a1, a7 bookkeeping) on CPU: the MovieLens
loader/preprocessing, feature tables and positives against the golden made by
importing the reference on tiny synthetic .dat files; the per-sample Dataset /
collate_fn contract; the CSR of positives the device sampler reads; the batch
builder's sampling properties; the trainer's plateau scheduler vs torch's."""
import numpy as np
import pandas as pd
import pytest
import torch

from rtrec_amd.data.movielens import MovieLensLoader, build_batches, feature_tables, get_user_positive_items
from rtrec_amd.training.datasets.movielens import MovieLensDataset, PositiveCSR, collate_fn


@pytest.fixture(scope="module")
def tiny(tmp_path_factory):
    from conftest import load_golden
    g = load_golden("movielens_tiny")
    d = tmp_path_factory.mktemp("ml")
    for name in ("ratings", "users", "movies"):
        (d / f"{name}.dat").write_text(str(g[f"{name}_dat"]))
    data = MovieLensLoader(str(d)).load_and_preprocess(split_method="time", min_user_interactions=1,
                                                      min_item_interactions=1)
    return g, data


def test_loader_splits_match_reference(tiny):
    g, data = tiny
    assert data.num_users == int(g["num_users"]) and data.num_movies == int(g["num_movies"])
    for split, df in (("train", data.train_interactions), ("val", data.val_interactions),
                      ("test", data.test_interactions)):
        for c in ("user_idx", "movie_idx", "label", "timestamp", "user_id", "movie_id", "rating"):
            np.testing.assert_array_equal(df[c].to_numpy(), g[f"{split}_{c}"], err_msg=f"{split}.{c}")


def test_feature_tables_and_positives_match_reference(tiny):
    g, data = tiny
    uf, mf = feature_tables(data)
    np.testing.assert_allclose(uf, g["user_features"], rtol=0, atol=1e-6)
    np.testing.assert_array_equal(mf, g["movie_features"])
    pos = get_user_positive_items(data.train_interactions)
    csr = PositiveCSR.from_interactions(data.train_interactions, len(g["positives"]))
    for u in range(len(g["positives"])):
        ref = [int(x) for x in g["positives"][u] if x >= 0]
        assert sorted(pos.get(u, [])) == sorted(ref)
        seg = csr.items[csr.offsets[u]:csr.offsets[u + 1]]
        assert list(seg) == sorted(set(ref))          # sorted, unique: what rt_sample_negatives searches


def test_dataset_items_and_collate(tiny):
    g, data = tiny
    ds = MovieLensDataset(data.train_interactions, data.users, data.movies, num_negatives=3, seed=0)
    assert len(ds) == len(data.train_interactions)
    pos = get_user_positive_items(data.train_interactions)
    items = [ds[i] for i in range(len(ds))]
    for it in items:
        assert set(it) == {"user_idx", "user_features", "pos_item_idx", "pos_item_features", "neg_item_indices",
                           "neg_item_features", "label"}
        negs = it["neg_item_indices"].tolist()
        assert len(set(negs)) == len(negs)
        assert not set(negs) & set(pos[it["user_idx"]])
        np.testing.assert_array_equal(it["neg_item_features"].numpy(), g["movie_features"][negs])
    b = collate_fn(items[:5])
    assert b["user_features"].shape == (5, 3) and b["neg_item_features"].shape == (5, 3, 20)
    assert b["user_idx"].dtype == torch.int64 and b["label"].shape == (5,)
    ev = MovieLensDataset(data.val_interactions, data.users, data.movies, is_training=False)
    assert "neg_item_indices" not in ev[0]


def test_csr_from_pairs_dedups_and_handles_empty_users():
    csr = PositiveCSR.from_pairs(np.array([2, 0, 2, 2]), np.array([5, 1, 3, 5]), n_users=4)
    np.testing.assert_array_equal(csr.offsets, [0, 1, 1, 3, 3])
    np.testing.assert_array_equal(csr.items, [1, 3, 5])
    assert csr.items.dtype == np.int32


def test_build_batches_sampling_properties():
    rng = np.random.default_rng(0)
    inter = pd.DataFrame({"user_idx": rng.integers(0, 50, 4000), "movie_idx": rng.integers(0, 300, 4000)})
    bu, bp, bn = build_batches(inter, 300, 64, 16, 5, seed=1)
    assert bu.shape == (5, 64) and bn.shape == (5, 64 * 16)
    pos = set(zip(inter["user_idx"], inter["movie_idx"]))
    negs = bn.reshape(-1, 16)
    for u, row in zip(bu.reshape(-1), negs):
        assert len(set(row.tolist())) == 16
        assert not any((int(u), int(x)) in pos for x in row)
    assert ((negs >= 0) & (negs < 300)).all()


def test_plateau_scheduler_matches_torch():
    from rtrec_amd.training.trainers.two_tower import _ReduceLROnPlateau

    class _Step:
        lr = 1e-3

        def set_lr(self, lr):
            self.lr = lr

    st = _Step()
    ours = _ReduceLROnPlateau(st, factor=0.5, patience=2)
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.Adam([p], lr=1e-3)
    ref = torch.optim.lr_scheduler.ReduceLROnPlateau(opt, mode="min", factor=0.5, patience=2)
    for m in [1.0, 0.9, 0.95, 0.95, 0.95, 0.95, 0.8, 0.80001, 0.8, 0.8, 0.8, 0.7]:
        ours(m)
        ref.step(m)
        assert st.lr == pytest.approx(opt.param_groups[0]["lr"], rel=0, abs=1e-15)
