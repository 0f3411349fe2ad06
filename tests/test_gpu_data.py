"""GPU data feeder and trainer: the on-device
negative sampler keeps the reference sampler's contract (distinct, never an
interacted item, uniform over the pool, whole pool when it is small), the
feeder's id batches drive the fused step to the same loss as dense feature
batches, and the trainer mirror runs epochs and writes reference-keyed
checkpoints."""
import copy

import numpy as np
import pytest
import torch

from rtrec_amd import kernels
from rtrec_amd.training.datasets.movielens import DeviceFeeder, PositiveCSR

pytestmark = pytest.mark.gpu


def _csr(device, n_users, num_items, rng):
    users, items = [], []
    for u in range(n_users):
        if u == 0:
            its = np.arange(num_items)[np.arange(num_items) % 700 != 3]   # pool of 5 < num_neg
        elif u == 1:
            its = np.array([], np.int64)                                  # no positives
        else:
            its = rng.choice(num_items, rng.integers(1, num_items // 2), replace=False)
        users.append(np.full(len(its), u))
        items.append(its)
    csr = PositiveCSR.from_pairs(np.concatenate(users), np.concatenate(items), n_users)
    return csr, csr.to(device)


def test_sampler_contract(device):
    rng = np.random.default_rng(0)
    n_users, num_items, num_neg = 64, 3416, 16
    csr, dcsr = _csr(device, n_users, num_items, rng)
    users = torch.from_numpy(np.concatenate([np.arange(n_users), rng.integers(0, n_users, 4000), [-1, 999]])).to(device)
    out = kernels.sample_negatives(dcsr.offsets, dcsr.items, users, num_items, num_neg, seed=123)
    again = kernels.sample_negatives(dcsr.offsets, dcsr.items, users, num_items, num_neg, seed=123)
    other = kernels.sample_negatives(dcsr.offsets, dcsr.items, users, num_items, num_neg, seed=124)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    assert torch.equal(out, again) and not torch.equal(out, other)
    for r, u in enumerate(users.cpu().numpy()):
        row = o[r]
        pos = set(csr.items[csr.offsets[u]:csr.offsets[u + 1]].tolist()) if 0 <= u < n_users else set()
        if u == 0:   # pool smaller than num_neg: the pool in id order, then -1
            pool = [i for i in range(num_items) if i not in pos]
            assert row[:len(pool)].tolist() == pool and (row[len(pool):] == -1).all()
            continue
        assert len(set(row.tolist())) == num_neg
        assert ((row >= 0) & (row < num_items)).all()
        assert not set(row.tolist()) & pos


def test_sampler_contract_large_catalogue(device):
    """Catalogues over 65,536 items take the binary-search form (no LDS bitmap):
    same contract."""
    rng = np.random.default_rng(5)
    n_users, num_items, num_neg = 16, 100_000, 16
    users_l, items_l = [], []
    for u in range(n_users):
        its = rng.choice(num_items, int(rng.integers(1, 3000)), replace=False)
        users_l.append(np.full(len(its), u))
        items_l.append(its)
    csr = PositiveCSR.from_pairs(np.concatenate(users_l), np.concatenate(items_l), n_users)
    dcsr = csr.to(device)
    users = torch.from_numpy(rng.integers(0, n_users, 2000)).to(device)
    o = kernels.sample_negatives(dcsr.offsets, dcsr.items, users, num_items, num_neg, seed=11).cpu().numpy()
    for r, u in enumerate(users.cpu().numpy()):
        row = o[r]
        pos = set(csr.items[csr.offsets[u]:csr.offsets[u + 1]].tolist())
        assert len(set(row.tolist())) == num_neg
        assert ((row >= 0) & (row < num_items)).all()
        assert not set(row.tolist()) & pos


def test_sampler_is_uniform_over_the_pool(device):
    rng = np.random.default_rng(1)
    num_items, num_neg = 200, 8
    pos = np.sort(rng.choice(num_items, 120, replace=False))
    csr = PositiveCSR.from_pairs(np.zeros(len(pos), np.int64), pos, 1).to(device)
    users = torch.zeros(20000, dtype=torch.int64, device=device)
    out = kernels.sample_negatives(csr.offsets, csr.items, users, num_items, num_neg, seed=7).cpu().numpy()
    counts = np.bincount(out.reshape(-1), minlength=num_items)
    assert counts[pos].sum() == 0
    pool = np.setdiff1d(np.arange(num_items), pos)
    c = counts[pool]
    expected = out.size / len(pool)
    chi2 = ((c - expected) ** 2 / expected).sum()
    assert chi2 < len(pool) + 6 * np.sqrt(2 * len(pool)), chi2   # ~6 sigma on a chi2(79)


def _tiny_data():
    from rtrec_amd.data.movielens import synthetic_movielens
    return synthetic_movielens(n_users=300, n_movies=400, n_ratings=20000, seed=3)


def test_feeder_batches(device):
    data = _tiny_data()
    f = DeviceFeeder(data.train_interactions, data.users, data.movies, num_negatives=16, batch_size=256,
                     device=device, seed=5)
    pos = set(zip(data.train_interactions["user_idx"], data.train_interactions["movie_idx"]))
    n = 0
    for b in f:
        assert b["user_ids"].shape == (256,) and b["neg_ids"].shape == (256 * 16,)
        u = b["user_ids"].cpu().numpy()
        neg = b["neg_ids"].view(256, 16).cpu().numpy()
        for r in range(0, 256, 17):
            assert not any((int(u[r]), int(x)) in pos for x in neg[r])
        n += 1
    assert n == len(f) > 0


def test_sampler_heavy_users(device):
    """Users holding most of the catalogue (the LDS bitmap path's many-rejection
    case) and a few thousand positives each: exact contract at pools of 17..400."""
    rng = np.random.default_rng(4)
    num_items, num_neg = 3416, 16
    its = [np.sort(rng.choice(num_items, num_items - p, replace=False)) for p in (17, 40, 400, 1200)]
    csr = PositiveCSR.from_pairs(np.concatenate([np.full(len(x), u) for u, x in enumerate(its)]),
                                 np.concatenate(its), len(its))
    dcsr = csr.to(device)
    users = torch.from_numpy(rng.integers(0, len(its), 3000)).to(device)
    o = kernels.sample_negatives(dcsr.offsets, dcsr.items, users, num_items, num_neg, seed=21).cpu().numpy()
    for r, u in enumerate(users.cpu().numpy()):
        row = o[r]
        assert len(set(row.tolist())) == num_neg and ((row >= 0) & (row < num_items)).all()
        assert not set(row.tolist()) & set(its[u].tolist())


def test_id_batches_equal_dense_batches(device):
    from rtrec_amd.training.fused_step import FusedTrainStep
    from rtrec_amd.training.utils import create_two_tower_model_for_training
    data = _tiny_data()
    torch.manual_seed(0)
    m1 = create_two_tower_model_for_training(3, 20, {"embedding_dim": 64, "hidden_layers": [128, 64],
                                                     "dropout_rate": 0.0, "temperature": 0.05}).to(device)
    m2 = copy.deepcopy(m1)
    f = DeviceFeeder(data.train_interactions, data.users, data.movies, num_negatives=4, batch_size=128,
                     device=device, seed=1)
    b = next(iter(f))
    s1, s2 = FusedTrainStep(m1), FusedTrainStep(m2)
    l1 = s1(b["user_table"], b["item_table"], b["item_table"], user_ids=b["user_ids"], pos_ids=b["pos_ids"],
            neg_ids=b["neg_ids"])
    uf = kernels.gather_rows(b["user_table"], b["user_ids"])
    pf = kernels.gather_rows(b["item_table"], b["pos_ids"])
    nf = kernels.gather_rows(b["item_table"], b["neg_ids"])
    l2 = s2(uf, pf, nf)
    torch.cuda.synchronize()
    assert torch.equal(l1, l2)
    for a, c in zip(m1.parameters(), m2.parameters()):
        assert torch.allclose(a, c, rtol=0, atol=1e-6)


def test_trainer_epochs_and_checkpoint(device, tmp_path):
    from rtrec_amd.training.trainers.two_tower import TwoTowerTrainer
    from rtrec_amd.training.utils import create_two_tower_model_for_training
    data = _tiny_data()
    torch.manual_seed(0)
    model = create_two_tower_model_for_training(3, 20, {"embedding_dim": 64, "hidden_layers": [128, 64]})
    tr = DeviceFeeder(data.train_interactions, data.users, data.movies, num_negatives=8, batch_size=256,
                      device=device, seed=2)
    va = DeviceFeeder(data.val_interactions, data.users, data.movies, num_negatives=0, batch_size=256,
                      device=device, seed=3, shuffle=False, positives=data.train_interactions)
    t = TwoTowerTrainer(model, tr, va, {"learning_rate": 3e-3, "checkpoint_dir": str(tmp_path)}, device="cuda")
    t.train(3)
    h = t.get_training_history()
    assert len(h["train_losses"]) == 3 and all(np.isfinite(h["train_losses"]))
    assert h["train_losses"][-1] < h["train_losses"][0]
    ck = torch.load(tmp_path / "two_tower_latest.pth", weights_only=True)
    assert {"epoch", "user_tower_state", "item_tower_state", "temperature", "user_bias", "item_bias",
            "optimizer_state", "train_losses", "val_losses"} <= set(ck)
    n_params = len(list(model.parameters()))
    assert len(ck["optimizer_state"]["state"]) == n_params
    assert float(ck["optimizer_state"]["state"][0]["step"]) == 3 * len(tr)
