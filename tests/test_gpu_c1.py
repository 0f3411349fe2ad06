"""Config C1 (BASELINE.json configs[0]): the reference's
``scripts/train_movielens.py --embedding-dim 64 --batch-size 256 --epochs 1``
pipeline, through this build's entry ``rtrec_amd.train_movielens`` (device
feeder + fused step + TwoTowerTrainer), on the ML-1M-shaped synthetic stream
(6,040 users x 3,416 movies, ~1M ratings; ratings.dat is not available).

One full epoch (every train batch, dropout 0) is replayed batch by batch
through oracle/two_tower.train_step on the SAME id batches (the feeder is
deterministic: same seed, same shuffle, same on-device negatives), from the
same initial weights. Bars: the early steps' losses within 1e-4 relative
(north_star); the epoch-1 mean loss — the number the reference logs — within
1e-3 relative (thousands of Adam steps let fp32 rounding differences grow; see
the measured gap printed by the test)."""
import json

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(600)
def test_c1_one_epoch_vs_oracle(device, tmp_path):
    from oracle import two_tower as orc
    from rtrec_amd import train_movielens as tm
    from rtrec_amd.training.datasets.movielens import DeviceFeeder
    from rtrec_amd.training.utils import create_two_tower_model_for_training

    args = tm.build_parser().parse_args([
        "--synthetic", "--epochs", "1", "--batch-size", "256", "--embedding-dim", "64", "--dropout", "0",
        "--init-seed", "1234", "--checkpoint-dir", str(tmp_path / "ckpt"), "--output-dir", str(tmp_path / "out")])
    res = tm.run(args)
    got = np.asarray(res["trainer"].last_epoch_step_losses, np.float64)
    assert res["epochs_run"] == 1 and len(got) == res["batches_last_epoch"] > 2000
    assert np.isfinite(got).all()

    # artefacts of the reference script: checkpoints with the reference keys, metadata
    ck = torch.load(tmp_path / "ckpt" / "two_tower_best.pth", map_location="cpu", weights_only=True)
    assert {"epoch", "user_tower_state", "item_tower_state", "temperature", "user_bias", "item_bias",
            "optimizer_state", "train_losses", "val_losses"} <= set(ck)
    meta = json.loads((tmp_path / "ckpt" / "data_metadata.json").read_text())
    assert meta["user_feature_dim"] == 3 and meta["movie_feature_dim"] == 20

    # oracle: same initial weights, same batches
    torch.manual_seed(1234)
    m0 = create_two_tower_model_for_training(3, 20, {"embedding_dim": 64, "hidden_layers": [256, 128],
                                                     "dropout_rate": 0.0, "temperature": 0.05})
    us = {k: v.detach().clone() for k, v in m0.user_tower.state_dict().items()}
    its = {k: v.detach().clone() for k, v in m0.item_tower.state_dict().items()}
    biases = {"user_bias": torch.zeros(1), "item_bias": torch.zeros(1)}
    data, _ = tm.load_data(args)
    n_train = len(data.train_interactions)
    feeder = DeviceFeeder(data.train_interactions, data.users, data.movies, num_negatives=16, batch_size=256,
                          device=device, seed=0, shuffle=True, drop_last=n_train % 256 == 1)
    uf = feeder.user_table.cpu()
    mf = feeder.item_table.cpu()
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    opt, ref = {}, []
    for b in feeder:
        u = uf[b["user_ids"].cpu()]
        p = mf[b["pos_ids"].cpu()]
        n = mf[b["neg_ids"].cpu()].view(u.shape[0], 16, 20)
        r = orc.train_step(us, its, biases, opt, u, p, n, temperature=0.05, lr=1e-3, weight_decay=1e-5)
        ref.append(r["loss"])
    ref = np.asarray(ref)
    assert len(ref) == len(got)
    early = np.abs(got[:10] - ref[:10]) / np.abs(ref[:10])
    gap = abs(got.mean() - ref.mean()) / ref.mean()
    print(f"C1 epoch-1 mean loss: HIP {got.mean():.6f} oracle {ref.mean():.6f} rel gap {gap:.2e}; "
          f"first-10 max rel {early.max():.2e}; steps {len(got)}")
    assert early.max() <= 1e-4, early
    assert gap <= 1e-3, gap
    assert abs(res["train_losses"][0] - got.mean()) <= 1e-9 * abs(got.mean())


@pytest.mark.timeout(300)
def test_c1_train_then_evaluate_cli(device, tmp_path):
    """train_movielens → evaluate_model, the reference's two-script workflow
    (scripts/train_movielens.py then scripts/evaluate_model.py), end to end on
    the device: a short training run, then masked top-100 + metrics for every
    test user; the metrics equal the oracle's on the same recommendation lists."""
    from oracle import metrics as om
    from rtrec_amd import evaluate_model as em
    from rtrec_amd import train_movielens as tm
    tm.run(tm.build_parser().parse_args([
        "--synthetic", "--epochs", "1", "--batch-size", "256", "--embedding-dim", "64", "--max-batches", "50",
        "--checkpoint-dir", str(tmp_path / "ckpt"), "--output-dir", str(tmp_path / "out")]))
    res = em.run(em.build_parser().parse_args([
        "--synthetic", "--checkpoint", str(tmp_path / "ckpt" / "two_tower_best.pth"),
        "--output", str(tmp_path / "results.json")]))
    r = json.loads((tmp_path / "results.json").read_text())
    assert r["num_test_users"] > 1000 and 0.0 <= r["recall@10"] <= 1.0
    data, _ = tm.load_data(tm.build_parser().parse_args(["--synthetic"]))
    train_items, gt, _, mf = em.prepare_evaluation_data(data)
    recs = res["recommendations"]
    assert all(len(v) == 100 and not (set(v) & set(train_items.get(u, []))) for u, v in recs.items())
    ref = om.evaluate(recs, gt, [5, 10, 20, 50, 100], num_items=mf.shape[0],
                      exclude_items={u: set(v) for u, v in train_items.items()})
    for key in ("recall@10", "ndcg@10", "hit_rate@10", "mrr", "map", "coverage", "precision@100"):
        np.testing.assert_allclose(r[key], ref[key], rtol=1e-12, err_msg=key)
