#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/.

Two kinds:

1. Reference vectors — produced by IMPORTING the reference Python
   (``/root/reference``, only present in the development container) with the
   ``tools/loguru_stub`` on ``sys.path`` (loguru is not installed). The
   reference's own classes compute every expected output: towers, losses, a
   full ``TwoTowerTrainer.train_epoch`` step, ``generate_recommendations`` and
   the MovieLens feature builders. Only inputs/outputs (arrays) are written.
2. Dyadic Flat-IP vectors — Faiss (the reference's IndexFlatIP backend) is not
   installed, so these are built from exactly-summable inputs whose expected
   top-K is computed in float64 (exact for these inputs, hence identical to any
   fp32 summation order Faiss/BLAS/MFMA might use).

Usage: python tools/make_goldens.py [--ref /root/reference] [--out tests/golden]
The GPU box never runs this (no /root/reference there); the .npz files travel.
"""
from __future__ import annotations

import argparse
import os
import sys
import tempfile
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent


def _save(out: Path, name: str, **arrays):
    out.mkdir(parents=True, exist_ok=True)
    clean = {}
    for k, v in arrays.items():
        if isinstance(v, torch.Tensor):
            v = v.detach().cpu().numpy()
        clean[k] = np.asarray(v)
    np.savez_compressed(out / f"{name}.npz", **clean)
    size = (out / f"{name}.npz").stat().st_size
    print(f"  wrote {name}.npz ({size / 1024:.1f} KiB, {len(clean)} arrays)")


def _state_arrays(prefix: str, module: torch.nn.Module):
    return {f"{prefix}/{k}": v.detach().clone() for k, v in module.state_dict().items()}


def _randomize_bn(module: torch.nn.Module, g: torch.Generator):
    """Give BatchNorm non-trivial running stats and affine params so eval-mode BN
    is not the identity."""
    for m in module.modules():
        if isinstance(m, torch.nn.BatchNorm1d):
            with torch.no_grad():
                m.running_mean.copy_(torch.randn(m.num_features, generator=g) * 0.3)
                m.running_var.copy_(torch.rand(m.num_features, generator=g) * 1.5 + 0.25)
                m.weight.copy_(1.0 + 0.2 * torch.randn(m.num_features, generator=g))
                m.bias.copy_(0.1 * torch.randn(m.num_features, generator=g))


def _tower_case(out, name, tower, num_in, cat_in=None, content=None, seed=0):
    g = torch.Generator().manual_seed(seed + 1000)
    _randomize_bn(tower, g)
    init = _state_arrays("state", tower)
    tower.eval()
    with torch.no_grad():
        out_eval = tower(num_in, cat_in, content) if content is not None else tower(num_in, cat_in)
    tower.train()
    x = num_in.clone().requires_grad_(True)
    y = tower(x, cat_in, content) if content is not None else tower(x, cat_in)
    r = torch.randn(y.shape, generator=g)
    (y * r).sum().backward()
    grads = {f"grad/{k}": p.grad.detach().clone() for k, p in tower.named_parameters() if p.grad is not None}
    post = {f"post/{k}": v.detach().clone() for k, v in tower.state_dict().items()
            if "running" in k or "num_batches" in k}
    cat = {f"cat/{k}": v for k, v in (cat_in or {}).items()}
    extra = {"content": content} if content is not None else {}
    _save(out, name, x=num_in, out_eval=out_eval, out_train=y, r=r, grad_x=x.grad, **init, **grads,
          **post, **cat, **extra)


def gen_reference(ref: Path, out: Path):
    sys.path.insert(0, str(HERE / "loguru_stub"))
    sys.path.insert(0, str(ref))
    from src.models.two_tower import UserTower, ItemTower, TwoTowerModel  # noqa: E402
    from src.training.utils import create_two_tower_model_for_training  # noqa: E402
    from src.training.trainers.two_tower import TwoTowerTrainer  # noqa: E402
    from src.data import movielens as ml  # noqa: E402
    import importlib.util  # noqa: E402

    print("reference towers")
    torch.manual_seed(0)
    ut = UserTower(3, 128, [256, 128], dropout_rate=0.0)
    _tower_case(out, "tower_user_c2", ut, torch.randn(64, 3), seed=1)
    torch.manual_seed(1)
    it = ItemTower(20, 128, [256, 128], dropout_rate=0.0, use_content_embedding=False)
    xi = (torch.rand(64, 20) < 0.15).float()
    xi[:, 18] = torch.rand(64)
    xi[:, 19] = torch.rand(64)
    _tower_case(out, "tower_item_c2", it, xi, seed=2)
    torch.manual_seed(2)
    ct = UserTower(10, 32, [64, 32], dropout_rate=0.0,
                   categorical_features={"category": 10, "subcategory": 5})
    cat = {"category": torch.randint(0, 11, (16,)), "subcategory": torch.randint(0, 6, (16,))}
    cat["category"][0] = 0  # padding_idx row
    _tower_case(out, "tower_user_cat", ct, torch.randn(16, 10), cat_in=cat, seed=3)
    torch.manual_seed(3)
    cn = ItemTower(15, 32, [64, 32], dropout_rate=0.0, use_content_embedding=True,
                   content_embedding_dim=768)
    _tower_case(out, "tower_item_content", cn, torch.randn(16, 15), content=torch.randn(16, 768), seed=4)
    for j, act in enumerate(["gelu", "leaky_relu", "tanh", "sigmoid"]):
        torch.manual_seed(10 + j)
        at = UserTower(10, 32, [64, 48], dropout_rate=0.0, activation=act)
        _tower_case(out, f"tower_act_{act}", at, torch.randn(32, 10), seed=20 + j)

    print("reference losses")
    dummy = TwoTowerModel(UserTower(4, 8, [8]), ItemTower(4, 8, [8], use_content_embedding=False),
                          temperature=0.05)
    for b, d in [(8, 64), (8, 128), (256, 64), (256, 128), (1024, 128)]:
        g = torch.Generator().manual_seed(b * 1000 + d)
        u = torch.nn.functional.normalize(torch.randn(b, d, generator=g), dim=-1).requires_grad_(True)
        i = torch.nn.functional.normalize(torch.randn(b, d, generator=g), dim=-1).requires_grad_(True)
        loss = dummy.in_batch_negative_loss(u, i)
        loss.backward()
        _save(out, f"loss_inbatch_B{b}_D{d}", u=u, i=i, tau=np.float32(0.05), loss=loss,
              grad_u=u.grad, grad_i=i.grad)
    g = torch.Generator().manual_seed(77)
    b, n, d = 64, 16, 128
    u = torch.nn.functional.normalize(torch.randn(b, d, generator=g), dim=-1).requires_grad_(True)
    p = torch.nn.functional.normalize(torch.randn(b, d, generator=g), dim=-1).requires_grad_(True)
    ng = torch.nn.functional.normalize(torch.randn(b * n, d, generator=g), dim=-1).requires_grad_(True)
    with torch.no_grad():
        dummy.user_bias.fill_(0.3)
        dummy.item_bias.fill_(-0.2)
    dummy.zero_grad()
    loss = dummy.contrastive_loss(u, p, ng)
    loss.backward()
    _save(out, "loss_contrastive", u=u, p=p, n=ng, tau=np.float32(0.05), user_bias=np.float32(0.3),
          item_bias=np.float32(-0.2), loss=loss, grad_u=u.grad, grad_p=p.grad, grad_n=ng.grad,
          grad_user_bias=dummy.user_bias.grad, grad_item_bias=dummy.item_bias.grad)
    sim = dummy.compute_similarity(u.detach(), p.detach())
    _save(out, "similarity", u=u, i=p, tau=np.float32(0.05), user_bias=np.float32(0.3),
          item_bias=np.float32(-0.2), sim=sim)

    print("reference trainer step (C2 architecture, 2 steps)")
    torch.manual_seed(5)
    model = create_two_tower_model_for_training(3, 20, {"embedding_dim": 128, "hidden_layers": [256, 128],
                                                        "dropout_rate": 0.0, "temperature": 0.05})
    init = {**_state_arrays("user", model.user_tower), **_state_arrays("item", model.item_tower)}
    g = torch.Generator().manual_seed(6)
    batches = []
    for _ in range(2):
        bsz, nneg = 64, 16
        uf = torch.randn(bsz, 3, generator=g)
        pf = (torch.rand(bsz, 20, generator=g) < 0.15).float()
        pf[:, 18:] = torch.rand(bsz, 2, generator=g)
        nf = (torch.rand(bsz, nneg, 20, generator=g) < 0.15).float()
        nf[:, :, 18:] = torch.rand(bsz, nneg, 2, generator=g)
        batches.append({"user_features": uf, "pos_item_features": pf, "neg_item_features": nf})
    with tempfile.TemporaryDirectory() as td:
        trainer = TwoTowerTrainer(model, [batches[0]], [batches[0]],
                                  {"learning_rate": 1e-3, "weight_decay": 1e-5, "checkpoint_dir": td})
        trainer.train_epoch(1)
        mid = {**_state_arrays("mid_user", model.user_tower), **_state_arrays("mid_item", model.item_tower),
               "mid_user_bias": model.user_bias.detach().clone(),
               "mid_item_bias": model.item_bias.detach().clone()}
        trainer.train_loader = [batches[1]]
        trainer.train_epoch(2)
        final = {**_state_arrays("final_user", model.user_tower), **_state_arrays("final_item", model.item_tower),
                 "final_user_bias": model.user_bias.detach().clone(),
                 "final_item_bias": model.item_bias.detach().clone()}
        losses = np.array(trainer.train_losses, np.float64)
        model.eval()
        val_loss = trainer.validate()
    _save(out, "train_step_c2", **init, **mid, **final, losses=losses, val_loss=np.float64(val_loss),
          temperature=np.float32(0.05),
          **{f"b{j}_{k}": v for j, bt in enumerate(batches) for k, v in bt.items()})

    print("reference generate_recommendations (masked top-100)")
    spec = importlib.util.spec_from_file_location("ref_evaluate_model", ref / "scripts" / "evaluate_model.py")
    evm = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(evm)
    torch.manual_seed(7)
    m2 = create_two_tower_model_for_training(3, 20, {"embedding_dim": 64, "hidden_layers": [128, 64],
                                                     "dropout_rate": 0.2, "temperature": 0.05})
    _randomize_bn(m2, torch.Generator().manual_seed(8))
    m2.eval()
    rng = np.random.default_rng(9)
    uf = rng.standard_normal((600, 3)).astype(np.float32)
    mf = (rng.random((400, 20)) < 0.15).astype(np.float32)
    mf[:, 18:] = rng.random((400, 2)).astype(np.float32)
    test_users = sorted(rng.choice(600, 300, replace=False).tolist())
    train_items = {u: sorted(rng.choice(400, int(rng.integers(0, 40)), replace=False).tolist())
                   for u in test_users}
    recs = evm.generate_recommendations(m2, test_users, train_items, uf, mf, top_k=100, batch_size=256)
    with torch.no_grad():
        ue = m2.get_user_embeddings({"numerical": torch.from_numpy(uf), "categorical": {}}).numpy()
        ie = m2.get_item_embeddings({"numerical": torch.from_numpy(mf), "categorical": {}}).numpy()
    excl = np.full((len(test_users), 40), -1, np.int64)
    for r, u in enumerate(test_users):
        excl[r, :len(train_items[u])] = train_items[u]
    _save(out, "eval_topk", **_state_arrays("user", m2.user_tower), **_state_arrays("item", m2.item_tower),
          user_features=uf, movie_features=mf, test_users=np.array(test_users, np.int64),
          exclude=excl, recs=np.array([recs[u] for u in test_users], np.int64),
          user_emb=ue, item_emb=ie)

    print("reference MovieLens feature builders")
    with tempfile.TemporaryDirectory() as td:
        td = Path(td)
        rng = np.random.default_rng(11)
        lines = []
        for u in range(1, 13):
            for mv in rng.choice(np.arange(1, 16), 7, replace=False):
                lines.append(f"{u}::{mv}::{int(rng.integers(1, 6))}::{978300000 + int(rng.integers(0, 10**6))}")
        (td / "ratings.dat").write_text("\n".join(lines) + "\n")
        ul = []
        for u in range(1, 13):
            ul.append(f"{u}::{'MF'[u % 2]}::{[1, 18, 25, 35, 45, 50, 56][u % 7]}::{u % 21}::{10000 + u}")
        (td / "users.dat").write_text("\n".join(ul) + "\n")
        genres = ml.MovieLensLoader.GENRES
        mlines = []
        for mv in range(1, 16):
            gs = "|".join(sorted(set(rng.choice(genres, int(rng.integers(1, 4))).tolist())))
            mlines.append(f"{mv}::Movie {mv} ({1930 + 5 * mv})::{gs}")
        (td / "movies.dat").write_text("\n".join(mlines) + "\n")
        loader = ml.MovieLensLoader(str(td))
        data = loader.load_and_preprocess(split_method="time", min_user_interactions=1,
                                          min_item_interactions=1)
        uidx = np.arange(data.users["user_idx"].max() + 1)
        midx = np.arange(data.movies["movie_idx"].max() + 1)
        ufeat = ml.create_user_features(data.users, uidx, normalize=True)
        mfeat = ml.create_movie_features(data.movies, midx, normalize=True)
        pos = ml.get_user_positive_items(data.train_interactions)
        pos_arr = np.full((len(uidx), 16), -1, np.int64)
        for u, its in pos.items():
            pos_arr[u, :len(its)] = its
        cols = ["user_idx", "movie_idx", "label", "timestamp", "user_id", "movie_id", "rating"]
        _save(out, "movielens_tiny",
              ratings_dat=np.array((td / "ratings.dat").read_text()),
              users_dat=np.array((td / "users.dat").read_text()),
              movies_dat=np.array((td / "movies.dat").read_text()),
              user_features=ufeat, movie_features=mfeat, positives=pos_arr,
              **{f"train_{c}": data.train_interactions[c].to_numpy() for c in cols},
              **{f"val_{c}": data.val_interactions[c].to_numpy() for c in cols},
              **{f"test_{c}": data.test_interactions[c].to_numpy() for c in cols},
              num_users=np.int64(data.num_users), num_movies=np.int64(data.num_movies))

    print("reference parameter counts")
    counts = {}
    for emb, hid, name in [(128, [256, 128], "c2"), (64, [256, 128], "c1")]:
        mm = create_two_tower_model_for_training(3, 20, {"embedding_dim": emb, "hidden_layers": hid})
        counts[name] = sum(p.numel() for p in mm.parameters())
    _save(out, "param_counts", **{k: np.int64(v) for k, v in counts.items()})


def gen_reference_r2(ref: Path, out: Path):
    """Round-2 fixtures: the reference Evaluator on the eval_topk recommendations,
    and checkpoints written by the reference's own save_model / save_checkpoint."""
    sys.path.insert(0, str(HERE / "loguru_stub"))
    sys.path.insert(0, str(ref))
    from src.training.utils import create_two_tower_model_for_training  # noqa: E402
    from src.training.trainers.two_tower import TwoTowerTrainer  # noqa: E402
    from src.evaluation.metrics import Evaluator  # noqa: E402

    print("reference Evaluator.evaluate on the eval_topk recommendations")
    with np.load(out / "eval_topk.npz", allow_pickle=False) as z:
        recs, test_users, excl = z["recs"], z["test_users"], z["exclude"]
    rng = np.random.default_rng(21)
    n_items = 400
    preds, gt, ex = {}, {}, {}
    for r, u in enumerate(test_users.tolist()):
        u = int(u)
        train = set(int(x) for x in excl[r] if x >= 0)
        pool = np.array(sorted(set(range(n_items)) - train))
        # ground truth: a few of the top recommendations plus random held-out items
        n_gt = int(rng.integers(0, 12))
        picks = set(rng.choice(pool, n_gt, replace=False).tolist()) if n_gt else set()
        if rng.random() < 0.5:
            picks |= set(int(x) for x in recs[r, rng.integers(0, 100, 3)])
        gt[u] = picks
        preds[u] = [int(x) for x in recs[r]]
        ex[u] = train
    # users present in predictions but not in the ground truth are skipped by the Evaluator
    for u in range(1000, 1010):
        preds[u] = list(range(100))
    ev = Evaluator(k_values=[5, 10, 20, 50, 100], num_items=n_items)
    m = ev.evaluate(preds, gt, ex)
    # a second run where predictions contain excluded items (the Evaluator's filter shifts ranks)
    preds2 = {u: (sorted(ex[u])[:5] + p) for u, p in preds.items() if u in ex}
    m2 = ev.evaluate(preds2, gt, ex)
    gt_arr = np.full((len(test_users), 20), -1, np.int64)
    for r, u in enumerate(test_users.tolist()):
        g = sorted(gt[int(u)])
        gt_arr[r, :len(g)] = g
    p2 = np.full((len(test_users), 105), -1, np.int64)
    for r, u in enumerate(test_users.tolist()):
        row = preds2[int(u)]
        p2[r, :len(row)] = row

    def flat(mm, tag):
        d = {f"{tag}/{k}": np.float64(v) for k, v in mm.to_dict().items()}
        for k in mm.per_user_recall:
            d[f"{tag}/per_user_recall@{k}"] = np.asarray(mm.per_user_recall[k], np.float64)
            d[f"{tag}/per_user_ndcg@{k}"] = np.asarray(mm.per_user_ndcg[k], np.float64)
        return d
    _save(out, "eval_metrics", test_users=test_users, recs=recs, exclude=excl, ground_truth=gt_arr,
          preds_with_excluded=p2, k_values=np.array([5, 10, 20, 50, 100], np.int64), num_items=np.int64(n_items),
          **flat(m, "plain"), **flat(m2, "filtered"))

    print("reference checkpoints (save_model, TwoTowerTrainer.save_checkpoint)")
    torch.manual_seed(31)
    model = create_two_tower_model_for_training(3, 20, {"embedding_dim": 64, "hidden_layers": [128, 64],
                                                        "dropout_rate": 0.0, "temperature": 0.05})
    g = torch.Generator().manual_seed(32)
    batches = []
    for _ in range(2):
        bsz, nneg = 64, 8
        uf = torch.randn(bsz, 3, generator=g)
        pf = (torch.rand(bsz, 20, generator=g) < 0.15).float()
        pf[:, 18:] = torch.rand(bsz, 2, generator=g)
        nf = (torch.rand(bsz, nneg, 20, generator=g) < 0.15).float()
        nf[:, :, 18:] = torch.rand(bsz, nneg, 2, generator=g)
        batches.append({"user_features": uf, "pos_item_features": pf, "neg_item_features": nf})
    with tempfile.TemporaryDirectory() as td:
        trainer = TwoTowerTrainer(model, [batches[0]], [batches[0]],
                                  {"learning_rate": 1e-3, "weight_decay": 1e-5, "checkpoint_dir": td})
        trainer.train_epoch(1)
        trainer.save_checkpoint(1, is_best=True)
        ck_bytes = (Path(td) / "two_tower_best.pth").read_bytes()
        model.save_model(str(Path(td) / "model.pth"))
        sm_bytes = (Path(td) / "model.pth").read_bytes()
        # what the reference model computes from these weights (eval mode)
        model.eval()
        q_u = torch.randn(32, 3, generator=g)
        q_i = (torch.rand(48, 20, generator=g) < 0.15).float()
        q_i[:, 18:] = torch.rand(48, 2, generator=g)
        with torch.no_grad():
            ue = model.get_user_embeddings({"numerical": q_u, "categorical": {}})
            ie = model.get_item_embeddings({"numerical": q_i, "categorical": {}})
        # the step after the checkpoint, continued by the same reference optimizer
        model.train()
        trainer.train_loader = [batches[1]]
        trainer.train_epoch(2)
        after = {**_state_arrays("after_user", model.user_tower), **_state_arrays("after_item", model.item_tower)}
    (out / "ckpt_ref_trainer.pth").write_bytes(ck_bytes)
    (out / "ckpt_ref_model.pth").write_bytes(sm_bytes)
    print(f"  wrote ckpt_ref_trainer.pth ({len(ck_bytes) / 1024:.1f} KiB), ckpt_ref_model.pth "
          f"({len(sm_bytes) / 1024:.1f} KiB)")
    _save(out, "ckpt_ref_expect", q_user=q_u, q_item=q_i, user_emb=ue, item_emb=ie,
          losses=np.array(trainer.train_losses, np.float64), **after,
          **{f"b1_{k}": v for k, v in batches[1].items()})


def gen_reference_r3(ref: Path, out: Path):
    """Round-3 fixture: the reference generate_recommendations on heavy users
    (more train items than top_k leaves eligible), whose lists the reference
    pads with its -inf train items (scripts/evaluate_model.py:224-232)."""
    sys.path.insert(0, str(HERE / "loguru_stub"))
    sys.path.insert(0, str(ref))
    from src.training.utils import create_two_tower_model_for_training  # noqa: E402

    import importlib.util

    print("reference generate_recommendations on heavy users (padded lists)")
    spec = importlib.util.spec_from_file_location("ref_evaluate_model", ref / "scripts" / "evaluate_model.py")
    evm = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(evm)
    torch.manual_seed(41)
    m = create_two_tower_model_for_training(3, 20, {"embedding_dim": 64, "hidden_layers": [128, 64],
                                                    "dropout_rate": 0.2, "temperature": 0.05})
    _randomize_bn(m, torch.Generator().manual_seed(42))
    m.eval()
    rng = np.random.default_rng(43)
    n_items, n_users = 160, 120
    uf = rng.standard_normal((n_users, 3)).astype(np.float32)
    mf = (rng.random((n_items, 20)) < 0.15).astype(np.float32)
    mf[:, 18:] = rng.random((n_items, 2)).astype(np.float32)
    test_users = sorted(rng.choice(n_users, 60, replace=False).tolist())
    # 0..150 train items: most users leave fewer than 100 eligible items
    train_items = {u: sorted(rng.choice(n_items, int(rng.integers(0, 151)), replace=False).tolist())
                   for u in test_users}
    recs = evm.generate_recommendations(m, test_users, train_items, uf, mf, top_k=100, batch_size=256)
    excl = np.full((len(test_users), 160), -1, np.int64)
    for r, u in enumerate(test_users):
        excl[r, :len(train_items[u])] = train_items[u]
    _save(out, "eval_topk_heavy", **_state_arrays("user", m.user_tower), **_state_arrays("item", m.item_tower),
          user_features=uf, movie_features=mf, test_users=np.array(test_users, np.int64), exclude=excl,
          recs=np.array([recs[u] for u in test_users], np.int64))

    print("reference Adam moments after the step that follows ckpt_ref_trainer.pth")
    from src.training.trainers.two_tower import TwoTowerTrainer  # noqa: E402
    ck = torch.load(out / "ckpt_ref_trainer.pth", map_location="cpu", weights_only=True)
    with np.load(out / "ckpt_ref_expect.npz", allow_pickle=False) as z:
        b1 = {k[3:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("b1_")}
    model = create_two_tower_model_for_training(3, 20, {"embedding_dim": 64, "hidden_layers": [128, 64],
                                                        "dropout_rate": 0.0, "temperature": 0.05})
    model.user_tower.load_state_dict(ck["user_tower_state"])
    model.item_tower.load_state_dict(ck["item_tower_state"])
    with torch.no_grad():
        model.user_bias.copy_(ck["user_bias"])
        model.item_bias.copy_(ck["item_bias"])
    with tempfile.TemporaryDirectory() as td:
        trainer = TwoTowerTrainer(model, [b1], [b1], {"learning_rate": 1e-3, "weight_decay": 1e-5,
                                                      "checkpoint_dir": td})
        trainer.optimizer.load_state_dict(ck["optimizer_state"])
        trainer.train_epoch(2)
    st = trainer.optimizer.state_dict()["state"]
    moments = {}
    for i, v in st.items():
        moments[f"exp_avg/{i}"] = v["exp_avg"].numpy()
        moments[f"exp_avg_sq/{i}"] = v["exp_avg_sq"].numpy()
        moments[f"step/{i}"] = np.float64(float(v["step"]))
    _save(out, "ckpt_ref_moments", **moments)


def _dyadic_unit(rng, n, d, nnz=16):
    """Unit-norm rows with `nnz` entries of ±1/4 (nnz=16): the renorm is exactly
    the identity and every inner product is an exact multiple of 1/16."""
    x = np.zeros((n, d), np.float32)
    for r in range(n):
        cols = rng.choice(d, nnz, replace=False)
        x[r, cols] = rng.choice([-0.25, 0.25], nnz)
    return x


def _exact_topk(q, x, k, excl=None):
    s = q.astype(np.float64) @ x.astype(np.float64).T
    if excl is not None:
        s = np.where(excl, -np.inf, s)
    ids = np.broadcast_to(np.arange(x.shape[0]), s.shape)
    order = np.lexsort((ids, -s), axis=1)[:, :k]
    sc = np.take_along_axis(s, order, 1)
    if order.shape[1] < k:  # k > N: Faiss pads with (-FLT_MAX, -1)
        pad = k - order.shape[1]
        order = np.pad(order, ((0, 0), (0, pad)))
        sc = np.pad(sc, ((0, 0), (0, pad)), constant_values=-np.inf)
    valid = np.isfinite(sc)
    out_ids = np.where(valid, order, -1).astype(np.int64)
    out_s = np.where(valid, sc, -np.finfo(np.float32).max).astype(np.float32)
    return out_s, out_ids


def gen_dyadic(out: Path):
    print("dyadic Flat-IP fixtures (no reference needed)")
    rng = np.random.default_rng(1234)
    # normalized path (index build + search normalize, retrieval.py:86,167)
    x = _dyadic_unit(rng, 1000, 64)
    x[500:520] = x[100:120]  # planted exact duplicates → exact ties
    q = _dyadic_unit(rng, 200, 64)
    q[:10] = x[100:110]
    cases = {}
    for k in (1, 10, 100):
        s, i = _exact_topk(q, x, k)
        cases[f"k{k}_scores"], cases[f"k{k}_ids"] = s, i
    _save(out, "flatip_dyadic_unit", queries=q, items=x, **cases)
    # raw (un-normalized) multiples of 2^-6 in [-1, 1], D=128, with exclusion mask
    x = (rng.integers(-64, 65, (3000, 128)) / 64.0).astype(np.float32)
    x[2000:2100] = x[:100]
    q = (rng.integers(-64, 65, (300, 128)) / 64.0).astype(np.float32)
    excl = rng.random((300, 3000)) < 0.05
    cases = {}
    for k in (10, 100, 256):
        s, i = _exact_topk(q, x, k)
        cases[f"k{k}_scores"], cases[f"k{k}_ids"] = s, i
    s, i = _exact_topk(q, x, 100, excl)
    bm = np.zeros((300, (3000 + 31) // 32), np.uint32)
    rr, cc = np.nonzero(excl)
    np.bitwise_or.at(bm, (rr, cc >> 5), (np.uint32(1) << (cc & 31).astype(np.uint32)))
    _save(out, "flatip_dyadic_raw", queries=q, items=x, exclude_bits=bm, excl_k100_scores=s,
          excl_k100_ids=i, **cases)
    # tiny corpus: k > N → (-FLT_MAX, -1) padding (retrieval.py:183 drops them)
    x = _dyadic_unit(rng, 7, 32, nnz=16)
    q = _dyadic_unit(rng, 5, 32, nnz=16)
    s, i = _exact_topk(q, x, 10)
    _save(out, "flatip_dyadic_small", queries=q, items=x, k10_scores=s, k10_ids=i)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=str(HERE.parent / "tests" / "golden"))
    ap.add_argument("--only", choices=["reference", "dyadic", "r2", "r3"], default=None)
    a = ap.parse_args()
    out = Path(a.out)
    if a.only in (None, "dyadic"):
        gen_dyadic(out)
    if a.only in (None, "reference"):
        ref = Path(a.ref)
        if not (ref / "src" / "models" / "two_tower.py").exists():
            print(f"reference not found at {ref}; skipping reference vectors")
            return
        gen_reference(ref, out)
    if a.only in (None, "reference", "r2"):
        ref = Path(a.ref)
        if (ref / "src" / "models" / "two_tower.py").exists():
            gen_reference_r2(ref, out)
    if a.only in (None, "reference", "r3"):
        ref = Path(a.ref)
        if (ref / "src" / "models" / "two_tower.py").exists():
            gen_reference_r3(ref, out)


if __name__ == "__main__":
    main()
