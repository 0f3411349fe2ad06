"""Offline evaluation caller of the top-K path (reference scripts/evaluate_model.py).

``generate_recommendations`` (evaluate_model.py:162-234): all item embeddings
once, the user tower over the test users in ``batch_size`` batches, then per
user the train items masked out and the top ``top_k`` items by inner product.
The reference does the last step as ``np.dot`` + ``-inf`` masking + a full-row
``argsort`` (≈299 ms for 6,040 × 3,416 on the survey host); here it is one
``rt_flatip_topk`` launch with the train-item exclusion bitmap built on the
device (``rt_exclusion_bitmap``) from a CSR of the train items — no score
matrix is materialised.

Ordering: (score desc, item id asc). The reference's ``argsort(...)[::-1]``
orders exact score ties by a quicksort-dependent rule; outside exact ties the
lists are identical (tests/test_gpu_eval.py checks this tie-aware against the
reference's own output, tests/golden/eval_topk.npz). When a user has fewer
than ``top_k`` non-train items the reference appends its ``-inf`` train items
in argsort order; by default this build returns only the eligible items (the
reference's Evaluator removes those train items again before scoring,
metrics.py:279-281). ``pad_excluded=True`` returns the reference's full-length
lists instead: such a user's top_k already holds every eligible item with its
score, so the masked score row is known exactly, and the list is
``np.argsort(row)[::-1][:top_k]`` over it — the reference's own call
(evaluate_model.py:225-231), whose order among the ``-inf`` ties is numpy's
(its introsort/SIMD sort is not stable, so no other rule reproduces it).

``load_model`` (evaluate_model.py:36-95): architecture inferred from the
checkpoint's weight shapes, ``weights_only=True``.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from .. import kernels
from ..models.two_tower import ItemTower, TwoTowerModel, UserTower
from .metrics import csr_from_sets


def _dev(device) -> torch.device:
    if device in (None, "auto", "cuda"):
        if not torch.cuda.is_available():
            raise RuntimeError("generate_recommendations: no ROCm device; this MI355X build has no CPU fallback")
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device(device)


@torch.no_grad()
def recommend_tensors(model: TwoTowerModel, user_features: torch.Tensor, item_features: torch.Tensor,
                      test_users: torch.Tensor, train_offsets: torch.Tensor, train_items: torch.Tensor,
                      top_k: int = 100, batch_size: int = 256):
    """Device-resident form: ``user_features`` [n_users, Fu] / ``item_features``
    [n_items, Fi] fp32 tables, ``test_users`` int64 [U], train items as a CSR
    over user rows. Returns (scores fp32 [U, top_k], item ids int64 [U, top_k]),
    (-FLT_MAX, -1) where fewer than top_k items are eligible."""
    item_emb = model.get_item_embeddings({"numerical": item_features, "categorical": {}})
    n_items = item_emb.shape[0]
    u_idx = test_users.to(torch.int64)
    parts = []
    for i in range(0, u_idx.numel(), batch_size):  # evaluate_model.py:201-215 (eval BN: batching is exact)
        uf = kernels.gather_rows(user_features, u_idx[i:i + batch_size], check=True)
        parts.append(model.get_user_embeddings({"numerical": uf, "categorical": {}}))
    user_emb = torch.cat(parts) if len(parts) != 1 else parts[0]
    bits = kernels.exclusion_bitmap_csr(train_offsets, train_items, n_items, rows=u_idx)
    return kernels.flatip_topk(user_emb.contiguous(), item_emb.contiguous(), top_k, exclude_bits=bits)


def _pad_like_reference(ids_row: np.ndarray, scores_row: np.ndarray, n_items: int, top_k: int) -> List[int]:
    """A user with fewer than top_k eligible items: rebuild the reference's masked
    score row (eligible items' scores, -inf elsewhere) and take its argsort,
    as scripts/evaluate_model.py:225-231 does."""
    ok = ids_row >= 0
    row = np.full(n_items, -np.inf, dtype=np.float32)
    row[ids_row[ok]] = scores_row[ok]
    return [int(x) for x in np.argsort(row)[::-1][:top_k]]


def generate_recommendations(model: TwoTowerModel, test_users: list, train_items: Dict[int, list],
                             user_features: np.ndarray, movie_features: np.ndarray, top_k: int = 100,
                             batch_size: int = 256, device: Optional[str] = None,
                             return_tensors: bool = False, pad_excluded: bool = False):
    """evaluate_model.py:162-234 → Dict[user_idx, List[movie_idx]] (or the
    device (scores, ids) with ``return_tensors``). ``pad_excluded``: lists of
    users with fewer than ``top_k`` eligible items are padded with their
    excluded items as the reference pads them (see the module docstring)."""
    dev = _dev(device)
    uf = torch.as_tensor(np.asarray(user_features, np.float32)).to(dev)
    mf = torch.as_tensor(np.asarray(movie_features, np.float32)).to(dev)
    users = [int(u) for u in test_users]
    n_users = uf.shape[0]
    rows: List[Optional[Sequence[int]]] = [None] * n_users
    for u, its in train_items.items():
        if 0 <= int(u) < n_users:
            rows[int(u)] = its
    t_off, t_items = csr_from_sets(rows, dev)
    scores, ids = recommend_tensors(model, uf, mf, torch.tensor(users, dtype=torch.int64, device=dev), t_off,
                                    t_items, top_k=top_k, batch_size=batch_size)
    if return_tensors:
        return scores, ids
    host = ids.cpu().numpy()
    if not pad_excluded:
        return {u: [int(x) for x in host[r] if x >= 0] for r, u in enumerate(users)}
    n_items = mf.shape[0]
    host_s = scores.cpu().numpy()
    out = {}
    for r, u in enumerate(users):
        if top_k <= n_items and (host[r] < 0).any():
            out[u] = _pad_like_reference(host[r], host_s[r], n_items, top_k)
        else:
            out[u] = [int(x) for x in host[r] if x >= 0]
    return out


def load_model(checkpoint_path: str, user_dim: int, item_dim: int, device: Optional[str] = None) -> TwoTowerModel:
    """evaluate_model.py:36-95: hidden sizes from mlp.0 / mlp.4, embedding dim from
    mlp.8 (two hidden layers, as the reference infers), dropout 0.2, ReLU, no
    content projection, biases not restored (the reference ignores them)."""
    ck = torch.load(checkpoint_path, map_location="cpu", weights_only=True)
    us = ck["user_tower_state"]
    hidden = [us["mlp.0.weight"].shape[0], us["mlp.4.weight"].shape[0]]
    emb = us["mlp.8.weight"].shape[0]
    ut = UserTower(input_dim=user_dim, embedding_dim=emb, hidden_layers=hidden, dropout_rate=0.2, activation="relu")
    it = ItemTower(input_dim=item_dim, embedding_dim=emb, hidden_layers=hidden, dropout_rate=0.2, activation="relu",
                   use_content_embedding=False)
    model = TwoTowerModel(user_tower=ut, item_tower=it, temperature=ck.get("temperature", 0.1), use_bias=True)
    model.user_tower.load_state_dict(ck["user_tower_state"])
    model.item_tower.load_state_dict(ck["item_tower_state"])
    model.to(_dev(device))
    model.eval()
    return model
