"""ORACLE — test infrastructure only (see oracle/__init__.py).

Functional torch-CPU restatement of the reference two-tower math:

* towers ``UserTower.forward`` / ``ItemTower.forward``
  (src/models/two_tower.py:56-72, 98-134, 184-212, 238-281);
* ``compute_similarity`` (:380-404), ``contrastive_loss`` (:406-451),
  ``in_batch_negative_loss`` (:453-479);
* the trainer step ``TwoTowerTrainer.train_epoch`` inner loop
  (src/training/trainers/two_tower.py:98-146): 0.7 explicit + 0.3 in-batch,
  ``clip_grad_norm_(1.0)`` and ``Adam(lr, weight_decay)``;
* the feature-row gathers of ``MovieLensDataset.__getitem__``
  (src/training/datasets/movielens.py:108-116).

Parameters are plain tensors in the reference ``state_dict`` key layout
(``mlp.{4l}.weight`` = hidden Linear l, ``mlp.{4l+2}.*`` = its BatchNorm1d,
``mlp.{4L}.*`` = final projection), so reference checkpoints and golden
fixtures map 1:1. Gradients come from CPU autograd, exactly as the reference
computes them.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.nn.functional as F

# src/models/two_tower.py:77-86 (unknown names fall back to ReLU)
_ACTS = {
    "relu": F.relu,
    "gelu": F.gelu,
    "leaky_relu": lambda x: F.leaky_relu(x, 0.1),
    "tanh": torch.tanh,
    "sigmoid": torch.sigmoid,
}


def activation_fn(name: str):
    return _ACTS.get(name, F.relu)


def n_hidden_layers(state: Dict[str, torch.Tensor]) -> int:
    """Number of [Linear, act, BN, Dropout] blocks in a tower state dict."""
    idx = sorted(int(k.split(".")[1]) for k in state if k.startswith("mlp.") and k.endswith(".weight")
                 and f"mlp.{k.split('.')[1]}.running_mean" not in state)
    return idx[-1] // 4


def gather_rows(table: np.ndarray, ids: np.ndarray) -> np.ndarray:
    """``self.user_features[user_idx]`` / ``self.movie_features[neg_item_indices]``
    (src/training/datasets/movielens.py:108-116): numpy fancy indexing."""
    return table[np.asarray(ids, dtype=np.int64)]


def tower_forward(state: Dict[str, torch.Tensor], numerical: torch.Tensor,
                  categorical: Optional[Dict[str, torch.Tensor]] = None,
                  content: Optional[torch.Tensor] = None, *, train: bool = False,
                  dropout_p: float = 0.0, activation: str = "relu",
                  bn_eps: float = 1e-5, bn_momentum: float = 0.1,
                  use_content: bool = True) -> torch.Tensor:
    """UserTower/ItemTower forward (two_tower.py:98-134 / 238-281).
    Updates ``running_mean``/``running_var``/``num_batches_tracked`` in ``state``
    when ``train`` (BatchNorm1d training semantics)."""
    act = activation_fn(activation)
    embedded: List[torch.Tensor] = []
    if categorical:
        for name, t in categorical.items():  # two_tower.py:115-119 (dict order)
            w = state.get(f"embeddings.{name}.weight")
            if w is not None:
                embedded.append(F.embedding(t, w, padding_idx=0))
    if content is not None and use_content and "content_projection.0.weight" in state:
        # two_tower.py:184-191, 264-266: Linear(768,256) → ReLU → Dropout → Linear(256,128)
        c = F.linear(content, state["content_projection.0.weight"], state["content_projection.0.bias"])
        c = F.dropout(F.relu(c), dropout_p, training=train)
        c = F.linear(c, state["content_projection.3.weight"], state["content_projection.3.bias"])
        embedded.append(c)
    x = torch.cat([numerical, torch.cat(embedded, dim=-1)], dim=-1) if embedded else numerical
    L = n_hidden_layers(state)
    for layer in range(L):
        x = F.linear(x, state[f"mlp.{4 * layer}.weight"], state[f"mlp.{4 * layer}.bias"])
        x = act(x)
        bn = f"mlp.{4 * layer + 2}"
        x = F.batch_norm(x, state[f"{bn}.running_mean"], state[f"{bn}.running_var"],
                         state[f"{bn}.weight"], state[f"{bn}.bias"], training=train,
                         momentum=bn_momentum, eps=bn_eps)
        if train and f"{bn}.num_batches_tracked" in state:
            state[f"{bn}.num_batches_tracked"] += 1
        x = F.dropout(x, dropout_p, training=train)
    x = F.linear(x, state[f"mlp.{4 * L}.weight"], state[f"mlp.{4 * L}.bias"])
    return F.normalize(x, p=2, dim=-1)  # two_tower.py:132


def compute_similarity(u: torch.Tensor, i: torch.Tensor, temperature: float,
                       user_bias: Optional[torch.Tensor] = None,
                       item_bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """two_tower.py:380-404."""
    s = torch.sum(u * i, dim=-1) / temperature
    if user_bias is not None:
        s = s + user_bias + item_bias
    return s


def contrastive_loss(u: torch.Tensor, pos: torch.Tensor, neg: torch.Tensor, temperature: float,
                     user_bias: Optional[torch.Tensor] = None,
                     item_bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """two_tower.py:406-451: biases on the positive logit only."""
    b = u.shape[0]
    pos_sim = compute_similarity(u, pos, temperature, user_bias, item_bias)
    if neg.shape[0] > b:
        r = neg.shape[0] // b
        neg = neg.view(b, r, -1)
        neg_sim = torch.sum(u.unsqueeze(1).expand(-1, r, -1) * neg, dim=-1) / temperature
    else:
        neg_sim = compute_similarity(u, neg, temperature, user_bias, item_bias)
    logits = torch.cat([pos_sim.unsqueeze(1), neg_sim], dim=1)
    return F.cross_entropy(logits, torch.zeros(b, dtype=torch.long))


def in_batch_negative_loss(u: torch.Tensor, i: torch.Tensor, temperature: float) -> torch.Tensor:
    """two_tower.py:453-479: CE over U·Iᵀ/τ with diagonal labels, no bias."""
    s = torch.matmul(u, i.t()) / temperature
    return F.cross_entropy(s, torch.arange(u.shape[0]))


# ---------------------------------------------------------------------------
# Trainer step (src/training/trainers/two_tower.py:98-146)
# ---------------------------------------------------------------------------

def param_names(user_state: Dict[str, torch.Tensor], item_state: Dict[str, torch.Tensor],
                use_bias: bool = True) -> List[str]:
    """Order of ``model.parameters()`` for a reference TwoTowerModel:
    user_tower params, item_tower params, user_bias, item_bias."""
    def tower(prefix, st):
        return [f"{prefix}.{k}" for k in st
                if not (k.endswith("running_mean") or k.endswith("running_var")
                        or k.endswith("num_batches_tracked"))]
    names = tower("user_tower", user_state) + tower("item_tower", item_state)
    if use_bias:
        names += ["user_bias", "item_bias"]
    return names


def adam_update(p: torch.Tensor, g: torch.Tensor, m: torch.Tensor, v: torch.Tensor, step: int,
                lr: float, wd: float, beta1: float = 0.9, beta2: float = 0.999,
                eps: float = 1e-8) -> None:
    """torch.optim.Adam single-tensor update (trainer two_tower.py:60-64: Adam(lr, wd))."""
    if wd != 0:
        g = g.add(p, alpha=wd)
    m.lerp_(g, 1 - beta1)
    v.mul_(beta2).addcmul_(g, g.conj(), value=1 - beta2)
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    step_size = lr / bc1
    denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
    p.addcdiv_(m, denom, value=-step_size)


def train_step(user_state: Dict[str, torch.Tensor], item_state: Dict[str, torch.Tensor],
               biases: Optional[Dict[str, torch.Tensor]], opt_state: Dict[str, dict],
               user_feat: torch.Tensor, pos_feat: torch.Tensor, neg_feat: Optional[torch.Tensor],
               *, temperature: float, lr: float = 1e-3, weight_decay: float = 1e-5,
               max_norm: float = 1.0, activation: str = "relu", dropout_p: float = 0.0,
               explicit_weight: float = 0.7, in_batch_weight: float = 0.3) -> Dict[str, float]:
    """One mixed-loss step (trainers/two_tower.py:98-146), in place on the states.
    ``opt_state``: name -> {"step": int, "exp_avg": T, "exp_avg_sq": T}."""
    params = {}
    for prefix, st in (("user_tower", user_state), ("item_tower", item_state)):
        for k, t in st.items():
            if k.endswith("running_mean") or k.endswith("running_var") or k.endswith("num_batches_tracked"):
                continue
            t.requires_grad_(True)
            params[f"{prefix}.{k}"] = t
    if biases is not None:
        for k, t in biases.items():
            t.requires_grad_(True)
            params[k] = t
    ub = biases["user_bias"] if biases is not None else None
    ib = biases["item_bias"] if biases is not None else None
    kw = dict(train=True, dropout_p=dropout_p, activation=activation, use_content=False)
    u = tower_forward(user_state, user_feat, **kw)
    p = tower_forward(item_state, pos_feat, **kw)
    if neg_feat is not None:
        b, r, f = neg_feat.shape
        n = tower_forward(item_state, neg_feat.reshape(-1, f), **kw)
        e = contrastive_loss(u, p, n, temperature, ub, ib)
        ibl = in_batch_negative_loss(u, p, temperature)
        loss = explicit_weight * e + in_batch_weight * ibl
    else:
        e = torch.zeros(())
        ibl = in_batch_negative_loss(u, p, temperature)
        loss = ibl
    grads = torch.autograd.grad(loss, list(params.values()), allow_unused=True)
    grads = [torch.zeros_like(t) if g is None else g for t, g in zip(params.values(), grads)]
    # clip_grad_norm_(max_norm=1.0): trainers/two_tower.py:144
    norms = torch.stack([torch.linalg.vector_norm(g, 2) for g in grads])
    total_norm = torch.linalg.vector_norm(norms, 2)
    coef = torch.clamp(max_norm / (total_norm + 1e-6), max=1.0)
    with torch.no_grad():
        for (name, t), g in zip(params.items(), grads):
            g = g * coef
            stt = opt_state.setdefault(name, {"step": 0, "exp_avg": torch.zeros_like(t),
                                              "exp_avg_sq": torch.zeros_like(t)})
            stt["step"] += 1
            adam_update(t, g, stt["exp_avg"], stt["exp_avg_sq"], stt["step"], lr, weight_decay)
            t.requires_grad_(False)
    return {"loss": float(loss.detach()), "explicit": float(e.detach()), "in_batch": float(ibl.detach()),
            "grad_norm": float(total_norm)}
