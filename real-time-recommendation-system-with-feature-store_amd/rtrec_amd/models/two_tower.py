"""Two-Tower model — the reference ``src/models/two_tower.py`` surface
(``UserTower`` :12-134, ``ItemTower`` :137-281, ``TwoTowerModel`` :284-546,
``create_two_tower_model`` :549-595) executed by MI355X kernels.

Module structure, parameter names, initialisation and ``state_dict`` layout are
identical to the reference (``mlp.{i}``, ``embeddings.*``,
``content_projection.*``, ``user_bias``/``item_bias``), so reference
checkpoints load unchanged. ``forward`` never runs the ``nn.Linear`` /
``nn.BatchNorm1d`` modules: each tower is one fused chain of gfx950 launches
(rtrec_amd.models.fused) and the losses are fused forward+backward kernels
(librtrec_hip.so). CPU tensors raise: there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import logging
from typing import Any, Dict, List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F  # noqa: F401  (reference API parity)

from .. import kernels, native
from ..native import call, ptr
from .fused import ParamSlab, blocks_from_sequential, chain_backward, chain_forward

logger = logging.getLogger("rtrec_amd.models")


# ---------------------------------------------------------------------------
# autograd bridges
# ---------------------------------------------------------------------------
def _slab_of(module: nn.Module) -> ParamSlab:
    root = getattr(module, "_slab_root", None)
    owner = root() if callable(root) else None
    owner = owner if owner is not None else module
    slab = owner.__dict__.get("_slab")
    if slab is None:
        slab = ParamSlab(owner)
        owner.__dict__["_slab"] = slab
    return slab.ensure()


class _ChainFn(torch.autograd.Function):
    """A tower MLP (or the content projection) as one autograd node. Parameter
    gradients are accumulated by the kernels straight into the slab ``.grad``
    views, so ``None`` is returned for them."""

    @staticmethod
    def forward(ctx, module, seq, normalize, x, *params):
        slab = _slab_of(module)
        blocks = blocks_from_sequential(seq)
        cctx = chain_forward(blocks, x, normalize=normalize)
        ctx.slab, ctx.blocks, ctx.cctx = slab, blocks, cctx
        ctx.x_needs_grad = x.requires_grad
        ctx.n_params = len(params)
        return cctx.out

    @staticmethod
    def backward(ctx, gout):
        dx = chain_backward(ctx.blocks, ctx.cctx, gout, ctx.slab, want_dsrc=ctx.x_needs_grad)
        return (None, None, None, dx) + (None,) * ctx.n_params


class _EmbeddingFn(torch.autograd.Function):
    """nn.Embedding(padding_idx=0) lookup: rt_gather_rows forward, rt_scatter_add_rows_f32 backward."""

    @staticmethod
    def forward(ctx, module, emb, ids, weight):
        slab = _slab_of(module)
        out = kernels.gather_rows(weight, ids, check=True)
        ctx.slab, ctx.emb, ctx.ids = slab, emb, ids
        return out

    @staticmethod
    def backward(ctx, gout):
        ctx.slab.attach_grads()
        g = ctx.slab.grad_of(ctx.emb.weight)
        kernels.scatter_add_rows(g, ctx.ids.reshape(-1), gout.reshape(-1, g.shape[1]),
                                 padding_idx=ctx.emb.padding_idx if ctx.emb.padding_idx is not None else -1)
        return None, None, None, None


def _tower_forward(tower: nn.Module, numerical: torch.Tensor,
                   categorical: Optional[Dict[str, torch.Tensor]], content: Optional[torch.Tensor]):
    """Shared UserTower/ItemTower forward (two_tower.py:112-134 / 254-281)."""
    native.require_device(numerical, what=type(tower).__name__)
    embedded = []
    if categorical:
        for name, t in categorical.items():
            if name in tower.embeddings:
                emb = tower.embeddings[name]
                embedded.append(_EmbeddingFn.apply(tower, emb, t, emb.weight))
    if content is not None and getattr(tower, "use_content_embedding", False):
        cp = tower.content_projection
        embedded.append(_ChainFn.apply(tower, cp, False, content.float(), *cp.parameters()))
    x = torch.cat([numerical, torch.cat(embedded, dim=-1)], dim=-1) if embedded else numerical
    x = x.float()
    params = list(tower.mlp.parameters())
    return _ChainFn.apply(tower, tower.mlp, True, x, *params)


def _activation(activation: str) -> nn.Module:
    """two_tower.py:77-86 (unknown names → ReLU)."""
    acts = {"relu": nn.ReLU(), "gelu": nn.GELU(), "leaky_relu": nn.LeakyReLU(0.1), "tanh": nn.Tanh(),
            "sigmoid": nn.Sigmoid()}
    return acts.get(activation, nn.ReLU())


def _init_weights(module: nn.Module):
    """two_tower.py:88-96."""
    for m in module.modules():
        if isinstance(m, nn.Linear):
            nn.init.xavier_uniform_(m.weight)
            if m.bias is not None:
                nn.init.zeros_(m.bias)
        elif isinstance(m, nn.Embedding):
            nn.init.normal_(m.weight, mean=0, std=0.01)


def _build_embeddings(categorical_features: Dict[str, int]):
    embeddings = nn.ModuleDict()
    total = 0
    for name, card in categorical_features.items():
        dim = min(50, (card + 1) // 2)
        embeddings[name] = nn.Embedding(card + 1, dim, padding_idx=0)
        total += dim
    return embeddings, total


def _build_mlp(in_dim: int, hidden_layers: List[int], embedding_dim: int, dropout_rate: float,
               activation: str) -> nn.Sequential:
    layers: List[nn.Module] = []
    prev = in_dim
    for h in hidden_layers:
        layers.extend([nn.Linear(prev, h), _activation(activation), nn.BatchNorm1d(h), nn.Dropout(dropout_rate)])
        prev = h
    layers.append(nn.Linear(prev, embedding_dim))
    return nn.Sequential(*layers)


class UserTower(nn.Module):
    """User tower (two_tower.py:12-134)."""

    def __init__(self, input_dim: int, embedding_dim: int = 128, hidden_layers: List[int] = [512, 256, 128],
                 dropout_rate: float = 0.2, activation: str = "relu",
                 categorical_features: Optional[Dict[str, int]] = None):
        super().__init__()
        self.input_dim = input_dim
        self.embedding_dim = embedding_dim
        self.categorical_features = categorical_features or {}
        self.embeddings, emb_total = _build_embeddings(self.categorical_features)
        self.mlp = _build_mlp(input_dim + emb_total, list(hidden_layers), embedding_dim, dropout_rate, activation)
        _init_weights(self)

    def _get_activation(self, activation: str) -> nn.Module:
        return _activation(activation)

    def forward(self, numerical_features: torch.Tensor,
                categorical_features: Optional[Dict[str, torch.Tensor]] = None) -> torch.Tensor:
        return _tower_forward(self, numerical_features, categorical_features, None)


class ItemTower(nn.Module):
    """Item tower (two_tower.py:137-281)."""

    def __init__(self, input_dim: int, embedding_dim: int = 128, hidden_layers: List[int] = [512, 256, 128],
                 dropout_rate: float = 0.2, activation: str = "relu",
                 categorical_features: Optional[Dict[str, int]] = None, use_content_embedding: bool = True,
                 content_embedding_dim: int = 768):
        super().__init__()
        self.input_dim = input_dim
        self.embedding_dim = embedding_dim
        self.categorical_features = categorical_features or {}
        self.use_content_embedding = use_content_embedding
        self.embeddings, emb_total = _build_embeddings(self.categorical_features)
        if use_content_embedding:
            self.content_projection = nn.Sequential(nn.Linear(content_embedding_dim, 256), nn.ReLU(),
                                                    nn.Dropout(dropout_rate), nn.Linear(256, 128))
            emb_total += 128
        self.mlp = _build_mlp(input_dim + emb_total, list(hidden_layers), embedding_dim, dropout_rate, activation)
        _init_weights(self)

    def _get_activation(self, activation: str) -> nn.Module:
        return _activation(activation)

    def forward(self, numerical_features: torch.Tensor,
                categorical_features: Optional[Dict[str, torch.Tensor]] = None,
                content_embeddings: Optional[torch.Tensor] = None) -> torch.Tensor:
        return _tower_forward(self, numerical_features, categorical_features, content_embeddings)


class _SimilarityFn(torch.autograd.Function):
    """compute_similarity (two_tower.py:380-404): forward on rt_similarity_f32."""

    @staticmethod
    def forward(ctx, u, v, inv_tau, ub, ib):
        u = u.contiguous().float()
        v = v.contiguous().float()
        out = torch.empty(u.shape[0], dtype=torch.float32, device=u.device)
        call("rt_similarity_f32", ptr(u), ptr(v), u.shape[0], u.shape[1], inv_tau, ptr(ub), ptr(ib), ptr(out),
             native.stream_of(u))
        ctx.save_for_backward(u, v)
        ctx.inv_tau = inv_tau
        ctx.has_bias = ub is not None
        return out

    @staticmethod
    def backward(ctx, g):
        u, v = ctx.saved_tensors
        gs = (g * ctx.inv_tau).unsqueeze(1)
        db = g.sum().reshape(1) if ctx.has_bias else None
        return gs * v, gs * u, None, db, db


class _LossFn(torch.autograd.Function):
    """Fused contrastive / in-batch CE: loss and its input gradients come from one
    rt_twotower_loss_fwd_bwd call; backward only rescales them."""

    @staticmethod
    def forward(ctx, u, p, q, ub, ib, inv_tau, n_neg, w_explicit, w_in_batch):
        native.require_device(u, p, what="two-tower loss")
        u = u.contiguous().float()
        p = p.contiguous().float()
        if q is not None:
            q = q.contiguous().float()
        b, d = u.shape
        dev = u.device
        loss = torch.zeros(3, dtype=torch.float64, device=dev)
        ws = kernels.workspace(dev, native.lib().rt_twotower_loss_workspace_bytes(b, d), "loss")
        st = native.stream_of(u)
        need_grad = torch.is_grad_enabled() or any(
            t is not None and t.requires_grad for t in (u, p, q, ub, ib))
        if need_grad:
            du = torch.empty_like(u)
            dp = torch.empty_like(p)
            dq = torch.empty_like(q) if q is not None else None
            dub = torch.zeros(1, dtype=torch.float32, device=dev) if ub is not None else None
            dib = torch.zeros(1, dtype=torch.float32, device=dev) if ib is not None else None
            call("rt_twotower_loss_fwd_bwd", ptr(u), ptr(p), ptr(q), 0, b, d, n_neg, inv_tau, ptr(ub), ptr(ib),
                 w_explicit, w_in_batch, ptr(loss), ptr(du), ptr(dp), ptr(dq), ptr(dub), ptr(dib), ptr(ws),
                 ws.numel(), st)
            ctx.grads = (du, dp, dq, dub, dib)
        else:
            call("rt_twotower_loss_fwd", ptr(u), ptr(p), ptr(q), 0, b, d, n_neg, inv_tau, ptr(ub), ptr(ib),
                 w_explicit, w_in_batch, ptr(loss), ptr(ws), ws.numel(), st)
            ctx.grads = None
        return loss[0].float()

    @staticmethod
    def backward(ctx, g):
        du, dp, dq, dub, dib = ctx.grads
        sc = lambda t: None if t is None else t * g  # noqa: E731
        return sc(du), sc(dp), sc(dq), sc(dub), sc(dib), None, None, None, None


class TwoTowerModel(nn.Module):
    """Two-Tower model for recommendation (two_tower.py:284-546)."""

    def __init__(self, user_tower: UserTower, item_tower: ItemTower, temperature: float = 0.05,
                 use_bias: bool = True):
        super().__init__()
        self.user_tower = user_tower
        self.item_tower = item_tower
        self.temperature = temperature
        if use_bias:
            self.user_bias = nn.Parameter(torch.zeros(1))
            self.item_bias = nn.Parameter(torch.zeros(1))
        else:
            self.register_parameter("user_bias", None)
            self.register_parameter("item_bias", None)
        import weakref
        ref = weakref.ref(self)
        for t in (user_tower, item_tower):
            t.__dict__["_slab_root"] = ref  # towers share the model's flat parameter slab

    # -- kernels' view of the model ---------------------------------------
    def slab(self) -> ParamSlab:
        return _slab_of(self)

    def forward(self, user_features: Dict[str, torch.Tensor], item_features: Dict[str, torch.Tensor],
                compute_loss: bool = False,
                negative_items: Optional[Dict[str, torch.Tensor]] = None) -> Dict[str, torch.Tensor]:
        """two_tower.py:316-378."""
        user_embedding = self.user_tower(user_features.get("numerical", torch.empty(0)),
                                         user_features.get("categorical", {}))
        item_embedding = self.item_tower(item_features.get("numerical", torch.empty(0)),
                                         item_features.get("categorical", {}),
                                         item_features.get("content_embeddings", None))
        outputs = {"user_embedding": user_embedding, "item_embedding": item_embedding}
        outputs["similarity"] = self.compute_similarity(user_embedding, item_embedding)
        if compute_loss:
            if negative_items is not None:
                neg = self.item_tower(negative_items.get("numerical", torch.empty(0)),
                                      negative_items.get("categorical", {}),
                                      negative_items.get("content_embeddings", None))
                outputs["loss"] = self.contrastive_loss(user_embedding, item_embedding, neg)
            else:
                outputs["loss"] = self.in_batch_negative_loss(user_embedding, item_embedding)
        return outputs

    def compute_similarity(self, user_embedding: torch.Tensor, item_embedding: torch.Tensor) -> torch.Tensor:
        """two_tower.py:380-404."""
        native.require_device(user_embedding, item_embedding, what="compute_similarity")
        return _SimilarityFn.apply(user_embedding, item_embedding, 1.0 / self.temperature,
                                   self.user_bias, self.item_bias)

    def contrastive_loss(self, user_embedding: torch.Tensor, pos_item_embedding: torch.Tensor,
                         neg_item_embedding: torch.Tensor) -> torch.Tensor:
        """two_tower.py:406-451 (biases on the positive logit only)."""
        b = user_embedding.shape[0]
        if neg_item_embedding.shape[0] <= b:
            # the reference falls into compute_similarity and then fails to concatenate
            # a [B] tensor with [B, 1] (two_tower.py:439-443)
            raise RuntimeError("Tensors must have same number of dimensions: got 2 and 1")
        if neg_item_embedding.shape[0] % b != 0:
            raise RuntimeError(f"shape '[{b}, {neg_item_embedding.shape[0] // b}, -1]' is invalid for input of "
                               f"size {neg_item_embedding.numel()}")
        n_neg = neg_item_embedding.shape[0] // b
        return _LossFn.apply(user_embedding, pos_item_embedding, neg_item_embedding, self.user_bias,
                             self.item_bias, 1.0 / self.temperature, n_neg, 1.0, 0.0)

    def in_batch_negative_loss(self, user_embedding: torch.Tensor, item_embedding: torch.Tensor) -> torch.Tensor:
        """two_tower.py:453-479 (no bias)."""
        return _LossFn.apply(user_embedding, item_embedding, None, None, None, 1.0 / self.temperature, 0,
                             0.0, 1.0)

    def mixed_loss(self, user_embedding, pos_item_embedding, neg_item_embedding, explicit_weight: float = 0.7,
                   in_batch_weight: float = 0.3) -> torch.Tensor:
        """The trainer's 0.7·explicit + 0.3·in-batch (trainers/two_tower.py:111-134) in one kernel pair."""
        b = user_embedding.shape[0]
        n_neg = neg_item_embedding.shape[0] // b
        return _LossFn.apply(user_embedding, pos_item_embedding, neg_item_embedding, self.user_bias,
                             self.item_bias, 1.0 / self.temperature, n_neg, explicit_weight, in_batch_weight)

    def get_user_embeddings(self, user_features: Dict[str, torch.Tensor]) -> torch.Tensor:
        return self.user_tower(user_features.get("numerical", torch.empty(0)), user_features.get("categorical", {}))

    def get_item_embeddings(self, item_features: Dict[str, torch.Tensor]) -> torch.Tensor:
        return self.item_tower(item_features.get("numerical", torch.empty(0)),
                               item_features.get("categorical", {}),
                               item_features.get("content_embeddings", None))

    def save_model(self, path: str):
        """two_tower.py:516-529 (same checkpoint keys)."""
        torch.save({"user_tower_state": self.user_tower.state_dict(),
                    "item_tower_state": self.item_tower.state_dict(),
                    "temperature": self.temperature,
                    "user_bias": self.user_bias,
                    "item_bias": self.item_bias}, path)
        logger.info("Saved model checkpoint to %s", path)

    def load_model(self, path: str):
        """two_tower.py:531-546. Loads with ``weights_only=True`` (no code from the file
        runs); bias values are copied into the existing parameters."""
        checkpoint = torch.load(path, map_location="cpu", weights_only=True)
        self.user_tower.load_state_dict(checkpoint["user_tower_state"])
        self.item_tower.load_state_dict(checkpoint["item_tower_state"])
        self.temperature = checkpoint["temperature"]
        if checkpoint.get("user_bias") is not None and self.user_bias is not None:
            with torch.no_grad():
                self.user_bias.copy_(torch.as_tensor(checkpoint["user_bias"]).reshape(1))
                self.item_bias.copy_(torch.as_tensor(checkpoint["item_bias"]).reshape(1))
        logger.info("Loaded model checkpoint from %s", path)


def create_two_tower_model(config: Dict[str, Any]) -> TwoTowerModel:
    """two_tower.py:549-595 (same keys and defaults)."""
    user_config = config.get("user_tower", {})
    item_config = config.get("item_tower", {})
    user_tower = UserTower(input_dim=user_config.get("input_dim", 50),
                           embedding_dim=config.get("embedding_dim", 128),
                           hidden_layers=user_config.get("hidden_layers", [512, 256, 128]),
                           dropout_rate=user_config.get("dropout_rate", 0.2),
                           activation=user_config.get("activation", "relu"),
                           categorical_features=user_config.get("categorical_features", {}))
    item_tower = ItemTower(input_dim=item_config.get("input_dim", 50),
                           embedding_dim=config.get("embedding_dim", 128),
                           hidden_layers=item_config.get("hidden_layers", [512, 256, 128]),
                           dropout_rate=item_config.get("dropout_rate", 0.2),
                           activation=item_config.get("activation", "relu"),
                           categorical_features=item_config.get("categorical_features", {}),
                           use_content_embedding=item_config.get("use_content_embedding", True))
    model = TwoTowerModel(user_tower=user_tower, item_tower=item_tower,
                          temperature=config.get("temperature", 0.05), use_bias=config.get("use_bias", True))
    logger.info("Created Two-Tower model")
    return model
