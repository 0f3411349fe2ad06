"""Training utilities (reference src/training/utils.py:14-113)."""
from __future__ import annotations

from typing import Any, Dict, Optional

import torch

from ..models.two_tower import ItemTower, TwoTowerModel, UserTower


def create_two_tower_model_for_training(user_feature_dim: int, item_feature_dim: int,
                                        config: Optional[Dict[str, Any]] = None) -> TwoTowerModel:
    """utils.py:14-71: defaults emb 64, hidden [128, 64], dropout 0.2, τ 0.1, content off."""
    config = config or {}
    embedding_dim = config.get("embedding_dim", 64)
    hidden_layers = config.get("hidden_layers", [128, 64])
    dropout_rate = config.get("dropout_rate", 0.2)
    activation = config.get("activation", "relu")
    temperature = config.get("temperature", 0.1)
    use_bias = config.get("use_bias", True)
    user_tower = UserTower(input_dim=user_feature_dim, embedding_dim=embedding_dim, hidden_layers=hidden_layers,
                           dropout_rate=dropout_rate, activation=activation)
    item_tower = ItemTower(input_dim=item_feature_dim, embedding_dim=embedding_dim, hidden_layers=hidden_layers,
                           dropout_rate=dropout_rate, activation=activation, use_content_embedding=False)
    return TwoTowerModel(user_tower=user_tower, item_tower=item_tower, temperature=temperature, use_bias=use_bias)


def get_device(prefer_gpu: bool = True) -> str:
    """utils.py:74-85."""
    if prefer_gpu and torch.cuda.is_available():
        return "cuda"
    return "cpu"


def count_parameters(model: torch.nn.Module) -> int:
    """utils.py:88-97."""
    return sum(p.numel() for p in model.parameters() if p.requires_grad)


def set_seed(seed: int = 42) -> None:
    """utils.py:100-113."""
    import random

    import numpy as np
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)
