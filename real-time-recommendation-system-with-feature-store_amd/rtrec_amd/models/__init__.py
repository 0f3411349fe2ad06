"""Two-tower models (reference src/models/__init__.py surface; the ranking
models are outside the hot path and not part of the MI355X build)."""
from .two_tower import ItemTower, TwoTowerModel, UserTower, create_two_tower_model

__all__ = ["UserTower", "ItemTower", "TwoTowerModel", "create_two_tower_model"]
