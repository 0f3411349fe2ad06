"""MovieLens training data (reference src/training/datasets/movielens.py:22-162)
plus the device-resident feeder of SURVEY §8(f) rank 2.

* ``MovieLensDataset`` / ``collate_fn`` keep the reference's per-sample
  interface (same constructor, same item dict keys, same collation) for code
  that drives a ``DataLoader``; it is host-side plumbing.
* ``DeviceFeeder`` is the MI355X path: the user/movie feature tables, the
  interaction list and a CSR of every user's interacted items live in HBM;
  per batch the shuffle is a device permutation, negatives come from
  ``rt_sample_negatives`` (uniform without replacement over the user's
  non-interacted items — the reference's ``sample_negative_items`` semantics)
  and the rows are never materialised: batches are id vectors that the first
  tower Linear gathers inside its A-tile staging (``rt_linear_fwd_f32.ids``).
  The reference spends ≈345 ms per 1024-sample batch here.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Iterator, Optional

import numpy as np
import pandas as pd
import torch
from torch.utils.data import Dataset

from ... import kernels
from ...data.movielens import (create_movie_features, create_user_features, get_user_positive_items,
                               sample_negative_items)


class MovieLensDataset(Dataset):
    """movielens.py:22-134: one (user, positive[, negatives]) sample per interaction."""

    def __init__(self, interactions: pd.DataFrame, users: pd.DataFrame, movies: pd.DataFrame,
                 num_negatives: int = 4, is_training: bool = True, seed: Optional[int] = None):
        self.interactions = interactions.reset_index(drop=True)
        self.users = users
        self.movies = movies
        self.num_negatives = num_negatives
        self.is_training = is_training
        self.user_positive_items = get_user_positive_items(interactions)
        self.num_items = int(movies["movie_idx"].max()) + 1
        self.user_features = create_user_features(users, np.arange(users["user_idx"].max() + 1), normalize=True)
        self.movie_features = create_movie_features(movies, np.arange(movies["movie_idx"].max() + 1),
                                                    normalize=True)
        self._u = self.interactions["user_idx"].to_numpy(np.int64)
        self._m = self.interactions["movie_idx"].to_numpy(np.int64)
        self._y = self.interactions["label"].to_numpy(np.float32) if "label" in self.interactions else \
            np.ones(len(self.interactions), np.float32)
        self._rng = np.random.default_rng(seed)

    def __len__(self) -> int:
        return len(self.interactions)

    def __getitem__(self, idx: int) -> Dict[str, torch.Tensor]:
        user_idx, pos_item_idx, label = int(self._u[idx]), int(self._m[idx]), float(self._y[idx])
        item = {
            "user_idx": user_idx,
            "user_features": torch.tensor(self.user_features[user_idx], dtype=torch.float32),
            "pos_item_idx": pos_item_idx,
            "pos_item_features": torch.tensor(self.movie_features[pos_item_idx], dtype=torch.float32),
        }
        if self.is_training and self.num_negatives > 0:
            neg = sample_negative_items(user_idx, self.user_positive_items, self.num_items, self.num_negatives,
                                        rng=self._rng)
            item["neg_item_indices"] = torch.tensor(neg, dtype=torch.long)
            item["neg_item_features"] = torch.tensor(self.movie_features[neg], dtype=torch.float32)
        item["label"] = torch.tensor(label, dtype=torch.float32)
        return item


def collate_fn(batch: list) -> Dict[str, torch.Tensor]:
    """movielens.py:137-162: stack feature / index tensors, tensorise scalars."""
    out = {}
    for key in batch[0].keys():
        if "features" in key or "indices" in key:
            out[key] = torch.stack([b[key] for b in batch])
        else:
            out[key] = torch.tensor([b[key] for b in batch])
    return out


# ---------------------------------------------------------------------------
@dataclass
class PositiveCSR:
    """Every user's interacted items (any label — get_user_positive_items,
    src/data/movielens.py:469-485) as CSR: offsets int64 [n_users+1], items
    int32 sorted and unique inside each user's segment."""
    offsets: np.ndarray
    items: np.ndarray

    @staticmethod
    def from_pairs(users: np.ndarray, items: np.ndarray, n_users: int) -> "PositiveCSR":
        users = np.asarray(users, np.int64)
        items = np.asarray(items, np.int64)
        key = np.unique(users * (int(items.max(initial=0)) + 1) + items)
        span = int(items.max(initial=0)) + 1
        u, it = key // span, key % span
        counts = np.bincount(u, minlength=n_users)[:n_users]
        offsets = np.zeros(n_users + 1, np.int64)
        np.cumsum(counts, out=offsets[1:])
        return PositiveCSR(offsets, it.astype(np.int32))

    @staticmethod
    def from_interactions(interactions: pd.DataFrame, n_users: int) -> "PositiveCSR":
        return PositiveCSR.from_pairs(interactions["user_idx"].to_numpy(), interactions["movie_idx"].to_numpy(),
                                      n_users)

    def to(self, device) -> "DeviceCSR":
        return DeviceCSR(torch.from_numpy(self.offsets).to(device), torch.from_numpy(self.items).to(device))


@dataclass
class DeviceCSR:
    offsets: torch.Tensor
    items: torch.Tensor


class DeviceFeeder:
    """HBM-resident batch source for ``FusedTrainStep``: yields dicts with
    ``user_ids`` [B], ``pos_ids`` [B], ``neg_ids`` [B·N] (device int64) and the
    feature tables ``user_table`` / ``item_table`` (device fp32)."""

    def __init__(self, interactions: pd.DataFrame, users: pd.DataFrame, movies: pd.DataFrame,
                 num_negatives: int = 16, batch_size: int = 1024, device: Optional[torch.device] = None,
                 seed: int = 0, shuffle: bool = True, drop_last: bool = True,
                 positives: Optional[pd.DataFrame] = None):
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        n_users = int(users["user_idx"].max()) + 1
        self.num_items = int(movies["movie_idx"].max()) + 1
        self.user_table = torch.from_numpy(
            create_user_features(users, np.arange(n_users), normalize=True)).to(self.device)
        self.item_table = torch.from_numpy(
            create_movie_features(movies, np.arange(self.num_items), normalize=True)).to(self.device)
        self.inter_u = torch.from_numpy(interactions["user_idx"].to_numpy(np.int64)).to(self.device)
        self.inter_m = torch.from_numpy(interactions["movie_idx"].to_numpy(np.int64)).to(self.device)
        pos_src = positives if positives is not None else interactions
        self.csr = PositiveCSR.from_interactions(pos_src, n_users).to(self.device)
        self.num_negatives = num_negatives
        self.batch_size = batch_size
        self.seed = seed
        self.shuffle = shuffle
        self.drop_last = drop_last
        self.epoch = 0

    def __len__(self) -> int:
        n = self.inter_u.numel()
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)

    def batch(self, idx: torch.Tensor, salt: int) -> Dict[str, torch.Tensor]:
        users = self.inter_u[idx]
        pos = self.inter_m[idx]
        out = {"user_ids": users, "pos_ids": pos, "user_table": self.user_table, "item_table": self.item_table}
        if self.num_negatives > 0:
            neg = kernels.sample_negatives(self.csr.offsets, self.csr.items, users, self.num_items,
                                           self.num_negatives, seed=(self.seed * 1_000_003 + salt))
            out["neg_ids"] = neg.reshape(-1)
        return out

    def __iter__(self) -> Iterator[Dict[str, torch.Tensor]]:
        n = self.inter_u.numel()
        g = torch.Generator(device=self.device)
        g.manual_seed(self.seed + 7919 * self.epoch)
        order = torch.randperm(n, device=self.device, generator=g) if self.shuffle else \
            torch.arange(n, device=self.device)
        for b in range(len(self)):
            idx = order[b * self.batch_size:(b + 1) * self.batch_size]
            yield self.batch(idx, salt=self.epoch * 1_000_000 + b)
        self.epoch += 1
