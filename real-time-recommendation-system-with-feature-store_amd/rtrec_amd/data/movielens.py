"""MovieLens-1M data (reference src/data/movielens.py) — host-side feeder.

* ``MovieLensLoader`` reads ``ratings.dat``/``users.dat``/``movies.dat`` with the
  reference's preprocessing (k-core filter, implicit labels, LabelEncoder ids,
  time split; movielens.py:44-382) — only when the real files are present.
* ``create_user_features`` / ``create_movie_features`` (:385-466) vectorised:
  the same feature values as the reference's per-row loops.
* ``synthetic_movielens`` — a seeded ML-1M-SHAPED stream (6,040 users,
  3,416 movies after filtering, ~1M ratings, >= 20 ratings per user) for the
  benchmark and tests, since ``ml-1m/ratings.dat`` is absent
  (/root/reference/.MISSING_LARGE_BLOBS) and the data may not be redistributed.
* ``get_user_positive_items`` / ``sample_negative_items`` (:469-512) and a
  vectorised batch sampler used to pre-build device-resident training batches.
"""
from __future__ import annotations

from dataclasses import dataclass
from pathlib import Path
from typing import Dict, List, Optional, Tuple

import numpy as np
import pandas as pd

GENRES = ["Action", "Adventure", "Animation", "Children's", "Comedy", "Crime", "Documentary", "Drama", "Fantasy",
          "Film-Noir", "Horror", "Musical", "Mystery", "Romance", "Sci-Fi", "Thriller", "War", "Western"]
AGES = [1, 18, 25, 35, 45, 50, 56]


@dataclass
class MovieLensData:
    train_interactions: pd.DataFrame
    val_interactions: pd.DataFrame
    test_interactions: pd.DataFrame
    users: pd.DataFrame
    movies: pd.DataFrame
    num_users: int
    num_movies: int
    num_interactions: int
    user_feature_dim: int
    movie_feature_dim: int


def _genre_col(g: str) -> str:
    return "genre_" + g.lower().replace("-", "_").replace("'", "")


class MovieLensLoader:
    """Reference movielens.py:44-382 for the real ``.dat`` files."""

    def __init__(self, data_path: str = "ml-1m"):
        self.data_path = Path(data_path)
        for f in ["ratings.dat", "users.dat", "movies.dat"]:
            if not (self.data_path / f).exists():
                raise FileNotFoundError(f"Required file {f} not found in {self.data_path}")

    def _read(self, name, cols):
        return pd.read_csv(self.data_path / name, sep="::", names=cols, engine="python", encoding="latin-1")

    def load_ratings(self) -> pd.DataFrame:
        r = self._read("ratings.dat", ["user_id", "movie_id", "rating", "timestamp"])
        r["datetime"] = pd.to_datetime(r["timestamp"], unit="s")
        return r

    def load_users(self) -> pd.DataFrame:
        u = self._read("users.dat", ["user_id", "gender", "age", "occupation", "zip_code"])
        u["gender_encoded"] = (u["gender"] == "M").astype(int)
        return u

    def load_movies(self) -> pd.DataFrame:
        m = self._read("movies.dat", ["movie_id", "title", "genres"])
        m["year"] = pd.to_numeric(m["title"].str.extract(r"\((\d{4})\)$")[0], errors="coerce").fillna(1990).astype(int)
        for g in GENRES:
            m[_genre_col(g)] = m["genres"].str.contains(g, case=False, regex=False).astype(int)
        m["num_genres"] = m["genres"].str.count(r"\|") + 1
        return m

    def load_and_preprocess(self, split_method: str = "time", val_ratio: float = 0.1, test_ratio: float = 0.1,
                            implicit_threshold: float = 4.0, min_user_interactions: int = 5,
                            min_item_interactions: int = 5) -> MovieLensData:
        ratings = self.load_ratings()
        return preprocess(ratings, self.load_users(), self.load_movies(), split_method, val_ratio, test_ratio,
                          implicit_threshold, min_user_interactions, min_item_interactions)


def preprocess(ratings, users, movies, split_method="time", val_ratio=0.1, test_ratio=0.1, implicit_threshold=4.0,
               min_user=5, min_item=5) -> MovieLensData:
    """movielens.py:263-343: k-core (3 rounds), implicit labels, dense ids, split."""
    for _ in range(3):
        uc = ratings["user_id"].value_counts()
        ratings = ratings[ratings["user_id"].isin(uc[uc >= min_user].index)]
        ic = ratings["movie_id"].value_counts()
        ratings = ratings[ratings["movie_id"].isin(ic[ic >= min_item].index)]
    ratings = ratings.copy()
    ratings["label"] = (ratings["rating"] >= implicit_threshold).astype(int)
    uids = np.sort(ratings["user_id"].unique())
    mids = np.sort(ratings["movie_id"].unique())
    ratings["user_idx"] = np.searchsorted(uids, ratings["user_id"].to_numpy())
    ratings["movie_idx"] = np.searchsorted(mids, ratings["movie_id"].to_numpy())
    if split_method == "time":
        rs = ratings.sort_values("timestamp", kind="stable")
        n = len(rs)
        a, b = int(n * (1 - val_ratio - test_ratio)), int(n * (1 - test_ratio))
        train, val, test = rs.iloc[:a].copy(), rs.iloc[a:b].copy(), rs.iloc[b:].copy()
    elif split_method == "leave_one_out":
        rs = ratings.sort_values(["user_id", "timestamp"], kind="stable")
        test = rs.groupby("user_id").tail(1)
        rem = rs[~rs.index.isin(test.index)]
        val = rem.groupby("user_id").tail(1)
        train = rem[~rem.index.isin(val.index)]
    else:
        raise ValueError(f"Unknown split method: {split_method}")
    users = users[users["user_id"].isin(uids)].copy()
    movies = movies[movies["movie_id"].isin(mids)].copy()
    users["user_idx"] = np.searchsorted(uids, users["user_id"].to_numpy())
    movies["movie_idx"] = np.searchsorted(mids, movies["movie_id"].to_numpy())
    return MovieLensData(train, val, test, users, movies, len(uids), len(mids), len(ratings), 3, len(GENRES) + 2)


def create_user_features(users: pd.DataFrame, user_idx: np.ndarray, normalize: bool = True) -> np.ndarray:
    """movielens.py:385-424: [gender, age/56, occupation/20], default 0.5, z-scored (std+1e-8)."""
    feats = np.full((len(user_idx), 3), 0.5, dtype=np.float32)
    u = users.set_index("user_idx")
    idx = np.asarray(user_idx)
    present = np.isin(idx, u.index.to_numpy())
    rows = u.loc[idx[present]]
    feats[present, 0] = rows["gender_encoded"].to_numpy(np.float32)
    feats[present, 1] = (rows["age"].to_numpy(np.float64) / 56.0).astype(np.float32)
    feats[present, 2] = (rows["occupation"].to_numpy(np.float64) / 20.0).astype(np.float32)
    if normalize:
        feats = (feats - feats.mean(axis=0)) / (feats.std(axis=0) + 1e-8)
    return feats.astype(np.float32)


def create_movie_features(movies: pd.DataFrame, movie_idx: np.ndarray, normalize: bool = True) -> np.ndarray:
    """movielens.py:427-466: 18 genre bits, (year-1920)/80, num_genres/5; NOT
    normalised despite the flag (reference quirk, :464-466)."""
    genre_cols = [c for c in movies.columns if c.startswith("genre_")]
    feats = np.zeros((len(movie_idx), len(genre_cols) + 2), dtype=np.float32)
    m = movies.set_index("movie_idx")
    idx = np.asarray(movie_idx)
    present = np.isin(idx, m.index.to_numpy())
    rows = m.loc[idx[present]]
    feats[present, :len(genre_cols)] = rows[genre_cols].to_numpy(np.float32)
    feats[present, len(genre_cols)] = ((rows["year"].to_numpy(np.float64) - 1920) / 80.0).astype(np.float32)
    feats[present, len(genre_cols) + 1] = (rows["num_genres"].to_numpy(np.float64) / 5.0).astype(np.float32)
    return feats


def get_user_positive_items(interactions: pd.DataFrame) -> Dict[int, List[int]]:
    """movielens.py:469-485 (ALL interacted items, any label)."""
    return {int(u): g["movie_idx"].tolist() for u, g in interactions.groupby("user_idx")}


def sample_negative_items(user_idx: int, positive_items: Dict[int, List[int]], num_items: int,
                          num_negatives: int = 1, rng: Optional[np.random.Generator] = None) -> List[int]:
    """movielens.py:488-512: uniform without replacement from items the user has not interacted with."""
    rng = rng or np.random.default_rng()
    pool = np.setdiff1d(np.arange(num_items), np.asarray(positive_items.get(user_idx, []), dtype=np.int64))
    if len(pool) < num_negatives:
        return pool.tolist()
    return rng.choice(pool, num_negatives, replace=False).tolist()


# ---------------------------------------------------------------------------
# synthetic ML-1M-shaped data (the real ratings.dat is not available)
# ---------------------------------------------------------------------------
def synthetic_movielens(n_users: int = 6040, n_movies: int = 3416, n_ratings: int = 1_000_209,
                        seed: int = 0) -> MovieLensData:
    """Seeded stand-in with ML-1M's published shape (ml-1m/README:4-5,88;
    results/EVALUATION_REPORT.md:41-44): every user has >= 20 ratings, user
    activity and item popularity are Zipf-like, ratings 1-5 (label = >= 4)."""
    rng = np.random.default_rng(seed)
    users = pd.DataFrame({"user_id": np.arange(1, n_users + 1),
                          "gender": rng.choice(["F", "M"], n_users, p=[0.28, 0.72]),
                          "age": rng.choice(AGES, n_users),
                          "occupation": rng.integers(0, 21, n_users)})
    users["gender_encoded"] = (users["gender"] == "M").astype(int)
    users["user_idx"] = np.arange(n_users)
    movies = pd.DataFrame({"movie_id": np.arange(1, n_movies + 1), "year": rng.integers(1919, 2001, n_movies)})
    gbits = rng.random((n_movies, len(GENRES))) < 0.1
    gbits[np.arange(n_movies), rng.integers(0, len(GENRES), n_movies)] = True
    for j, g in enumerate(GENRES):
        movies[_genre_col(g)] = gbits[:, j].astype(int)
    movies["num_genres"] = gbits.sum(1)
    movies["movie_idx"] = np.arange(n_movies)
    # per-user counts: 20 + Zipf-like tail, rescaled to ~n_ratings
    extra = rng.zipf(1.6, n_users).astype(np.float64)
    extra = np.minimum(extra, 2000)
    extra = extra / extra.sum() * max(0, n_ratings - 20 * n_users)
    counts = np.minimum(20 + np.floor(extra).astype(np.int64), n_movies)
    pop = 1.0 / np.arange(1, n_movies + 1) ** 0.8
    pop = pop / pop.sum()
    perm = rng.permutation(n_movies)
    u_col, m_col = [], []
    for u, c in enumerate(counts):
        items = rng.choice(n_movies, int(c), replace=False, p=pop)
        u_col.append(np.full(len(items), u, np.int64))
        m_col.append(perm[items])
    uu = np.concatenate(u_col)
    mm = np.concatenate(m_col)
    ratings = pd.DataFrame({"user_id": uu + 1, "movie_id": mm + 1,
                            "rating": rng.choice([1, 2, 3, 4, 5], len(uu), p=[0.06, 0.11, 0.26, 0.35, 0.22]),
                            "timestamp": 956703932 + rng.integers(0, 90_000_000, len(uu))})
    return preprocess(ratings, users, movies, "time", min_user=5, min_item=1)


def feature_tables(data: MovieLensData) -> Tuple[np.ndarray, np.ndarray]:
    """Precomputed [num_users, 3] and [num_movies, 20] tables
    (training/datasets/movielens.py:61-84)."""
    uf = create_user_features(data.users, np.arange(data.users["user_idx"].max() + 1), normalize=True)
    mf = create_movie_features(data.movies, np.arange(data.movies["movie_idx"].max() + 1), normalize=True)
    return uf, mf


def build_batches(interactions: pd.DataFrame, num_items: int, batch_size: int, num_negatives: int, n_batches: int,
                  seed: int = 0) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Shuffled (user, positive) rows plus ``num_negatives`` uniform negatives per
    row that avoid the user's interacted items (rejection sampling: the same
    distribution as sample_negative_items, vectorised). Returns int64 arrays
    [n_batches, B], [n_batches, B], [n_batches, B*N]."""
    rng = np.random.default_rng(seed)
    users = interactions["user_idx"].to_numpy(np.int64)
    items = interactions["movie_idx"].to_numpy(np.int64)
    pos_keys = np.unique(users * num_items + items)
    total = n_batches * batch_size
    sel = rng.integers(0, len(users), total) if total > len(users) else rng.permutation(len(users))[:total]
    bu, bp = users[sel], items[sel]
    neg = rng.integers(0, num_items, (total, num_negatives))
    for _ in range(256):
        bad = np.isin(bu[:, None] * num_items + neg, pos_keys)
        for j in range(1, num_negatives):  # without replacement inside a row
            bad[:, j] |= (neg[:, :j] == neg[:, j:j + 1]).any(1)
        if not bad.any():
            break
        neg[bad] = rng.integers(0, num_items, int(bad.sum()))
    return (bu.reshape(n_batches, batch_size), bp.reshape(n_batches, batch_size),
            neg.reshape(n_batches, batch_size * num_negatives))
