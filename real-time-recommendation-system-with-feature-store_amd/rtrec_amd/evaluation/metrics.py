"""Ranking metrics of the reference's offline evaluation
(src/evaluation/metrics.py:21-319) computed on the MI355X.

Same surface: ``EvaluationMetrics`` (to_dict / __str__), the per-user
functions ``recall_at_k`` … ``average_precision`` and ``Evaluator(k_values,
num_items).evaluate(predictions, ground_truth, exclude_items)`` /
``evaluate_model``. Every value comes from ``rt_rank_metrics`` (one wave per
user: exclusion filter, ranks by ballot/popcount, ground-truth membership by
binary search, the per-user sums in the reference's rank-ascending fp64 order)
and ``rt_rank_metrics_reduce`` (means over evaluated users in a fixed order,
coverage by popcount). ``evaluate_tensors`` is the device-resident form used
by ``generate_recommendations`` output (no host round trip per user).

Contract differences, stated: a prediction list may not repeat a ground-truth
item (the top-K kernels never emit duplicates; the reference would count such
a repeat once in recall but twice in NDCG), and ids must be >= 0 (-1 pads a
ragged list). Both raise ``ValueError`` in the dict path.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Sequence, Set

import numpy as np
import torch

from .. import kernels


@dataclass
class EvaluationMetrics:
    """metrics.py:21-70."""
    recall: Dict[int, float] = field(default_factory=dict)
    precision: Dict[int, float] = field(default_factory=dict)
    ndcg: Dict[int, float] = field(default_factory=dict)
    hit_rate: Dict[int, float] = field(default_factory=dict)
    mrr: float = 0.0
    map_score: float = 0.0
    coverage: float = 0.0
    per_user_recall: Dict[int, List[float]] = field(default_factory=dict)
    per_user_ndcg: Dict[int, List[float]] = field(default_factory=dict)

    def to_dict(self) -> Dict[str, float]:
        result = {}
        for k, v in self.recall.items():
            result[f"recall@{k}"] = v
        for k, v in self.precision.items():
            result[f"precision@{k}"] = v
        for k, v in self.ndcg.items():
            result[f"ndcg@{k}"] = v
        for k, v in self.hit_rate.items():
            result[f"hit_rate@{k}"] = v
        result["mrr"] = self.mrr
        result["map"] = self.map_score
        result["coverage"] = self.coverage
        return result

    def __str__(self) -> str:
        lines = ["=" * 50, "Evaluation Results", "=" * 50]
        for k in sorted(self.recall.keys()):
            lines.append(f"@{k}:")
            lines.append(f"  Recall:    {self.recall[k]:.4f}")
            lines.append(f"  Precision: {self.precision[k]:.4f}")
            lines.append(f"  NDCG:      {self.ndcg[k]:.4f}")
            lines.append(f"  Hit Rate:  {self.hit_rate[k]:.4f}")
        lines.append("-" * 50)
        lines.append(f"MRR:      {self.mrr:.4f}")
        lines.append(f"MAP:      {self.map_score:.4f}")
        lines.append(f"Coverage: {self.coverage:.4f}")
        lines.append("=" * 50)
        return "\n".join(lines)


def _device(device=None) -> torch.device:
    if device is not None:
        return torch.device(device)
    if not torch.cuda.is_available():
        raise RuntimeError("evaluation metrics: no ROCm device; this MI355X build has no CPU fallback")
    return torch.device("cuda", torch.cuda.current_device())


def csr_from_sets(rows: Sequence[Optional[Iterable[int]]], device) -> tuple:
    """(offsets int64 [n+1], items int32 sorted unique) on ``device`` from one
    item collection per row (None = empty row)."""
    offs = np.zeros(len(rows) + 1, np.int64)
    parts = []
    for i, s in enumerate(rows):
        a = np.unique(np.fromiter((int(x) for x in s), np.int64)) if s is not None else np.zeros(0, np.int64)
        if a.size and (a[0] < np.iinfo(np.int32).min or a[-1] > np.iinfo(np.int32).max):
            raise ValueError("item ids must fit in int32")
        parts.append(a)
        offs[i + 1] = offs[i] + a.size
    items = np.concatenate(parts).astype(np.int32) if parts else np.zeros(0, np.int32)
    return torch.from_numpy(offs).to(device), torch.from_numpy(items).to(device)


def _pack_predictions(lists: Sequence[Sequence[int]], device) -> torch.Tensor:
    width = max([len(x) for x in lists] + [1])
    arr = np.full((len(lists), width), -1, np.int64)
    for i, x in enumerate(lists):
        if len(x):
            a = np.asarray(x, np.int64)
            if (a < 0).any():
                raise ValueError("predicted item ids must be >= 0 (-1 pads ragged lists on the device)")
            arr[i, :len(a)] = a
    return torch.from_numpy(arr).to(device)


def _check_repeats(lists, gts):
    for x, g in zip(lists, gts):
        if g is None or len(x) == len(set(x)):
            continue
        seen, rep = set(), set()
        for it in x:
            (rep if it in seen else seen).add(it)
        if rep & set(g):
            raise ValueError("a prediction list repeats a ground-truth item (unsupported; top-K output never does)")


def evaluate_tensors(preds: torch.Tensor, gt_offsets: torch.Tensor, gt_items: torch.Tensor, k_values: Sequence[int],
                     gt_rows: Optional[torch.Tensor] = None, ex_offsets: Optional[torch.Tensor] = None,
                     ex_items: Optional[torch.Tensor] = None, ex_rows: Optional[torch.Tensor] = None,
                     num_items: Optional[int] = None) -> EvaluationMetrics:
    """Evaluator.evaluate on device-resident rankings [n, L] (-1 = no item) and
    CSR ground truth / exclusions (row indirection via *_rows)."""
    ks = sorted(int(k) for k in k_values)
    per_row, valid, summary = kernels.rank_metrics(preds, gt_offsets, gt_items, ks, gt_rows=gt_rows,
                                                   ex_offsets=ex_offsets, ex_items=ex_items, ex_rows=ex_rows,
                                                   num_items=int(num_items or 0))
    return _to_metrics(per_row, valid, summary, ks)


def _to_metrics(per_row, valid, summary, ks) -> EvaluationMetrics:
    nk = len(ks)
    s = summary.cpu().numpy()
    v = valid.cpu().numpy().astype(bool)
    pr = per_row.cpu().numpy()[v]
    m = EvaluationMetrics()
    for i, k in enumerate(ks):
        m.recall[k] = float(s[i])
        m.precision[k] = float(s[nk + i])
        m.ndcg[k] = float(s[2 * nk + i])
        m.hit_rate[k] = float(s[3 * nk + i])
        m.per_user_recall[k] = pr[:, i].tolist()
        m.per_user_ndcg[k] = pr[:, 2 * nk + i].tolist()
    m.mrr = float(s[4 * nk])
    m.map_score = float(s[4 * nk + 1])
    m.coverage = float(s[4 * nk + 3])
    return m


class Evaluator:
    """metrics.py:231-399."""

    def __init__(self, k_values: List[int] = [5, 10, 20, 50, 100], num_items: Optional[int] = None,
                 device=None):
        self.k_values = sorted(k_values)
        self.num_items = num_items
        self.device = device

    def evaluate(self, predictions: Dict[int, List[int]], ground_truth: Dict[int, Set[int]],
                 exclude_items: Optional[Dict[int, Set[int]]] = None) -> EvaluationMetrics:
        """metrics.py:248-319: per-user metrics over users present in both dicts
        (empty ground truth skipped), excluded items removed from each list first."""
        dev = _device(self.device)
        users = list(predictions.keys())
        lists = [list(predictions[u]) for u in users]
        gts = [ground_truth.get(u) if u in ground_truth else None for u in users]
        _check_repeats(lists, gts)
        preds = _pack_predictions(lists, dev)
        go, gi = csr_from_sets(gts, dev)
        eo = ei = None
        if exclude_items:
            eo, ei = csr_from_sets([exclude_items.get(u) for u in users], dev)
        return evaluate_tensors(preds, go, gi, self.k_values, ex_offsets=eo, ex_items=ei, num_items=self.num_items)

    def evaluate_model(self, model, test_users: List[int], test_ground_truth: Dict[int, Set[int]],
                       train_items: Dict[int, Set[int]], user_features: np.ndarray, item_features: np.ndarray,
                       item_ids: List[int], batch_size: int = 256, device=None) -> EvaluationMetrics:
        """metrics.py:321-399: masked top-max(k) for every test user on the device
        (generate_recommendations), mapped through ``item_ids``, then evaluate."""
        from .offline import generate_recommendations
        model.eval()
        recs = generate_recommendations(model, test_users, train_items, user_features, item_features,
                                        top_k=max(self.k_values), batch_size=batch_size, device=device)
        ids = list(item_ids)
        predictions = {u: [ids[i] for i in recs[u]] for u in test_users}
        return self.evaluate(predictions, test_ground_truth)


def _single(predicted: List[int], ground_truth: Set[int], k: int):
    """Per-row values of one user (one rt_rank_metrics row)."""
    dev = _device()
    _check_repeats([list(predicted)], [ground_truth])
    preds = _pack_predictions([list(predicted)], dev)
    go, gi = csr_from_sets([ground_truth], dev)
    per_row, _, _ = kernels.rank_metrics(preds, go, gi, [int(k)])
    return per_row[0].cpu().numpy()


def recall_at_k(predicted: List[int], ground_truth: Set[int], k: int) -> float:
    """metrics.py:73-96."""
    return float(_single(predicted, ground_truth, k)[0])


def precision_at_k(predicted: List[int], ground_truth: Set[int], k: int) -> float:
    """metrics.py:99-119 (hits / k even for an empty ground truth: 0)."""
    return float(_single(predicted, ground_truth, k)[1])


def ndcg_at_k(predicted: List[int], ground_truth: Set[int], k: int) -> float:
    """metrics.py:122-157."""
    return float(_single(predicted, ground_truth, k)[2])


def hit_rate_at_k(predicted: List[int], ground_truth: Set[int], k: int) -> float:
    """metrics.py:160-178."""
    return float(_single(predicted, ground_truth, k)[3])


def reciprocal_rank(predicted: List[int], ground_truth: Set[int]) -> float:
    """metrics.py:181-199."""
    return float(_single(predicted, ground_truth, 1)[4])


def average_precision(predicted: List[int], ground_truth: Set[int]) -> float:
    """metrics.py:202-228."""
    return float(_single(predicted, ground_truth, 1)[5])
