"""ORACLE — test infrastructure only (see oracle/__init__.py).

Pure-Python/numpy restatement of the reference's ranking metrics
(src/evaluation/metrics.py): the per-user functions (:73-228) and
``Evaluator.evaluate`` (:248-319). Pinned by the reference's own known-answer
tests (tests/test_evaluation_metrics.py:31-374, replayed in
tests/test_oracle_golden.py) and by tests/golden/eval_metrics.npz, written by
importing the reference's Evaluator (tools/make_goldens.py --only r2).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Set

import numpy as np


def recall_at_k(predicted: List[int], ground_truth: Set[int], k: int) -> float:
    """metrics.py:73-96."""
    if len(ground_truth) == 0:
        return 0.0
    return len(set(predicted[:k]) & ground_truth) / len(ground_truth)


def precision_at_k(predicted: List[int], ground_truth: Set[int], k: int) -> float:
    """metrics.py:99-119."""
    return len(set(predicted[:k]) & ground_truth) / k


def ndcg_at_k(predicted: List[int], ground_truth: Set[int], k: int) -> float:
    """metrics.py:122-157 (binary relevance, log2(i + 2) discount)."""
    if len(ground_truth) == 0:
        return 0.0
    dcg = 0.0
    for i, item in enumerate(predicted[:k]):
        if item in ground_truth:
            dcg += 1.0 / np.log2(i + 2)
    idcg = sum(1.0 / np.log2(i + 2) for i in range(min(len(ground_truth), k)))
    return dcg / idcg if idcg != 0 else 0.0


def hit_rate_at_k(predicted: List[int], ground_truth: Set[int], k: int) -> float:
    """metrics.py:160-178."""
    return 1.0 if len(set(predicted[:k]) & ground_truth) > 0 else 0.0


def reciprocal_rank(predicted: List[int], ground_truth: Set[int]) -> float:
    """metrics.py:181-199."""
    for i, item in enumerate(predicted):
        if item in ground_truth:
            return 1.0 / (i + 1)
    return 0.0


def average_precision(predicted: List[int], ground_truth: Set[int]) -> float:
    """metrics.py:202-228."""
    if len(ground_truth) == 0:
        return 0.0
    score, hits = 0.0, 0
    for i, item in enumerate(predicted):
        if item in ground_truth:
            hits += 1
            score += hits / (i + 1)
    return score / len(ground_truth)


def evaluate(predictions: Dict[int, List[int]], ground_truth: Dict[int, Set[int]], k_values: List[int],
             num_items: Optional[int] = None, exclude_items: Optional[Dict[int, Set[int]]] = None) -> dict:
    """Evaluator.evaluate (metrics.py:248-319) → the reference's to_dict() keys
    plus per-user recall/ndcg lists."""
    ks = sorted(k_values)
    acc = {k: {"recall": [], "precision": [], "ndcg": [], "hit_rate": []} for k in ks}
    rr, ap, seen = [], [], set()
    for u, pred in predictions.items():
        if u not in ground_truth:
            continue
        gt = ground_truth[u]
        if exclude_items and u in exclude_items:
            pred = [i for i in pred if i not in exclude_items[u]]
        if len(gt) == 0:
            continue
        seen.update(pred[:max(ks)])
        for k in ks:
            acc[k]["recall"].append(recall_at_k(pred, gt, k))
            acc[k]["precision"].append(precision_at_k(pred, gt, k))
            acc[k]["ndcg"].append(ndcg_at_k(pred, gt, k))
            acc[k]["hit_rate"].append(hit_rate_at_k(pred, gt, k))
        rr.append(reciprocal_rank(pred, gt))
        ap.append(average_precision(pred, gt))
    out = {}
    for k in ks:
        for name in ("recall", "precision", "ndcg", "hit_rate"):
            vals = acc[k][name]
            out[f"{name}@{k}"] = float(np.mean(vals)) if vals else 0.0
        out[f"per_user_recall@{k}"] = acc[k]["recall"]
        out[f"per_user_ndcg@{k}"] = acc[k]["ndcg"]
    out["mrr"] = float(np.mean(rr)) if rr else 0.0
    out["map"] = float(np.mean(ap)) if ap else 0.0
    out["coverage"] = len(seen) / num_items if num_items else 0.0
    return out
