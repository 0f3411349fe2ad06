"""Offline evaluation on the MI355X (reference src/evaluation/metrics.py and
scripts/evaluate_model.py)."""
from .metrics import (EvaluationMetrics, Evaluator, average_precision, evaluate_tensors, hit_rate_at_k,  # noqa: F401
                      ndcg_at_k, precision_at_k, recall_at_k, reciprocal_rank)
from .offline import generate_recommendations, load_model, recommend_tensors  # noqa: F401
