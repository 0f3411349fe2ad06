"""Known-answer cases of the reference's metric tests
(/root/reference/tests/test_evaluation_metrics.py:31-374) as data:
(function, predicted, ground truth, k, expected). Used by the oracle test (CPU)
and the GPU test of rtrec_amd.evaluation."""
CASES = [
    ("recall_at_k", [1, 2, 3, 4, 5], {1, 2, 3}, 5, 1.0),
    ("recall_at_k", [1, 2, 6, 7, 8], {1, 2, 3, 4}, 5, 0.5),
    ("recall_at_k", [5, 6, 7, 8, 9], {1, 2, 3}, 5, 0.0),
    ("recall_at_k", [1, 2, 3, 4, 5], set(), 5, 0.0),
    ("recall_at_k", [1, 2, 3, 4, 5, 6, 7, 8, 9, 10], {1, 2, 6}, 3, 2 / 3),
    ("precision_at_k", [1, 2, 3, 4, 5], {1, 2, 3, 4, 5, 6, 7}, 5, 1.0),
    ("precision_at_k", [1, 2, 6, 7, 8], {1, 2, 3, 4}, 5, 0.4),
    ("precision_at_k", [5, 6, 7, 8, 9], {1, 2, 3}, 5, 0.0),
    ("ndcg_at_k", [1, 2, 3, 4, 5], {1, 2, 3}, 5, 1.0),
    ("ndcg_at_k", [5, 6, 7, 8, 9], {1, 2, 3}, 5, 0.0),
    ("ndcg_at_k", [1, 2, 3, 4, 5], set(), 5, 0.0),
    ("ndcg_at_k", [1, 2, 3, 4, 5], {1}, 5, 1.0),
    ("hit_rate_at_k", [1, 2, 3, 4, 5], {3}, 5, 1.0),
    ("hit_rate_at_k", [1, 2, 3, 4, 5], {6, 7}, 5, 0.0),
    ("hit_rate_at_k", [1, 2, 3, 4, 5], {5}, 5, 1.0),
    ("hit_rate_at_k", [1, 2, 3, 4, 5, 6], {6}, 5, 0.0),
    ("reciprocal_rank", [1, 2, 3, 4, 5], {1}, None, 1.0),
    ("reciprocal_rank", [1, 2, 3, 4, 5], {2}, None, 0.5),
    ("reciprocal_rank", [1, 2, 3, 4, 5], {5}, None, 0.2),
    ("reciprocal_rank", [1, 2, 3, 4, 5], {6, 7}, None, 0.0),
    ("reciprocal_rank", [1, 2, 3, 4, 5], {2, 4}, None, 0.5),
    ("average_precision", [1, 2, 3, 4, 5], {1, 2, 3}, None, 1.0),
    ("average_precision", [1, 0, 2, 0, 3], {1, 2, 3}, None, (1 + 2 / 3 + 3 / 5) / 3),
    ("average_precision", [1, 2, 3, 4, 5], set(), None, 0.0),
]
# reversed-order NDCG: strictly between 0 and 1 (test_reversed_order_ndcg)
NDCG_REVERSED = ([4, 5, 6, 1, 2], {1, 2}, 5)

# Evaluator cases: (predictions, ground_truth, exclude, k_values, num_items, {key: expected})
EVALUATOR = [
    ({0: [1, 2, 3, 4, 5]}, {0: {1, 3}}, None, [5], 10, {"recall@5": 1.0}),
    ({0: [1, 2, 3, 4, 5], 1: [5, 6, 7, 8, 9]}, {0: {1, 2}, 1: {1, 2}}, None, [5], None, {"recall@5": 0.5}),
    ({0: [1, 2, 3, 4, 5]}, {0: {1, 6}}, {0: {1}}, [5], None, {"recall@5": 0.0}),
    ({0: [1, 2, 3], 1: [1, 4, 5]}, {0: {1}, 1: {4}}, None, [3], 10, {"coverage": 0.5}),
]
