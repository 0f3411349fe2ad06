"""Offline evaluation entry (reference scripts/evaluate_model.py:237-362).

Same arguments and flow as the reference CLI: prepare the evaluation data
(train items per user to exclude, positive test items as ground truth, the
user / movie feature tables), load the checkpoint (architecture inferred from
its weight shapes), masked top-max(k) recommendations for every test user,
``Evaluator.evaluate``, JSON results. Every step after loading runs on the
MI355X (``generate_recommendations`` → rt_exclusion_bitmap + rt_flatip_topk,
metrics → rt_rank_metrics). Diversity / novelty (metrics.py:402-527) are
outside the hot-path scope and not computed. Without ``ml-1m/ratings.dat``
(not shipped with the reference) the seeded ML-1M-shaped stream is used.

    python -m rtrec_amd.evaluate_model --checkpoint models/checkpoints/two_tower_best.pth
"""
from __future__ import annotations

import argparse
import json
import logging
import time
from pathlib import Path
from typing import List, Optional

import numpy as np

logger = logging.getLogger("rtrec_amd.evaluate_model")


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="Evaluate Two-Tower model (MI355X)")
    p.add_argument("--checkpoint", type=str, default="models/checkpoints/two_tower_best.pth")
    p.add_argument("--data-path", type=str, default="ml-1m")
    p.add_argument("--output", type=str, default="results/evaluation_results.json")
    p.add_argument("--device", type=str, default="auto")
    p.add_argument("--batch-size", type=int, default=256)
    p.add_argument("--k-values", type=str, default="5,10,20,50,100")
    p.add_argument("--synthetic", action="store_true", help="seeded ML-1M-shaped stream (default if ratings.dat is absent)")
    return p


def prepare_evaluation_data(data):
    """evaluate_model.py:98-159: train items per user (exclusion), positive
    (label 1) test items per user (ground truth), full feature tables."""
    from .data.movielens import create_movie_features, create_user_features, get_user_positive_items
    train_items = get_user_positive_items(data.train_interactions)
    test = data.test_interactions
    pos = test[test["label"] == 1]
    test_ground_truth = {int(u): set(g["movie_idx"].tolist()) for u, g in pos.groupby("user_idx")}
    max_user = max(data.users["user_idx"].max(), data.train_interactions["user_idx"].max())
    max_movie = max(data.movies["movie_idx"].max(), data.train_interactions["movie_idx"].max())
    uf = create_user_features(data.users, np.arange(max_user + 1), normalize=True)
    mf = create_movie_features(data.movies, np.arange(max_movie + 1), normalize=True)
    return train_items, test_ground_truth, uf, mf


def run(args) -> dict:
    from .evaluation import Evaluator, generate_recommendations, load_model
    from .train_movielens import load_data
    k_values = [int(k) for k in args.k_values.split(",")]
    data, source = load_data(argparse.Namespace(data_path=args.data_path, synthetic=args.synthetic))
    train_items, gt, uf, mf = prepare_evaluation_data(data)
    device = None if args.device == "auto" else args.device
    model = load_model(args.checkpoint, user_dim=uf.shape[1], item_dim=mf.shape[1], device=device)
    test_users = list(gt.keys())
    t0 = time.time()
    recs = generate_recommendations(model, test_users, train_items, uf, mf, top_k=max(k_values),
                                    batch_size=args.batch_size, device=device)
    t_recs = time.time() - t0
    evaluator = Evaluator(k_values=k_values, num_items=mf.shape[0])
    metrics = evaluator.evaluate(recs, gt, exclude_items=train_items)
    results = metrics.to_dict()
    results.update({"num_test_users": len(test_users), "num_items": int(mf.shape[0]), "checkpoint": args.checkpoint,
                    "data": source, "recommendation_seconds": t_recs})
    out = Path(args.output)
    out.parent.mkdir(parents=True, exist_ok=True)
    out.write_text(json.dumps(results, indent=2))
    return {"metrics": metrics, "results": results, "recommendations": recs}


def main(argv: Optional[List[str]] = None) -> int:
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    res = run(build_parser().parse_args(argv))
    print("\n" + str(res["metrics"]))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
