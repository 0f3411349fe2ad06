"""MovieLens-1M two-tower training entry (reference scripts/train_movielens.py:39-186).

Same arguments and the same pipeline as the reference CLI — load and
preprocess (time split 80/10/10, implicit threshold 4.0, 5-core filter), train
and validation sources, the training-factory model (hidden [256,128], dropout
0.2, tau 0.05), ``TwoTowerTrainer`` (Adam, wd 1e-5, early stopping 5,
``models/checkpoints``), checkpoints and data metadata — with the MI355X
pieces in place of the host ones: ``DeviceFeeder`` instead of
``DataLoader(num_workers=4)`` (tables and interactions resident in HBM,
on-device negative sampling, fused gather) and the fused train step.

``ml-1m/ratings.dat`` is not shipped with the reference
(/root/reference/.MISSING_LARGE_BLOBS), so ``--synthetic`` (the default when
the file is absent) trains on the seeded ML-1M-shaped stream of
``rtrec_amd.data.movielens.synthetic_movielens``. The data metadata is
written as JSON (the reference pickles LabelEncoders this build does not
carry), test interactions as parquet like the reference.

    python -m rtrec_amd.train_movielens --epochs 1 --batch-size 256 --embedding-dim 64     # config C1
"""
from __future__ import annotations

import argparse
import json
import logging
import time
from pathlib import Path
from typing import List, Optional

import torch

logger = logging.getLogger("rtrec_amd.train_movielens")


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="Train Two-Tower model on MovieLens-1M (MI355X)")
    # the reference's arguments (scripts/train_movielens.py:41-49)
    p.add_argument("--data-path", type=str, default="ml-1m", help="Path to MovieLens-1M")
    p.add_argument("--epochs", type=int, default=50, help="Number of epochs")
    p.add_argument("--batch-size", type=int, default=1024, help="Batch size")
    p.add_argument("--lr", type=float, default=0.001, help="Learning rate")
    p.add_argument("--embedding-dim", type=int, default=128, help="Embedding dimension")
    p.add_argument("--device", type=str, default="auto", help="Device (cuda/auto); there is no CPU path")
    p.add_argument("--num-negatives", type=int, default=16, help="Negative samples per positive")
    # this build's additions
    p.add_argument("--synthetic", action="store_true", help="seeded ML-1M-shaped stream (default if ratings.dat is absent)")
    p.add_argument("--dropout", type=float, default=0.2, help="dropout rate (reference: 0.2)")
    p.add_argument("--seed", type=int, default=0, help="shuffle / negative-sampling seed")
    p.add_argument("--init-seed", type=int, default=None, help="torch.manual_seed before building the model")
    p.add_argument("--checkpoint-dir", type=str, default="models/checkpoints")
    p.add_argument("--output-dir", type=str, default="data/processed", help="test interactions / tables")
    p.add_argument("--max-batches", type=int, default=0, help="stop each epoch after this many batches (0: all)")
    return p


class _Limited:
    """An epoch of at most ``n`` batches of ``feeder`` (``--max-batches``)."""

    def __init__(self, feeder, n: int):
        self.feeder, self.n = feeder, n

    def __len__(self):
        return min(self.n, len(self.feeder)) if self.n > 0 else len(self.feeder)

    def __iter__(self):
        for i, b in enumerate(self.feeder):
            if self.n > 0 and i >= self.n:
                break
            yield b


def load_data(args):
    from .data.movielens import MovieLensLoader, synthetic_movielens
    ratings = Path(args.data_path) / "ratings.dat"
    if args.synthetic or not ratings.exists():
        if not args.synthetic:
            logger.warning("%s not found: training on the seeded ML-1M-shaped synthetic stream", ratings)
        return synthetic_movielens(seed=0), "synthetic ML-1M-shaped (seed 0)"
    loader = MovieLensLoader(args.data_path)
    data = loader.load_and_preprocess(split_method="time", val_ratio=0.1, test_ratio=0.1, implicit_threshold=4.0,
                                      min_user_interactions=5, min_item_interactions=5)
    return data, str(Path(args.data_path).resolve())


def run(args) -> dict:
    """The reference main() body; returns a summary (losses, timings, paths)."""
    from .training.datasets.movielens import DeviceFeeder
    from .training.trainers.two_tower import TwoTowerTrainer
    from .training.utils import create_two_tower_model_for_training

    if args.device in ("auto", "cuda"):
        if not torch.cuda.is_available():
            raise RuntimeError("no ROCm device: this MI355X build has no CPU training path")
        device = torch.device("cuda", torch.cuda.current_device())
    else:
        device = torch.device(args.device)
    t0 = time.time()
    data, source = load_data(args)
    logger.info("Dataset: %d users, %d movies, %d interactions (%s)", data.num_users, data.num_movies,
                data.num_interactions, source)
    # reference: the train loader samples negatives against the TRAIN interactions
    # (MovieLensDataset.user_positive_items), drop_last False (DataLoader default)
    n_train = len(data.train_interactions)
    drop_last = n_train % args.batch_size == 1   # a 1-row BatchNorm batch raises in the reference too
    train = DeviceFeeder(data.train_interactions, data.users, data.movies, num_negatives=args.num_negatives,
                         batch_size=args.batch_size, device=device, seed=args.seed, shuffle=True,
                         drop_last=drop_last)
    val = DeviceFeeder(data.val_interactions, data.users, data.movies, num_negatives=0,
                       batch_size=args.batch_size, device=device, seed=args.seed, shuffle=False,
                       drop_last=len(data.val_interactions) % args.batch_size == 1)
    user_dim = int(train.user_table.shape[1])
    movie_dim = int(train.item_table.shape[1])
    model_config = {"embedding_dim": args.embedding_dim, "hidden_layers": [256, 128],
                    "dropout_rate": args.dropout, "temperature": 0.05}
    if args.init_seed is not None:
        torch.manual_seed(args.init_seed)
    model = create_two_tower_model_for_training(user_dim, movie_dim, model_config)
    n_params = sum(p.numel() for p in model.parameters())
    logger.info("Model parameters: %d", n_params)
    trainer_config = {"learning_rate": args.lr, "weight_decay": 1e-5, "early_stopping_patience": 5,
                      "checkpoint_dir": args.checkpoint_dir}
    trainer = TwoTowerTrainer(model=model, train_loader=_Limited(train, args.max_batches),
                              val_loader=_Limited(val, args.max_batches), config=trainer_config, device=str(device))
    t_setup = time.time() - t0
    t1 = time.time()
    trainer.train(args.epochs)
    torch.cuda.synchronize(device)
    t_train = time.time() - t1

    ckpt = Path(args.checkpoint_dir)
    meta = {"num_users": int(data.num_users), "num_movies": int(data.num_movies), "user_feature_dim": user_dim,
            "movie_feature_dim": movie_dim, "source": source, "model_config": model_config}
    (ckpt / "data_metadata.json").write_text(json.dumps(meta, indent=2))
    out = Path(args.output_dir)
    out.mkdir(parents=True, exist_ok=True)
    try:
        data.test_interactions.to_parquet(out / "test_interactions.parquet")
        data.users.to_parquet(out / "users.parquet")
        data.movies.to_parquet(out / "movies.parquet")
    except (ImportError, ValueError) as e:  # parquet engine missing
        logger.warning("parquet export skipped: %s", e)
    steps = len(getattr(trainer, "last_epoch_step_losses", []))
    return {"epochs_run": len(trainer.train_losses), "train_losses": trainer.train_losses,
            "val_losses": trainer.val_losses, "setup_s": t_setup, "train_s": t_train,
            "batches_last_epoch": steps, "params": n_params, "trainer": trainer, "model": model,
            "checkpoint": str(ckpt / "two_tower_best.pth"), "source": source}


def main(argv: Optional[List[str]] = None) -> int:
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    args = build_parser().parse_args(argv)
    res = run(args)
    logger.info("Training completed: train losses %s, val losses %s (%.1fs)", res["train_losses"],
                res["val_losses"], res["train_s"])
    logger.info("Model checkpoint: %s", res["checkpoint"])
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
