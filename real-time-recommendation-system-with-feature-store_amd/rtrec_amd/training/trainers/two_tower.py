"""TwoTowerTrainer (reference src/training/trainers/two_tower.py:25-273) on the
fused MI355X step.

Same constructor, config keys, schedule and bookkeeping as the reference:
Adam(lr, weight_decay), ReduceLROnPlateau(mode=min, factor=0.5, patience=2) on
the validation loss, early stopping, ``two_tower_latest.pth`` /
``two_tower_best.pth`` checkpoints with the reference's keys. The inner step —
three tower calls, 0.7·contrastive + 0.3·in-batch, backward,
clip_grad_norm_(1.0), Adam — is ``FusedTrainStep`` (one fixed launch sequence,
no autograd). Batches are either the reference's feature dicts
(``user_features``, ``pos_item_features``, ``neg_item_features``) or the id
batches of ``DeviceFeeder`` (``user_ids``/``pos_ids``/``neg_ids`` + tables).
Per-batch losses are accumulated on the device; the host reads one number
per epoch.
"""
from __future__ import annotations

import time
from pathlib import Path
from typing import Any, Dict, Iterable, List

import torch

from ... import kernels
from ...models.two_tower import TwoTowerModel
from ..fused_step import FusedTrainStep


class _ReduceLROnPlateau:
    """torch.optim.lr_scheduler.ReduceLROnPlateau(mode='min', factor, patience)
    with torch's defaults (threshold 1e-4 relative, cooldown 0, min_lr 0, eps 1e-8)."""

    def __init__(self, step: FusedTrainStep, factor: float = 0.5, patience: int = 2, threshold: float = 1e-4,
                 eps: float = 1e-8):
        self.step, self.factor, self.patience, self.threshold, self.eps = step, factor, patience, threshold, eps
        self.best = float("inf")
        self.num_bad = 0

    def state_dict(self):
        return {"best": self.best, "num_bad_epochs": self.num_bad}

    def __call__(self, metric: float):
        if metric < self.best * (1.0 - self.threshold):
            self.best = metric
            self.num_bad = 0
        else:
            self.num_bad += 1
        if self.num_bad > self.patience:
            new_lr = self.step.lr * self.factor
            if self.step.lr - new_lr > self.eps:
                self.step.set_lr(new_lr)
            self.num_bad = 0


class TwoTowerTrainer:
    def __init__(self, model: TwoTowerModel, train_loader: Iterable, val_loader: Iterable,
                 config: Dict[str, Any], device: str = "cuda"):
        self.model = model.to(device)
        self.train_loader = train_loader
        self.val_loader = val_loader
        self.config = config
        self.device = torch.device(device)
        self.step = FusedTrainStep(model, lr=config.get("learning_rate", 0.001),
                                   weight_decay=config.get("weight_decay", 1e-5),
                                   max_norm=config.get("max_grad_norm", 1.0))
        self.scheduler = _ReduceLROnPlateau(self.step, factor=0.5, patience=2)
        self.early_stopping_patience = config.get("early_stopping_patience", 5)
        self.best_val_loss = float("inf")
        self.patience_counter = 0
        self.checkpoint_dir = Path(config.get("checkpoint_dir", "models/checkpoints"))
        self.checkpoint_dir.mkdir(parents=True, exist_ok=True)
        self.train_losses: List[float] = []
        self.val_losses: List[float] = []

    # ------------------------------------------------------------------
    def _feeder_graph(self):
        """(FeederGraph, batch limit) when the train loader is a ``DeviceFeeder``
        (or an epoch-limited view of one: ``.feeder`` / ``.n``), the step is
        single-process and ``config["graph_steps"]`` is not False; else None
        (the eager loop over the loader's batches)."""
        if not self.config.get("graph_steps", True) or self.step.pg is not None:
            return None
        from ..datasets.movielens import DeviceFeeder
        from ..fused_step import FeederGraph
        loader, limit = self.train_loader, 0
        if not isinstance(loader, DeviceFeeder) and isinstance(getattr(loader, "feeder", None), DeviceFeeder):
            loader, limit = loader.feeder, int(getattr(loader, "n", 0) or 0)
        if not isinstance(loader, DeviceFeeder) or loader.num_negatives <= 0 or loader.batch_size % 32:
            return None
        if getattr(self, "_fg", None) is None or self._fg.feeder is not loader:
            self._fg = FeederGraph(self.step, loader)
        return self._fg, limit

    def _run_step(self, batch: Dict[str, torch.Tensor]) -> torch.Tensor:
        dev = self.device
        if "user_ids" in batch:
            return self.step(batch["user_table"], batch["item_table"],
                             batch["item_table"] if "neg_ids" in batch else None,
                             user_ids=batch["user_ids"], pos_ids=batch["pos_ids"], neg_ids=batch.get("neg_ids"))
        neg = batch.get("neg_item_features")
        return self.step(batch["user_features"].to(dev), batch["pos_item_features"].to(dev),
                         neg.to(dev) if neg is not None else None)

    def train_epoch(self, epoch: int) -> float:
        """two_tower.py:84-156 (mixed loss when negatives are present, else in-batch only).
        Per-batch losses (the reference's tqdm postfix) stay on the device, one
        fp64 slot per batch; the host reads them once at the end of the epoch
        (``last_epoch_step_losses``)."""
        self.model.train()
        fg = self._feeder_graph()
        if fg is not None:  # one hipGraph replay per batch (FeederGraph)
            feeder, limit = fg
            losses = feeder.run_epoch(limit)
            self.last_epoch_step_losses = losses.cpu().numpy()
            n = len(self.last_epoch_step_losses)
            avg = float(self.last_epoch_step_losses.sum()) / n if n else 0.0
            self.train_losses.append(avg)
            return avg
        try:
            cap = len(self.train_loader)
        except TypeError:
            cap = 1024
        buf = torch.zeros(max(1, cap), dtype=torch.float64, device=self.device)
        n = 0
        for batch in self.train_loader:
            if n == buf.numel():
                buf = torch.cat([buf, torch.zeros_like(buf)])
            buf[n:n + 1].copy_(self._run_step(batch)[0:1])
            n += 1
        self.last_epoch_step_losses = buf[:n].cpu().numpy()
        avg = float(self.last_epoch_step_losses.sum()) / n if n else 0.0
        self.train_losses.append(avg)
        return avg

    @torch.no_grad()
    def validate(self) -> float:
        """two_tower.py:158-188: in-batch loss on positives, eval mode."""
        self.model.eval()
        total = torch.zeros((), dtype=torch.float64, device=self.device)
        n = 0
        for batch in self.val_loader:
            if "user_ids" in batch:
                uf = kernels.gather_rows(batch["user_table"], batch["user_ids"])
                pf = kernels.gather_rows(batch["item_table"], batch["pos_ids"])
            else:
                uf = batch["user_features"].to(self.device)
                pf = batch["pos_item_features"].to(self.device)
            u = self.model.get_user_embeddings({"numerical": uf, "categorical": {}})
            p = self.model.get_item_embeddings({"numerical": pf, "categorical": {}})
            total += self.model.in_batch_negative_loss(u, p).double()
            n += 1
        avg = float(total.item()) / n if n else 0.0
        self.val_losses.append(avg)
        return avg

    def save_checkpoint(self, epoch: int, is_best: bool = False) -> None:
        """two_tower.py:190-215 (same keys; optimizer_state in torch.optim.Adam format)."""
        ckpt = {
            "epoch": epoch,
            "user_tower_state": self.model.user_tower.state_dict(),
            "item_tower_state": self.model.item_tower.state_dict(),
            "temperature": self.model.temperature,
            "user_bias": self.model.user_bias,
            "item_bias": self.model.item_bias,
            "optimizer_state": self.step.optimizer_state_dict(),
            "train_losses": self.train_losses,
            "val_losses": self.val_losses,
        }
        torch.save(ckpt, self.checkpoint_dir / "two_tower_latest.pth")
        if is_best:
            torch.save(ckpt, self.checkpoint_dir / "two_tower_best.pth")

    def load_checkpoint(self, path) -> int:
        """Resume from a checkpoint written by ``save_checkpoint`` here or by the
        reference's (src/training/trainers/two_tower.py:190-215; same keys,
        torch.optim.Adam state layout): tower states, biases, Adam moments and
        step, learning rate, loss history. Loaded with ``weights_only=True``.
        Returns the checkpoint's epoch. (The reference has no resume path; this
        is the inverse of its save_checkpoint.)"""
        ck = torch.load(path, map_location="cpu", weights_only=True)
        m = self.model
        m.user_tower.load_state_dict(ck["user_tower_state"])
        m.item_tower.load_state_dict(ck["item_tower_state"])
        m.temperature = ck.get("temperature", m.temperature)
        with torch.no_grad():
            for name in ("user_bias", "item_bias"):
                v = ck.get(name)
                p = getattr(m, name)
                if v is not None and p is not None:
                    p.copy_(torch.as_tensor(v).reshape(p.shape))
        if ck.get("optimizer_state") is not None:
            self.step.load_optimizer_state_dict(ck["optimizer_state"])
        self.train_losses = list(ck.get("train_losses", []))
        self.val_losses = list(ck.get("val_losses", []))
        if self.val_losses:
            self.best_val_loss = min(self.val_losses)
        return int(ck.get("epoch", 0))

    def train(self, num_epochs: int) -> None:
        """two_tower.py:217-262."""
        for epoch in range(1, num_epochs + 1):
            start = time.time()
            train_loss = self.train_epoch(epoch)
            val_loss = self.validate()
            self.scheduler(val_loss)
            self.epoch_log = {"epoch": epoch, "train_loss": train_loss, "val_loss": val_loss,
                              "seconds": time.time() - start}
            is_best = val_loss < self.best_val_loss
            if is_best:
                self.best_val_loss = val_loss
                self.patience_counter = 0
            else:
                self.patience_counter += 1
            self.save_checkpoint(epoch, is_best)
            if self.patience_counter >= self.early_stopping_patience:
                break

    def get_training_history(self) -> Dict[str, List[float]]:
        return {"train_losses": self.train_losses, "val_losses": self.val_losses}
