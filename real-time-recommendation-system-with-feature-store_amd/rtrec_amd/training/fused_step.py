"""One mixed-loss training step of ``TwoTowerTrainer.train_epoch``
(src/training/trainers/two_tower.py:98-146) as a fixed sequence of gfx950
launches, with no autograd and no torch compute:

  user tower fwd │ pos item tower fwd │ neg item tower fwd   (gather fused into layer 1)
  fused loss fwd+bwd (0.7·contrastive + 0.3·in-batch)          rt_twotower_loss_fwd_bwd
  neg / pos / user tower bwd  (grads → flat slab, atomics)      rt_linear_bwd_f32 × 2(L+1) each
  clip_grad_norm_(1.0) + Adam(lr, wd)                           rt_grad_sqnorm + rt_clip_adam_step

Parameters, grads and Adam moments live in flat fp32 slabs; the step counter
and learning rate live on the device so the whole step can be captured in a
hipGraph and replayed (``capture``/``replay``).
"""
from __future__ import annotations

import ctypes
import itertools
from typing import Dict, Optional

import torch

from .. import kernels, native
from ..models.fused import (blocks_from_sequential, chain_backward, chain_backward_pair, chain_forward,
                            chain_forward_pair, stats_arena_size)
from ..models.two_tower import TwoTowerModel
from ..native import call, ptr
from ..profiling import TIMER


_STEP_SEEDS = itertools.count(0x5EED)


def _adjacent_or_cat(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """[a; b] flattened: a view when b directly follows a in one storage (no
    copy launch), else torch.cat."""
    if (a.is_contiguous() and b.is_contiguous() and a.dtype == b.dtype and a.device == b.device
            and a.untyped_storage().data_ptr() == b.untyped_storage().data_ptr()
            and b.data_ptr() == a.data_ptr() + a.numel() * a.element_size()):
        return torch.as_strided(a, (a.numel() + b.numel(),), (1,))
    return torch.cat([a.reshape(-1), b.reshape(-1)])


class FusedTrainStep:
    def __init__(self, model: TwoTowerModel, lr: float = 1e-3, weight_decay: float = 1e-5, max_norm: float = 1.0,
                 betas=(0.9, 0.999), eps: float = 1e-8, explicit_weight: float = 0.7,
                 in_batch_weight: float = 0.3, process_group=None, dropout_seed: Optional[int] = None):
        self.model = model
        self.pg = process_group
        self.slab = model.slab()
        dev = self.slab.data.device
        native.require_device(self.slab.data, what="FusedTrainStep")
        self.dev = dev
        self.exp_avg = torch.zeros_like(self.slab.data)
        self.exp_avg_sq = torch.zeros_like(self.slab.data)
        self.step_dev = torch.zeros(1, dtype=torch.int32, device=dev)
        self.lr_dev = torch.tensor([lr], dtype=torch.float32, device=dev)
        self.seed_dev = torch.zeros(1, dtype=torch.int64, device=dev)   # dropout mask counter
        # fixed per-chain dropout seed bases (+ the device counter above, bumped by
        # every step's clip+Adam): an eager step and a replay of the captured
        # step at the same counter draw identical masks
        if dropout_seed is None:  # deterministic per process, distinct per step object
            dropout_seed = next(_STEP_SEEDS)
        self.dropout_seed = int(dropout_seed)
        self._sb_user, self._sb_pos, self._sb_neg = (self.dropout_seed * 4 + r for r in (1, 2, 3))
        # the loss launch's workspace belongs to this step (a captured graph keeps
        # its pointer): grow-only, earlier buffers stay alive for graphs that hold them
        self._loss_ws: Optional[torch.Tensor] = None
        self._loss_ws_retired = []
        # fp64 accumulators, cleared without memset launches: the BN column sums of
        # the 3 tower calls (fwd + bwd) and the dbias slots live in ``arena``, which
        # clip+Adam zeroes as the step's last launch (with the grads it consumes);
        # the loss triple and the per-tensor grad norms live in ``small``, which the
        # step's first forward launch zeroes (the host reads the loss after a step)
        ua = stats_arena_size(blocks_from_sequential(model.user_tower.mlp))
        ia = stats_arena_size(blocks_from_sequential(model.item_tower.mlp))
        self._arena_sizes = [ua, ia, ia, ua, ia, ia]
        self.arena = torch.zeros(sum(self._arena_sizes), dtype=torch.float64, device=dev)
        parts, off = [], 0
        for sz in self._arena_sizes:
            parts.append(self.arena[off:off + sz])
            off += sz
        (self.a_uf, self.a_pf, self.a_nf, self.a_ub, self.a_pb, self.a_nb) = parts
        self.small = torch.zeros(3 + len(self.slab.params), dtype=torch.float64, device=dev)
        self.loss_buf, self.sumsq = self.small[:3], self.small[3:]
        self.slab.grad.zero_()  # the step owns the grad slab from here on (consumed by clip+Adam)
        # the step relies on the previous clip+Adam having zeroed the grad slab
        # and the stats arena; that holds only while nothing else wrote the slab
        # (an autograd backward bumps slab.grad_gen) and the last step finished
        self._clean = True
        self._grad_gen = self.slab.grad_gen
        # the pos and neg arenas are adjacent: together they are the [2]-segment
        # arena of the merged item chain
        self.a_pqf = self.arena[ua:ua + 2 * ia]
        self.a_pqb = self.arena[2 * ua + 2 * ia:2 * ua + 4 * ia]
        self.lr, self.wd, self.max_norm = lr, weight_decay, max_norm
        self.b1, self.b2 = betas
        self.eps = eps
        self.we, self.wb = explicit_weight, in_batch_weight
        self.steps = 0
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.graph_update: Optional[torch.cuda.CUDAGraph] = None
        self.static: Dict[str, torch.Tensor] = {}
        # the user chain and the positive-item chain overlap the negative-item chain
        # (three independent towers calls; BN running stats of the item tower still
        # update pos → neg in order, as the reference's sequential calls do)
        self.concurrent = True
        self.side = [torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)]

    def set_lr(self, lr: float):
        self.lr = lr
        self.lr_dev.fill_(lr)

    def optimizer_state_dict(self) -> dict:
        """The Adam state in torch.optim.Adam.state_dict() layout (params indexed
        in model.parameters() order), so checkpoints read like the reference's
        (src/training/trainers/two_tower.py:199)."""
        step = float(self.step_dev.item())
        state = {}
        for i, (o, e) in enumerate(self.slab.bounds):
            shape = self.slab.params[i].shape
            state[i] = {"step": torch.tensor(step), "exp_avg": self.exp_avg[o:e].view(shape).clone(),
                        "exp_avg_sq": self.exp_avg_sq[o:e].view(shape).clone()}
        group = {"lr": self.lr, "betas": (self.b1, self.b2), "eps": self.eps, "weight_decay": self.wd,
                 "amsgrad": False, "maximize": False, "foreach": None, "capturable": False,
                 "differentiable": False, "fused": None, "params": list(range(len(self.slab.params)))}
        return {"state": state, "param_groups": [group]}

    def load_optimizer_state_dict(self, sd: dict):
        """Inverse of optimizer_state_dict (also accepts a reference Adam state dict)."""
        steps = set()
        for i, (o, e) in enumerate(self.slab.bounds):
            st = sd["state"].get(i, sd["state"].get(str(i)))
            if st is None:
                continue
            self.exp_avg[o:e].copy_(st["exp_avg"].reshape(-1))
            self.exp_avg_sq[o:e].copy_(st["exp_avg_sq"].reshape(-1))
            steps.add(int(float(st["step"])))
        if len(steps) > 1:
            raise ValueError("per-parameter Adam step counts differ; the fused step keeps one counter")
        if steps:
            self.step_dev.fill_(steps.pop())
        self.set_lr(float(sd["param_groups"][0]["lr"]))

    # ------------------------------------------------------------------
    def _ensure_clean(self):
        """Zero the grad slab and the fp64 stats arena when a previous step did
        not finish or an autograd backward accumulated into the slab since (the
        common path is memset-free: clip+Adam zeroes what it consumes)."""
        if not self._clean or self.slab.grad_gen != self._grad_gen:
            self.slab.grad.zero_()
            self.arena.zero_()
            self._grad_gen = self.slab.grad_gen
        self._clean = False

    def _run(self, user_src, pos_src, neg_src, user_ids=None, pos_ids=None, neg_ids=None):
        self._ensure_clean()
        self._grads(user_src, pos_src, neg_src, user_ids, pos_ids, neg_ids)
        self._allreduce()
        out = self._update()
        self._clean = True
        return out

    def _grads(self, user_src, pos_src, neg_src, user_ids=None, pos_ids=None, neg_ids=None):
        """Forward, fused loss, backward: parameter grads in the slab."""
        m = self.model
        ub = blocks_from_sequential(m.user_tower.mlp)
        ib = blocks_from_sequential(m.item_tower.mlp)
        slab = self.slab
        st = native.stream_of(slab.data)
        so = self.seed_dev  # grads / arena are zero here (previous clip+Adam); loss / norms: first launch
        main = torch.cuda.current_stream(self.dev)
        s_u, s_p = self.side if self.concurrent else (main, main)
        b = user_ids.numel() if user_ids is not None else user_src.shape[0]
        # positives and negatives go through the item tower as ONE chain of
        # B + B·N rows whose two row segments are separate BatchNorm batches
        # (the reference's two item-tower calls, src/training/trainers/two_tower.py:
        # 107-121): half the item-tower launches. Needs B % 32 == 0.
        merged = neg_src is not None and b % 32 == 0 and (
            (pos_ids is not None and neg_ids is not None and pos_src is neg_src) or
            (pos_ids is None and neg_ids is None))
        if merged:
            if pos_ids is not None:
                item_src, item_ids = pos_src, _adjacent_or_cat(pos_ids, neg_ids)
            else:
                item_src, item_ids = torch.cat([pos_src, neg_src]), None
            # user tower and merged item tower: layer l of both in ONE launch
            pq, u = chain_forward_pair((ib, item_src, item_ids, True, so, self.a_pqf, b, self._sb_pos),
                                       (ub, user_src, user_ids, True, so, self.a_uf, 0, self._sb_user),
                                       zero_buf=self.small)
            p_out, q_out = pq.out[:b], pq.out[b:]
        else:
            p = chain_forward(ib, pos_src, pos_ids, seed_offset=so, stats_arena=self.a_pf, zero_buf=self.small,
                              seed_base=self._sb_pos)
            q = chain_forward(ib, neg_src, neg_ids, seed_offset=so, stats_arena=self.a_nf,
                              seed_base=self._sb_neg) if (neg_src is not None) else None
            p_out, q_out = p.out, (q.out if q is not None else None)
        if not merged:
            s_u.wait_stream(main)
            with torch.cuda.stream(s_u):
                u = chain_forward(ub, user_src, user_ids, seed_offset=so, stats_arena=self.a_uf,
                                  seed_base=self._sb_user)
            main.wait_stream(s_u)
        d = u.out.shape[1]
        n_neg = (q_out.shape[0] // b) if q_out is not None else 0
        du = torch.empty_like(u.out)
        if merged:
            dpq = torch.empty_like(pq.out)
            dp, dq = dpq[:b], dpq[b:]
        else:
            dp = torch.empty_like(p_out)
            dq = torch.empty_like(q_out) if q_out is not None else None
        ws = self._loss_workspace(native.lib().rt_twotower_loss_workspace_bytes(b, d))
        ubias, ibias = m.user_bias, m.item_bias
        with TIMER.region("loss_fwd_bwd", flops=6.0 * b * b * d + 6.0 * b * (n_neg + 1) * d,
                          bytes_=4.0 * d * (4 * b + 2 * b * n_neg)):
            call("rt_twotower_loss_fwd_bwd", ptr(u.out), ptr(p_out), ptr(q_out) if q_out is not None else None, 0,
                 b, d, n_neg, 1.0 / m.temperature, ptr(ubias), ptr(ibias), self.we, self.wb, ptr(self.loss_buf),
                 ptr(du), ptr(dp), ptr(dq),
                 ptr(slab.grad_of(ubias)) if ubias is not None else None,
                 ptr(slab.grad_of(ibias)) if ibias is not None else None, ptr(ws), ws.numel(), st)
        # backward: independent chains (grads meet in the slab through atomics)
        if merged:  # user and item tower layer l in one dz and one dW launch
            chain_backward_pair((ib, pq, dpq, slab, False, so, self.a_pqb, False),
                                (ub, u, du, slab, False, so, self.a_ub, False))
        else:
            s_u.wait_stream(main)
            with torch.cuda.stream(s_u):
                chain_backward(ub, u, du, slab, seed_offset=so, stats_arena=self.a_ub, attach=False)
            s_p.wait_stream(main)
            with torch.cuda.stream(s_p):
                chain_backward(ib, p, dp, slab, seed_offset=so, stats_arena=self.a_pb, attach=False)
            if q is not None:
                chain_backward(ib, q, dq, slab, seed_offset=so, stats_arena=self.a_nb, attach=False)
            main.wait_stream(s_p)
        main.wait_stream(s_u)

    def _loss_workspace(self, nbytes: int) -> torch.Tensor:
        """This step's own loss workspace (a shared, growable
        workspace could be swapped out from under a captured graph by any other
        caller, e.g. a validation batch larger than the training batch)."""
        if self._loss_ws is None or self._loss_ws.numel() < nbytes:
            if self._loss_ws is not None:
                self._loss_ws_retired.append(self._loss_ws)
            self._loss_ws = torch.empty(max(nbytes, 256), dtype=torch.uint8, device=self.dev)
        return self._loss_ws

    def _allreduce(self):
        if self.pg is not None:  # data parallel: average the flat grad slab (one RCCL all-reduce)
            import torch.distributed as dist
            if dist.get_backend(self.pg) == "nccl":
                # RCCL averages in the collective (ncclAvg): no separate scaling launch
                dist.all_reduce(self.slab.grad, op=dist.ReduceOp.AVG, group=self.pg)
            else:  # gloo has no AVG
                dist.all_reduce(self.slab.grad, op=dist.ReduceOp.SUM, group=self.pg)
                self.slab.grad.mul_(1.0 / dist.get_world_size(self.pg))

    def _update(self):
        """clip_grad_norm_ + Adam on the flat slabs (device step counter / lr)."""
        slab = self.slab
        st = native.stream_of(slab.data)
        nb = slab.data.numel() * 4.0
        with TIMER.region("clip_adam", flops=0.0, bytes_=nb * 7):
            call("rt_grad_sqnorm", ptr(slab.grad), ptr(slab.tensor_offsets()), len(slab.params), ptr(self.sumsq),
                 ptr(self.step_dev), ptr(self.seed_dev), st)
            call("rt_clip_adam_step", ptr(slab.data), ptr(slab.grad), ptr(self.exp_avg), ptr(self.exp_avg_sq),
                 slab.data.numel(), ptr(self.sumsq), len(slab.params), self.max_norm, self.lr, ptr(self.lr_dev),
                 self.b1, self.b2, self.eps, self.wd, 1, ptr(self.step_dev), ptr(self.arena), self.arena.numel(), st)
        return self.loss_buf

    def __call__(self, user_src: torch.Tensor, pos_src: torch.Tensor, neg_src: Optional[torch.Tensor],
                 user_ids: Optional[torch.Tensor] = None, pos_ids: Optional[torch.Tensor] = None,
                 neg_ids: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Dense features ([B,Fu], [B,Fi], [B*N,Fi] or [B,N,Fi]) or feature tables
        with row ids (fused gather). Returns the device fp64 [3] loss buffer
        (loss, explicit, in-batch) — read it only when needed (sync)."""
        self.model.train()
        if neg_src is not None and neg_ids is None and neg_src.dim() == 3:
            neg_src = neg_src.reshape(-1, neg_src.shape[-1])
        self.steps += 1
        return self._run(user_src, pos_src, neg_src, user_ids, pos_ids, neg_ids)

    # ------------------------------------------------------------------
    # hipGraph capture of the whole step (ids/features in static buffers)
    def _state_tensors(self):
        """Everything a step mutates besides grads/arena: parameters, Adam
        moments, BN running stats / batch counters, step and dropout counters."""
        return [self.slab.data, self.exp_avg, self.exp_avg_sq, self.step_dev, self.seed_dev] + \
            [b for b in self.model.buffers()]

    def capture(self, user_src, pos_src, neg_src, user_ids=None, pos_ids=None, neg_ids=None, warmup: int = 2,
                restore: bool = True):
        """Capture the step as hipGraph(s) over static inputs (copy new ids /
        features into the tensors passed here, then ``replay()``). With a
        process group the step is two graphs — gradients, then clip+Adam — with
        the RCCL all-reduce launched eagerly between them.

        The ``warmup`` eager steps before capture are real steps on the static
        inputs (Adam, BN running stats, counters). With ``restore`` (default)
        the whole training state is snapshotted first and put back afterwards,
        so the first ``replay()`` is step 1 from the state the caller handed
        in; ``restore=False`` keeps the warmup updates."""
        self.model.train()
        snap = [t.clone() for t in self._state_tensors()] if restore else None
        s = torch.cuda.Stream(device=self.dev)
        s.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self._run(user_src, pos_src, neg_src, user_ids, pos_ids, neg_ids)
        torch.cuda.current_stream(self.dev).wait_stream(s)
        if snap is not None:
            with torch.no_grad():
                for t, v in zip(self._state_tensors(), snap):
                    t.copy_(v)
            del snap
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._grads(user_src, pos_src, neg_src, user_ids, pos_ids, neg_ids)
            if self.pg is None:
                self._update()
        self.graph = g
        self.graph_update = None
        if self.pg is not None:
            g2 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g2):
                self._update()
            self.graph_update = g2
        if not restore:
            self.steps += warmup
        return g

    def capture_body(self, body, extra_state=(), warmup: int = 2) -> torch.cuda.CUDAGraph:
        """Capture ``body`` — a full step built from ``_grads`` and ``_update``
        plus whatever device work the caller adds around it (e.g. the batch
        source, ``FeederGraph``) — as ONE hipGraph. As in ``capture``, the
        ``warmup`` eager runs are real steps, so the training state and
        ``extra_state`` are snapshotted first and restored afterwards.
        Single process only (a process group splits the step at its all-reduce)."""
        if self.pg is not None:
            raise RuntimeError("capture_body: data-parallel steps are captured as two graphs (capture())")
        self.model.train()
        tensors = self._state_tensors() + list(extra_state)
        snap = [t.clone() for t in tensors]
        s = torch.cuda.Stream(device=self.dev)
        s.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self._ensure_clean()
                body()
                self._clean = True
        torch.cuda.current_stream(self.dev).wait_stream(s)
        with torch.no_grad():
            for t, v in zip(tensors, snap):
                t.copy_(v)
        del snap
        self._ensure_clean()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            body()
        self._clean = True
        return g

    def replay(self):
        self._ensure_clean()
        self.graph.replay()
        if self.graph_update is not None:
            self._allreduce()
            self.graph_update.replay()
        self._clean = True
        self.steps += 1
        return self.loss_buf



class FeederGraph:
    """``DeviceFeeder`` batches and ``FusedTrainStep`` as ONE hipGraph per batch
    — the reference's epoch loop (src/training/trainers/two_tower.py:84-156 over
    the DataLoader of src/training/datasets/movielens.py:86-134) without a host
    round trip per batch.

    The epoch's permutation and a (batch cursor, sampler salt) pair live on the
    device. One replay: the batch's user / positive ids at the cursor
    (``rt_feeder_batch``), the on-device negatives (``rt_sample_negatives``
    with the salt as its device seed offset), the fused step, then
    ``rt_feeder_commit``: the loss into slot ``cursor`` of the epoch's loss
    buffer, cursor and salt + 1. The batches are bit-identical to
    iterating the feeder (same permutation generator, same sampler seeds), so
    an epoch here equals the eager epoch step for step. A partial last batch
    (``drop_last=False``) runs as an eager step."""

    def __init__(self, step: FusedTrainStep, feeder):
        if feeder.num_negatives <= 0:
            raise ValueError("FeederGraph: the mixed-loss step needs negatives")
        self.step, self.feeder = step, feeder
        dev = step.dev
        b, nn_ = feeder.batch_size, feeder.num_negatives
        self.n_rows = int(feeder.inter_u.numel())
        self.n_full = self.n_rows // b
        self.order = torch.empty(self.n_rows, dtype=torch.int64, device=dev)
        self.state = torch.zeros(2, dtype=torch.int64, device=dev)  # [batch cursor, sampler salt]
        ids = torch.empty(b * (2 + nn_), dtype=torch.int64, device=dev)  # users | positives, negatives (adjacent)
        self.users, self.pos, self.neg = ids[:b], ids[b:2 * b], ids[2 * b:]
        self.losses = torch.zeros(max(1, len(feeder)), dtype=torch.float64, device=dev)
        self.graph: Optional[torch.cuda.CUDAGraph] = None

    def _body(self):
        f, b = self.feeder, self.feeder.batch_size
        st = native.stream_of(self.order)
        call("rt_feeder_batch", ptr(self.order), ptr(f.inter_u), ptr(f.inter_m), ptr(self.state), b,
             ptr(self.users), ptr(self.pos), st)
        kernels.sample_negatives(f.csr.offsets, f.csr.items, self.users, f.num_items, f.num_negatives,
                                 seed=f.seed * 1_000_003, seed_offset=self.state[1:2],
                                 out=self.neg.view(b, f.num_negatives))
        self.step._grads(f.user_table, f.item_table, f.item_table, self.users, self.pos, self.neg)
        loss = self.step._update()
        call("rt_feeder_commit", ptr(loss), ptr(self.losses), self.losses.numel(), ptr(self.state), st)

    def _start_epoch(self, epoch: int):
        f = self.feeder
        if f.shuffle:
            g = torch.Generator(device=self.step.dev)
            g.manual_seed(f.seed + 7919 * epoch)  # the feeder's own permutation (DeviceFeeder.__iter__)
            self.order.copy_(torch.randperm(self.n_rows, device=self.step.dev, generator=g))
        else:
            torch.arange(self.n_rows, out=self.order)
        self.state.copy_(torch.tensor([0, epoch * 1_000_000], dtype=torch.int64))

    def run_epoch(self, max_batches: int = 0) -> torch.Tensor:
        """One epoch (at most ``max_batches`` batches when > 0) at the feeder's
        epoch counter; returns the device fp64 per-batch losses."""
        f = self.feeder
        n_b = len(f)
        if max_batches > 0:
            n_b = min(n_b, max_batches)
        n_graph = min(n_b, self.n_full)
        epoch = f.epoch
        if self.graph is None:  # warmup steps run on epoch 0's first batches, then everything is restored
            self._start_epoch(epoch)
            self.graph = self.step.capture_body(self._body, extra_state=(self.state, self.losses))
        self._start_epoch(epoch)
        self.step.model.train()
        for _ in range(n_graph):
            self.step._ensure_clean()
            self.graph.replay()
            self.step._clean = True
        self.step.steps += n_graph
        if n_b > n_graph:  # the partial last batch, eagerly (the feeder's own batch)
            idx = self.order[n_graph * f.batch_size:]
            bt = f.batch(idx, salt=epoch * 1_000_000 + n_graph)
            loss = self.step(bt["user_table"], bt["item_table"], bt["item_table"], user_ids=bt["user_ids"],
                             pos_ids=bt["pos_ids"], neg_ids=bt["neg_ids"])
            self.losses[n_graph:n_graph + 1].copy_(loss[0:1])
        f.epoch += 1
        return self.losses[:n_b]
