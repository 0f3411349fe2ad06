"""Multi-GPU paths of SURVEY §8(e): one process per GPU, torch.distributed
(backend "nccl" = RCCL over xGMI on MI355X).

* Corpus-sharded exact top-K (config C4). The reference serves one
  ``faiss.IndexFlatIP`` per process (src/serving/retrieval.py:70-197); here the
  corpus is row-partitioned into contiguous shards, every rank runs
  ``rt_flatip_topk`` on the same query tile against its shard with the shard's
  global row offset, the per-rank (score, id) lists are exchanged ONCE with
  ``all_gather_into_tensor`` and merged by ``rt_topk_merge`` under the
  (score desc, id asc) rule. Scores depend only on (query, row) and the
  reduction runs over D, so the merged result is identical to one GPU holding
  the whole corpus.
* Table-sharded row gather (config C5): the owner of row ``id`` is the rank
  whose contiguous range holds it; the batch ids are all-gathered, every rank
  gathers the rows it owns (in batch order) into one segment, the segments are
  all-gathered and a permutation gather puts every row in batch order on every
  rank (copies only).
* Data-parallel in-batch step of config C5 (:func:`sharded_inbatch_step`):
  each rank scores its own users against the whole gathered batch of items;
  for a trainable table the item-row gradients go back to their owners with
  one reduce-scatter (:func:`sharded_scatter_add_rows`).
* Data-parallel training: the flat fp32 grad slab is averaged with one
  all-reduce (see training/fused_step.py).

The orchestration functions take the per-rank compute as callables so the
collective logic is testable on CPU with the gloo backend; the product class
(`ShardedFlatIPIndex`) binds them to the HIP kernels only.
"""
from __future__ import annotations

from typing import Callable, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

from .. import kernels

TopkFn = Callable[[torch.Tensor, int], Tuple[torch.Tensor, torch.Tensor]]
MergeFn = Callable[[torch.Tensor, torch.Tensor, int], Tuple[torch.Tensor, torch.Tensor]]


def _world(group) -> Tuple[int, int]:
    if not dist.is_available() or not dist.is_initialized():
        return 1, 0
    return dist.get_world_size(group), dist.get_rank(group)


def shard_range(n_total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous balanced row partition: (begin, count) of ``rank``'s shard;
    the first ``n_total % world`` ranks hold one extra row."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} for world {world}")
    base, extra = divmod(int(n_total), world)
    begin = rank * base + min(rank, extra)
    return begin, base + (1 if rank < extra else 0)


def owner_of(ids: torch.Tensor, n_total: int, world: int) -> torch.Tensor:
    """Rank owning each global row id under :func:`shard_range`."""
    base, extra = divmod(int(n_total), world)
    cut = extra * (base + 1)
    ids = ids.to(torch.int64)
    low = torch.div(ids, base + 1, rounding_mode="floor")
    high = extra + torch.div(ids - cut, max(base, 1), rounding_mode="floor")
    return torch.where(ids < cut, low, high)


def all_gather_candidates(scores: torch.Tensor, ids: torch.Tensor, group=None
                          ) -> Tuple[torch.Tensor, torch.Tensor]:
    """[nq, k] per rank → [world, nq, k] on every rank (two all_gather_into_tensor,
    the only exchange step of the sharded search)."""
    world, _ = _world(group)
    if world == 1:
        return scores.unsqueeze(0), ids.unsqueeze(0)
    scores = scores.contiguous()
    ids = ids.contiguous()
    # concatenated along dim 0 (the layout every backend accepts), viewed [world, nq, k]
    out_s = torch.empty((world * scores.shape[0],) + tuple(scores.shape[1:]), dtype=scores.dtype,
                        device=scores.device)
    out_i = torch.empty((world * ids.shape[0],) + tuple(ids.shape[1:]), dtype=ids.dtype, device=ids.device)
    dist.all_gather_into_tensor(out_s, scores, group=group)
    dist.all_gather_into_tensor(out_i, ids, group=group)
    return out_s.view((world,) + tuple(scores.shape)), out_i.view((world,) + tuple(ids.shape))


def sharded_topk(queries: torch.Tensor, k: int, local_topk: TopkFn, merge: MergeFn,
                 group=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Exact top-k over a row-sharded corpus. ``local_topk`` returns this rank's
    (scores [nq,k], GLOBAL ids [nq,k]) padded with (-FLT_MAX, -1); ``merge`` maps
    [world, nq, k] lists to the final [nq, k]. Every rank returns the result."""
    s, i = local_topk(queries, k)
    world, _ = _world(group)
    if world == 1:
        return s, i
    all_s, all_i = all_gather_candidates(s, i, group)
    return merge(all_s, all_i, k)


def sharded_topk_owner(queries: torch.Tensor, k: int, local_topk: TopkFn, merge: MergeFn,
                       group=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Exact top-k over a row-sharded corpus where each rank OWNS a contiguous
    slice of the queries (``shard_range(nq, world, rank)``): every rank scans
    all queries against its shard, one ``all_to_all_single`` sends each query
    slice's (score, id) lists to its owner, and the owner merges world lists
    per query. Per-rank exchange volume is nq·k·12 B (an all-gather would move
    world× that to every rank), so the step stays scan-bound as world grows.
    Returns this rank's slice [nq_own, k]. nq must split evenly (nq % world == 0)."""
    s, i = local_topk(queries, k)
    world, rank = _world(group)
    if world == 1:
        return s, i
    nq = s.shape[0]
    if nq % world:
        raise ValueError(f"{nq} queries do not split over {world} ranks")
    s = s.contiguous()
    i = i.contiguous()
    out_s = torch.empty_like(s)
    out_i = torch.empty_like(i)
    dist.all_to_all_single(out_s, s, group=group)
    dist.all_to_all_single(out_i, i, group=group)
    per = nq // world
    return merge(out_s.view(world, per, k), out_i.view(world, per, k), k)


def sharded_gather_rows(table_shard: torch.Tensor, row_begin: int, ids: torch.Tensor, group=None,
                        gather: Optional[Callable] = None) -> torch.Tensor:
    """C5 row fetch from a row-sharded table: returns the rows of the GLOBAL
    batch (all ranks' ``ids`` concatenated in rank order) on every rank.

    Owner-segment exchange: one all-gather of (count, window) metadata and one
    of the batch ids; every rank gathers the rows IT owns, in batch order, into
    a segment padded to the largest owner's count; one all-gather of those
    segments and a permutation gather (segment of owner o, slot = rank of the
    position among o's positions) put the rows in batch order. Every row moves
    once per receiving rank and is copied, never summed, so the result is
    bit-identical to a single-table gather. ``gather(table, ids, row_begin)``
    returns [len(ids), dim] (``rt_gather_rows`` semantics, the default)."""
    gather = gather or (lambda t, i, b: kernels.gather_rows(t, i, row_begin=b))
    world, rank = _world(group)
    if world == 1:
        return gather(table_shard, ids, row_begin)
    dev = ids.device
    meta = torch.tensor([ids.numel(), int(row_begin), int(row_begin) + table_shard.shape[0]], dtype=torch.int64,
                        device=dev)
    all_meta = torch.empty(world * 3, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(all_meta, meta, group=group)
    all_meta = all_meta.view(world, 3)
    counts = [int(c) for c in all_meta[:, 0].tolist()]
    width = max(counts)
    if width == 0:
        return torch.empty((0, table_shard.shape[1]), dtype=table_shard.dtype, device=table_shard.device)
    padded = torch.full((width,), -1, dtype=torch.int64, device=dev)
    padded[: ids.numel()] = ids.to(torch.int64)
    all_ids = torch.empty((world * width,), dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(all_ids, padded, group=group)
    keep = torch.cat([torch.arange(r * width, r * width + c, device=dev) for r, c in enumerate(counts)])
    global_ids = all_ids[keep]
    # owner of each position: the rank whose [begin, end) window holds the id
    begins = all_meta[:, 1].contiguous()
    owner = torch.searchsorted(begins, global_ids, right=True) - 1
    bad = (owner < 0) | (global_ids >= all_meta[owner.clamp(min=0), 2])
    if bool(bad.any()):
        raise IndexError("batch id outside every rank's table window")
    per_owner = torch.bincount(owner, minlength=world)
    seg = int(per_owner.max())
    send = torch.zeros((seg, table_shard.shape[1]), dtype=table_shard.dtype, device=table_shard.device)
    mine = torch.nonzero(owner == rank).flatten()
    if mine.numel():
        send[: mine.numel()] = gather(table_shard, global_ids[mine], row_begin)
    segs = torch.empty((world * seg, table_shard.shape[1]), dtype=table_shard.dtype, device=table_shard.device)
    dist.all_gather_into_tensor(segs, send, group=group)
    order = torch.argsort(owner, stable=True)
    starts = torch.cumsum(per_owner, 0) - per_owner
    slot = torch.empty_like(owner)
    slot[order] = torch.arange(owner.numel(), device=dev) - starts[owner[order]]
    return gather(segs, owner * seg + slot, 0)


def sharded_scatter_add_rows(grad_shard: torch.Tensor, row_begin: int, global_ids: torch.Tensor,
                             grad_rows: torch.Tensor, group=None,
                             scatter_add: Optional[Callable] = None) -> torch.Tensor:
    """Backward of :func:`sharded_gather_rows` for a TRAINABLE row-sharded table
    (the nn.Embedding path a2 under C5 sharding, SURVEY §8(e) "next"): every rank
    holds its d loss / d rows for the whole global batch (``grad_rows`` [B_total,
    D], rows in the order of ``global_ids``); the owner of each row receives the
    sum over ranks and adds it into its shard's gradient (``grad_shard`` [rows,
    D], shard rows start at global ``row_begin``).

    One reduce-scatter moves each row's gradient once per rank: positions are
    ordered by owner (stable), each owner's segment padded to the largest
    segment, summed over ranks by ``reduce_scatter_tensor`` (an all-reduce of the
    same buffer on gloo, which has no reduce-scatter), and the owner's segment is
    scatter-added (``rt_scatter_add_rows_f32``; repeated ids accumulate)."""
    scatter_add = scatter_add or (lambda t, ids, g: kernels.scatter_add_rows(t, ids, g))
    world, rank = _world(group)
    ids = global_ids.to(torch.int64)
    if world == 1:
        return scatter_add(grad_shard, ids - row_begin, grad_rows)
    dev = ids.device
    win = torch.tensor([int(row_begin), int(row_begin) + grad_shard.shape[0]], dtype=torch.int64, device=dev)
    all_win = torch.empty(world * 2, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(all_win, win, group=group)
    all_win = all_win.view(world, 2)
    owner = torch.searchsorted(all_win[:, 0].contiguous(), ids, right=True) - 1
    if bool(((owner < 0) | (ids >= all_win[owner.clamp(min=0), 1])).any()):
        raise IndexError("batch id outside every rank's table window")
    per_owner = torch.bincount(owner, minlength=world)
    seg = int(per_owner.max())
    if seg == 0:
        return grad_shard
    order = torch.argsort(owner, stable=True)
    starts = torch.cumsum(per_owner, 0) - per_owner
    slot = torch.arange(ids.numel(), device=dev) - starts[owner[order]]
    d = grad_rows.shape[1]
    send = torch.zeros((world * seg, d), dtype=grad_rows.dtype, device=grad_rows.device)
    send[owner[order] * seg + slot] = grad_rows[order]
    recv = torch.empty((seg, d), dtype=grad_rows.dtype, device=grad_rows.device)
    if dist.get_backend(group) == "gloo":
        dist.all_reduce(send, op=dist.ReduceOp.SUM, group=group)
        recv.copy_(send[rank * seg:(rank + 1) * seg])
    else:
        dist.reduce_scatter_tensor(recv, send, op=dist.ReduceOp.SUM, group=group)
    n_mine = int(per_owner[rank])
    if n_mine:
        mine_ids = ids[order[starts[rank]:starts[rank] + n_mine]]
        scatter_add(grad_shard, mine_ids - row_begin, recv[:n_mine])
    return grad_shard


def sharded_inbatch_step(table_shard: torch.Tensor, row_begin: int, user_emb: torch.Tensor,
                         item_ids: torch.Tensor, temperature: float, group=None,
                         gather: Optional[Callable] = None, loss_fn: Optional[Callable] = None):
    """Config C5 data-parallel in-batch step (SURVEY §8(e) training): the item
    table is row-sharded, every rank holds ``user_emb`` [b, D] for its own b
    users and ``item_ids`` [b] of their positives. The global batch's item rows
    are fetched with :func:`sharded_gather_rows` (one id all-gather + one
    all-reduce), each rank scores its users against ALL gathered items (label of
    local user i = global item rank·b + i) with ``rt_inbatch_loss_fwd_bwd``, and
    the loss is averaged over ranks. Returns (global mean loss, d loss/d user_emb
    for the local users, d loss/d item rows summed over ranks [B_total, D]) —
    the latter is what the owners would scatter-add if the table were trainable
    (in the reference it is a precomputed feature table, so it is not)."""
    world, rank = _world(group)
    b = user_emb.shape[0]
    rows = sharded_gather_rows(table_shard, row_begin, item_ids, group, gather)
    loss_fn = loss_fn or (lambda u, p, off: kernels.inbatch_loss(u, p, temperature, label_offset=off))
    loss, du, dp = loss_fn(user_emb, rows, rank * b)
    lv = loss[0:1].clone()
    if world > 1:
        dist.all_reduce(lv, op=dist.ReduceOp.SUM, group=group)
        dist.all_reduce(dp, op=dist.ReduceOp.SUM, group=group)
    # each rank's loss is a mean over its own b users; the global mean averages them
    return lv / world, du / world, dp / world


def allreduce_mean_(t: torch.Tensor, group=None) -> torch.Tensor:
    """Data-parallel gradient average (one all-reduce of the flat grad slab)."""
    world, _ = _world(group)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        t.mul_(1.0 / world)
    return t


# ---------------------------------------------------------------------------
class ShardedFlatIPIndex:
    """Row-sharded exact inner-product index, one shard per rank in its GPU's HBM.

    ``build(embeddings)`` takes the full corpus on every rank (each keeps its
    slice) or ``build_shard(rows, begin, n_total)`` its own rows only. Search
    returns GLOBAL row positions; ``metric='cosine'`` renormalises with the
    Faiss rule (``rt_l2_renorm_f32``) before any storage cast, like the
    single-GPU ``HipFlatIPIndex``."""

    def __init__(self, dimension: int, group=None, device: Optional[torch.device] = None,
                 storage_dtype: torch.dtype = torch.float32, metric: str = "cosine"):
        self.dimension = dimension
        self.group = group
        self.world, self.rank = _world(group)
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.storage_dtype = storage_dtype
        if metric not in ("cosine", "inner_product"):
            raise NotImplementedError("ShardedFlatIPIndex serves the inner-product metrics ('cosine', "
                                      "'inner_product'); the L2 mode is single-GPU (HipFlatIPIndex)")
        self.metric = metric
        self.shard: Optional[torch.Tensor] = None
        self.begin = 0
        self.n_total = 0

    def _prep(self, x) -> torch.Tensor:
        t = torch.as_tensor(x) if not isinstance(x, torch.Tensor) else x
        if t.dim() == 1:
            t = t.reshape(1, -1)
        t = t.to(device=self.device, dtype=torch.float32, copy=True).contiguous()
        if t.shape[1] != self.dimension:
            raise ValueError(f"expected dimension {self.dimension}, got {t.shape[1]}")
        if self.metric == "cosine":
            kernels.l2_renorm_(t)
        return t.to(self.storage_dtype)

    def build_shard(self, rows, begin: int, n_total: int):
        self.shard = self._prep(rows)
        self.begin, self.n_total = int(begin), int(n_total)
        return self

    def build(self, embeddings):
        n = len(embeddings)
        b, c = shard_range(n, self.world, self.rank)
        return self.build_shard(embeddings[b:b + c], b, n)

    @property
    def current_size(self) -> int:
        return self.n_total

    def _local(self, excluded: Optional[Sequence[Sequence[int]]]) -> TopkFn:
        def fn(q: torch.Tensor, k: int):
            bits = None
            if excluded is not None:
                n_loc = self.shard.shape[0]
                loc = [[int(i) - self.begin for i in ex if self.begin <= int(i) < self.begin + n_loc]
                       for ex in excluded]
                bits = kernels.exclusion_bitmap(q.shape[0], n_loc, loc, q.device)
            return kernels.flatip_topk(q, self.shard, k, exclude_bits=bits, id_offset=self.begin)
        return fn

    def search_tensors(self, queries, k: int, excluded: Optional[Sequence[Sequence[int]]] = None
                       ) -> Tuple[torch.Tensor, torch.Tensor]:
        if self.shard is None:
            raise ValueError("Index not built yet")
        q = self._prep(queries)
        return sharded_topk(q, k, self._local(excluded), kernels.topk_merge, self.group)

    def search(self, queries, k: int = 10) -> Tuple[np.ndarray, np.ndarray]:
        s, i = self.search_tensors(queries, k)
        return s.cpu().numpy(), i.cpu().numpy()
