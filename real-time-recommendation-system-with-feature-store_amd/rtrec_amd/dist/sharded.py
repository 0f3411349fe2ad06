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
  gathers the whole batch against its own window (zero rows elsewhere) and one
  byte-wise MAX all-reduce leaves every owner's rows everywhere (copies only,
  no host synchronisation, graph-capturable).
* Data-parallel in-batch step of config C5 (:func:`sharded_inbatch_step`):
  each rank scores its own users against the whole gathered batch of items;
  the table is frozen as in the reference (no item-gradient exchange), or, for
  a trainable table, the item-row gradients are summed and added by their
  owners (:func:`sharded_scatter_add_rows`).
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


def _exchange_rows(local: torch.Tensor, group) -> torch.Tensor:
    """Every rank holds [P, D] rows that are zero except at the positions it owns
    (exactly one owner per valid position): the max over ranks of the raw BYTES
    (non-owners contribute 0x00) is the owner's row bit for bit — including
    -0.0 and NaN payloads, which a float sum would not preserve. One all-reduce
    (uint8 MAX; RCCL ncclUint8), no host synchronisation."""
    flat = local.contiguous().view(torch.uint8)
    dist.all_reduce(flat, op=dist.ReduceOp.MAX, group=group)
    return local


def sharded_gather_rows(table_shard: torch.Tensor, row_begin: int, ids: torch.Tensor, group=None,
                        gather: Optional[Callable] = None, counts: Optional[Sequence[int]] = None,
                        status: Optional[torch.Tensor] = None, check: bool = False,
                        return_ids: bool = False):
    """C5 row fetch from a row-sharded table: returns the rows of the GLOBAL
    batch (all ranks' ``ids`` concatenated in rank order) on every rank.

    Sync-free, graph-capturable exchange (no device→host read anywhere):
    one all-gather of the batch ids (each rank's ids padded to the batch width
    with -1); every rank gathers the WHOLE global batch against its own row
    window (``rt_gather_rows`` with ``row_begin``: ids outside the window, and
    the -1 padding, give zero rows and are counted as out-of-window); one
    all-reduce of the rows' bytes (:func:`_exchange_rows`) leaves every
    position holding its owner's row. Rows are copied, never summed, so the
    result is bit-identical to a single-table gather.

    ``counts``: per-rank batch sizes when they differ (host data, e.g. the last
    ragged batch); by default every rank's batch has this rank's size (the C5
    step). ``status`` (int64 [2], device, optional): accumulates (positions,
    positions owned by some rank); they differ iff some id lies outside every
    window — the id-range check without a sync. ``check=True`` reads it and
    raises IndexError (one sync). ``gather(table, ids, row_begin)`` returns
    [len(ids), dim] with zero rows outside the window, as ``rt_gather_rows``
    does (the default). ``return_ids``: also return the global ids (-1 padding
    removed)."""
    gather_fn = gather
    oob = None
    if gather_fn is None:
        oob = torch.zeros(1, dtype=torch.int32, device=ids.device)
        gather_fn = lambda t, i, b: kernels.gather_rows(t, i, row_begin=b, oob=oob)  # noqa: E731
    world, rank = _world(group)
    ids = ids.to(torch.int64)
    width = max(counts) if counts is not None else ids.numel()
    if counts is not None and ids.numel() != counts[rank]:
        raise ValueError(f"rank {rank} holds {ids.numel()} ids, counts say {counts[rank]}")
    if world > 1:
        padded = ids
        if ids.numel() != width:
            padded = torch.full((width,), -1, dtype=torch.int64, device=ids.device)
            padded[: ids.numel()] = ids
        all_ids = torch.empty((world * width,), dtype=torch.int64, device=ids.device)
        dist.all_gather_into_tensor(all_ids, padded.contiguous(), group=group)
    else:
        all_ids = ids
    rows = gather_fn(table_shard, all_ids, row_begin)
    n_valid = sum(counts) if counts is not None else world * width
    if status is not None or check:
        if oob is not None:
            owned = all_ids.numel() - oob.to(torch.int64)
        else:
            loc = all_ids - int(row_begin)
            owned = ((loc >= 0) & (loc < table_shard.shape[0])).sum().reshape(1)
        if world > 1:
            dist.all_reduce(owned, op=dist.ReduceOp.SUM, group=group)
        # (no host→device copy: capturable) positions, positions owned by some rank
        st = torch.cat([torch.full((1,), n_valid, dtype=torch.int64, device=ids.device), owned])
        if status is not None:
            status += st
        if check and int(st[0]) != int(st[1]):
            raise IndexError("batch id outside every rank's table window")
    if world > 1:
        rows = _exchange_rows(rows, group)
    if counts is not None and any(c != width for c in counts):  # drop the padding (host-known positions)
        keep = torch.cat([torch.arange(r * width, r * width + c, device=ids.device) for r, c in enumerate(counts)])
        rows = rows.index_select(0, keep)
        all_ids = all_ids.index_select(0, keep)
    return (rows, all_ids) if return_ids else rows


def sharded_scatter_add_rows(grad_shard: torch.Tensor, row_begin: int, global_ids: torch.Tensor,
                             grad_rows: torch.Tensor, group=None,
                             scatter_add: Optional[Callable] = None) -> torch.Tensor:
    """Backward of :func:`sharded_gather_rows` for a TRAINABLE row-sharded table
    (the nn.Embedding path a2 under C5 sharding, SURVEY §8(e) "next"): every rank
    holds its own contribution to d loss / d rows for the whole global batch
    (``grad_rows`` [B_total, D], rows in the order of ``global_ids``); the owner
    of each row adds the sum over ranks into its shard's gradient
    (``grad_shard`` [rows, D], shard rows start at global ``row_begin``).

    Sync-free: one all-reduce (sum) of the row gradients, then every rank
    scatter-adds the rows of its own window (``rt_scatter_add_rows_f32`` skips
    ids outside [0, rows); repeated ids accumulate)."""
    scatter_add = scatter_add or (lambda t, ids, g: kernels.scatter_add_rows(t, ids, g))
    world, _ = _world(group)
    g = grad_rows
    if world > 1:
        g = grad_rows.contiguous().clone()
        dist.all_reduce(g, op=dist.ReduceOp.SUM, group=group)
    return scatter_add(grad_shard, global_ids.to(torch.int64) - int(row_begin), g)


def sharded_inbatch_step(table_shard: torch.Tensor, row_begin: int, user_emb: torch.Tensor,
                         item_ids: torch.Tensor, temperature: float, group=None,
                         gather: Optional[Callable] = None, loss_fn: Optional[Callable] = None,
                         grad_shard: Optional[torch.Tensor] = None, status: Optional[torch.Tensor] = None,
                         scatter_add: Optional[Callable] = None):
    """Config C5 data-parallel in-batch step (SURVEY §8(e) training): the item
    table is row-sharded, every rank holds ``user_emb`` [b, D] for its own b
    users and ``item_ids`` [b] of their positives (b equal on every rank). The
    global batch's item rows come from :func:`sharded_gather_rows` (sync-free);
    each rank scores its users against ALL gathered items (label of local user
    i = global item rank·b + i) with ``rt_inbatch_loss_fwd_bwd``; the loss is
    averaged over ranks (one 8-byte all-reduce).

    The item table is a frozen feature table in the reference
    (src/training/datasets/movielens.py:61-63,116), so by default the item-row
    gradients are NOT exchanged: the third result is this rank's own
    contribution [B_total, D]. With ``grad_shard`` (a trainable table) they are
    summed and added into the owners' shards (:func:`sharded_scatter_add_rows`).
    No host synchronisation at any world size, N = 1 included (the same code
    runs; its collectives are skipped), so the whole step can be captured in a
    hipGraph. Returns (global mean loss [1], d loss/d user_emb, d loss/d rows
    (this rank's part))."""
    world, rank = _world(group)
    b = user_emb.shape[0]
    rows, gids = sharded_gather_rows(table_shard, row_begin, item_ids, group, gather, status=status,
                                     return_ids=True)
    loss_fn = loss_fn or (lambda u, p, off: kernels.inbatch_loss(u, p, temperature, label_offset=off))
    loss, du, dp = loss_fn(user_emb, rows, rank * b)
    lv = loss[0:1].clone()
    if world > 1:
        dist.all_reduce(lv, op=dist.ReduceOp.SUM, group=group)
    if grad_shard is not None:
        sharded_scatter_add_rows(grad_shard, row_begin, gids, dp.float() / world, group, scatter_add)
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
