"""Retrieval layer: the reference's ``IndexBase`` / ``RetrievalEngine`` surface
(src/serving/retrieval.py:16-46, 505-692) over an MI355X-resident exact
inner-product index.

``HipFlatIPIndex`` is the drop-in for ``FaissIndex`` in ``Flat`` mode
(retrieval.py:49-329): same constructor config keys, same
``build/search/add/save/load`` behaviour and errors, same ``(ids, scores)``
result lists, but the corpus lives in HBM and ``search`` runs the gfx950
Flat-IP top-K kernel (MFMA scoring + wavefront select) instead of Faiss-CPU.
"""
from __future__ import annotations

import hashlib
import json
import pickle
import struct
import time
from abc import ABC, abstractmethod
from pathlib import Path
from typing import Any, Dict, List, Optional, Tuple, Union

import numpy as np
import torch

from .. import kernels

Array = Union[np.ndarray, torch.Tensor]


class _Log:
    """Tiny stand-in for the reference's loguru calls (loguru is not a dependency)."""

    def __init__(self):
        import logging
        self._l = logging.getLogger("rtrec_amd.retrieval")

    def info(self, *a):
        self._l.info(*a)

    def warning(self, *a):
        self._l.warning(*a)

    def debug(self, *a):
        self._l.debug(*a)


logger = _Log()


class IndexBase(ABC):
    """Abstract base class for ANN indices (retrieval.py:16-46)."""

    @abstractmethod
    def build(self, embeddings: np.ndarray, ids: List[str]):
        """Build the index from embeddings."""

    @abstractmethod
    def search(self, query_embeddings: np.ndarray, k: int = 10) -> Tuple[np.ndarray, np.ndarray]:
        """Search for nearest neighbors."""

    @abstractmethod
    def add(self, embeddings: np.ndarray, ids: List[str]):
        """Add new embeddings to the index."""

    @abstractmethod
    def save(self, path: str):
        """Save index to disk."""

    @abstractmethod
    def load(self, path: str):
        """Load index from disk."""


_STORAGE = {"float32": torch.float32, "float16": torch.float16, "bfloat16": torch.bfloat16}


MAX_DIM = 256   # rt_flatip_topk: d <= 256 (f32 d % 4 == 0, f16/bf16 d % 8 == 0)
MAX_K_L2 = 512  # IndexFlatL2 mode: k <= 512 (its exact re-selection holds k_sel <= 512 candidates);
                # the inner-product modes take any k (kernels.flatip_topk: k > 512 in exact 512-wide passes)


def _default_device() -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("HipFlatIPIndex needs a ROCm device (no CPU fallback in the MI355X build)")
    return torch.device("cuda", torch.cuda.current_device())


class HipFlatIPIndex(IndexBase):
    """Exact inner-product index resident in HBM (FaissIndex ``Flat`` semantics).

    Config keys (retrieval.py:58-63): ``dimension`` (128), ``metric``
    ("cosine" → normalize_L2 on build/add/search + inner product, like
    IndexFlatIP; any other value → squared L2 distances ascending, like
    IndexFlatL2, float32 rows; "inner_product" → raw inner product, this
    build's extension),
    ``index_factory`` (only recorded: every factory is served exactly),
    ``nprobe`` (ignored, exact), plus ``device`` and ``storage_dtype``
    ("float32" default = Faiss numerics; "float16"/"bfloat16" halve the bytes).
    """

    def __init__(self, config: Optional[Dict[str, Any]] = None):
        self.config = config or {}
        self.dimension = self.config.get("dimension", 128)
        self.index_factory = self.config.get("index_factory", "Flat")
        self.metric = self.config.get("metric", "cosine")
        self.nprobe = self.config.get("nprobe", 20)
        self.storage_dtype = _STORAGE[self.config.get("storage_dtype", "float32")]
        # retrieval.py:96-100: "cosine" → IndexFlatIP on normalised rows, any other
        # metric → IndexFlatL2; "inner_product" (this build's extension) → raw IP
        self._l2 = self.metric not in ("cosine", "inner_product")
        if self._l2 and self.storage_dtype != torch.float32:
            raise ValueError("the L2 metric (IndexFlatL2) stores float32 rows, like Faiss")
        # what rt_flatip_topk serves (include/rtrec_hip.h): fail at construction,
        # not at the first search
        d_max = MAX_DIM - 4 if self._l2 else MAX_DIM
        step = 4 if self.storage_dtype == torch.float32 else 8
        if not (0 < self.dimension <= d_max) or self.dimension % step:
            raise ValueError(f"dimension {self.dimension} unsupported: the MI355X index serves d % {step} == 0, "
                             f"d <= {d_max} for {self.metric!r} / {self.config.get('storage_dtype', 'float32')}")
        dev = self.config.get("device")
        self.device = torch.device(dev) if dev is not None else None
        self.index: Optional[torch.Tensor] = None   # [capacity, d] device rows; first current_size valid
        self.id_map: Dict[int, str] = {}
        self.reverse_id_map: Dict[str, int] = {}
        self._ids: List[str] = []                  # position -> id (vectorised id_map)
        self.current_size = 0
        if "IVF" in str(self.index_factory):
            logger.warning("index_factory %s: the MI355X index serves every factory exactly (Flat)",
                           self.index_factory)

    # -- helpers -----------------------------------------------------------
    def _dev(self) -> torch.device:
        if self.device is None:
            self.device = _default_device()
        return self.device

    def _prepare(self, x: Array) -> torch.Tensor:
        """Copy to a contiguous fp32 device tensor (the index owns its vectors,
        retrieval.py:82) and renormalise in place for the cosine metric."""
        t = torch.as_tensor(x) if not isinstance(x, torch.Tensor) else x
        if t.dim() == 1:
            t = t.reshape(1, -1)
        t = t.to(device=self._dev(), dtype=torch.float32, copy=True).contiguous()
        if t.shape[1] != self.dimension:
            raise ValueError(f"expected dimension {self.dimension}, got {t.shape[1]}")
        if self.metric == "cosine":
            kernels.l2_renorm_(t)
        return t

    def _row_width(self) -> int:
        """Stored row width: d, or d + 4 augmented columns in the L2 mode
        ([x, -||x||^2/2, 0, 0, 0], rt_l2_augment_f32)."""
        return self.dimension + 4 if self._l2 else self.dimension

    def _store(self, rows: torch.Tensor):
        rows = rows.to(self.storage_dtype)
        n_new = self.current_size + rows.shape[0]
        if self.index is None or self.index.shape[0] < n_new:
            cap = max(n_new, 2 * (self.index.shape[0] if self.index is not None else 0), 1024)
            buf = torch.empty((cap, self._row_width()), dtype=self.storage_dtype, device=self._dev())
            if self.index is not None and self.current_size:
                buf[: self.current_size].copy_(self.index[: self.current_size])
            self.index = buf
        if self._l2:
            kernels.l2_augment(rows, 1, out=self.index[self.current_size:n_new])
        else:
            self.index[self.current_size:n_new].copy_(rows)

    # -- IndexBase ---------------------------------------------------------
    def build(self, embeddings: Array, ids: List[str]):
        """retrieval.py:70-139 (Flat path)."""
        start = time.time()
        rows = self._prepare(embeddings)
        self.index = None
        self.current_size = 0
        self.id_map, self.reverse_id_map, self._ids = {}, {}, []
        self._store(rows)
        for i, item_id in enumerate(ids):
            self.id_map[i] = item_id
            self.reverse_id_map[item_id] = i
        self._ids = list(ids) + [None] * max(0, rows.shape[0] - len(ids))
        self.current_size = rows.shape[0]
        logger.info("Index built in %.2f seconds", time.time() - start)

    def search_tensors(self, query_embeddings: Array, k: int,
                       exclude_bits: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        """Device-level search: (scores [nq,k], positions [nq,k]) with -1 padding;
        scores are inner products (descending) or, in the L2 mode, squared L2
        distances (ascending, IndexFlatL2.search)."""
        if self.index is None:
            raise ValueError("Index not built yet")
        q = self._prepare(query_embeddings).to(self.storage_dtype)
        if self._l2:
            if k > MAX_K_L2:
                raise ValueError(f"k={k} > {MAX_K_L2}: the MI355X IndexFlatL2 mode returns at most {MAX_K_L2} "
                                 "results per query (the inner-product metrics take any k)")
            return kernels.flatl2_topk(kernels.l2_augment(q, 0), self.index[: self.current_size], self.dimension, k,
                                       exclude_bits=exclude_bits)
        return kernels.flatip_topk(q, self.index[: self.current_size], k, exclude_bits=exclude_bits)

    def search(self, query_embeddings: Array, k: int = 10,
               filter_ids: Optional[List[str]] = None) -> Tuple[List[List[str]], List[List[float]]]:
        """retrieval.py:141-197: normalise, top-k_search (2k when filtering), map
        positions to ids, drop -1 padding, apply the filter, stop at k."""
        if self.index is None:
            raise ValueError("Index not built yet")
        k_search = min(k * 2, self.current_size) if filter_ids else k
        if k_search <= 0:
            n = 1 if np.ndim(query_embeddings) == 1 else len(query_embeddings)
            return [[] for _ in range(n)], [[] for _ in range(n)]
        scores, pos = self.search_tensors(query_embeddings, k_search)
        return _lists_from_positions(scores.cpu().numpy(), pos.cpu().numpy(), self.id_map, k, filter_ids)

    def add(self, embeddings: Array, ids: List[str]):
        """retrieval.py:199-226: incremental append (Kafka item_update path)."""
        if self.index is None:
            raise ValueError("Index not built yet")
        rows = self._prepare(embeddings)
        self._store(rows)
        for i, item_id in enumerate(ids):
            new_idx = self.current_size + i
            self.id_map[new_idx] = item_id
            self.reverse_id_map[item_id] = new_idx
        self._ids.extend(list(ids) + [None] * max(0, rows.shape[0] - len(ids)))
        self.current_size += rows.shape[0]
        logger.info("Added %d items to index. Total size: %d", rows.shape[0], self.current_size)

    def update(self, embeddings: Array, ids: List[str]):
        """retrieval.py:228-237 (no-op with a warning, like the reference)."""
        logger.warning("Flat index doesn't support direct updates. Consider periodic rebuilds.")

    def remove(self, ids: List[str]):
        logger.warning("Flat index doesn't support removal. Consider periodic rebuilds.")

    def vectors(self) -> np.ndarray:
        if self.index is None:
            return np.zeros((0, self.dimension), np.float32)
        return self.index[: self.current_size, : self.dimension].float().cpu().numpy()

    def save(self, path: str):
        """retrieval.py:248-273: ``<path>.faiss`` (IndexFlatIP/IndexFlatL2 binary
        layout: fourcc, header, code vector) + ``<path>.pkl`` id maps."""
        if self.index is None:
            raise ValueError("No index to save")
        path = Path(path)
        path.parent.mkdir(parents=True, exist_ok=True)
        write_flat_index(path.with_suffix(".faiss"), self.vectors(), not self._l2)
        with open(path.with_suffix(".pkl"), "wb") as f:
            pickle.dump({"id_map": self.id_map, "reverse_id_map": self.reverse_id_map,
                         "current_size": self.current_size, "config": self.config}, f)
        logger.info("Saved index to %s", path)

    def load(self, path: str):
        """retrieval.py:275-299."""
        path = Path(path)
        vecs, _ip = read_flat_index(path.with_suffix(".faiss"))
        with open(path.with_suffix(".pkl"), "rb") as f:
            data = pickle.load(f)  # files this index wrote (same layout as the reference's)
        self.id_map = data["id_map"]
        self.reverse_id_map = data["reverse_id_map"]
        self.config = data.get("config", self.config)
        self.metric = self.config.get("metric", self.metric)
        self._l2 = self.metric not in ("cosine", "inner_product")
        self.dimension = vecs.shape[1]
        self.index = None
        self.current_size = 0
        self._store(torch.from_numpy(vecs).to(self._dev()))
        self.current_size = int(data["current_size"])
        self._ids = [self.id_map.get(i) for i in range(self.current_size)]
        logger.info("Loaded index from %s with %d items", path, self.current_size)


# Faiss 1.7.x binary layout of IndexFlat (restated from the published format:
# fourcc, d:int32, ntotal:int64, 2 x dummy int64, is_trained:bool, metric:int32,
# then the code vector as a size_t count of floats followed by the floats).
_FOURCC_IP = b"IxFI"
_FOURCC_L2 = b"IxF2"


def write_flat_index(path: Path, vecs: np.ndarray, inner_product: bool = True):
    vecs = np.ascontiguousarray(vecs, dtype=np.float32)
    n, d = vecs.shape
    with open(path, "wb") as f:
        f.write(_FOURCC_IP if inner_product else _FOURCC_L2)
        f.write(struct.pack("<iqqq?i", d, n, 1 << 20, 1 << 20, True, 0 if inner_product else 1))
        f.write(struct.pack("<Q", n * d))
        f.write(vecs.tobytes())


def read_flat_index(path: Path) -> Tuple[np.ndarray, bool]:
    with open(path, "rb") as f:
        four = f.read(4)
        if four not in (_FOURCC_IP, _FOURCC_L2):
            raise ValueError(f"{path}: not a flat index (fourcc {four!r})")
        d, n, _, _, _, _metric = struct.unpack("<iqqq?i", f.read(struct.calcsize("<iqqq?i")))
        (cnt,) = struct.unpack("<Q", f.read(8))
        if cnt != n * d:
            raise ValueError(f"{path}: corrupt code vector ({cnt} != {n}*{d})")
        vecs = np.frombuffer(f.read(cnt * 4), dtype=np.float32).reshape(n, d).copy()
    return vecs, four == _FOURCC_IP


class HipShardedFlatIPIndex(IndexBase):
    """The same ``IndexBase`` contract as :class:`HipFlatIPIndex` (FaissIndex
    ``Flat``, retrieval.py:49-329) over a corpus ROW-SHARDED across the ranks
    of a process group, one shard in each GPU's HBM.

    It is an SPMD object: every rank constructs it and makes the same calls
    with the same arguments (``build``/``add`` with the whole batch of rows,
    ``search`` with the same queries), like every collective API, and every
    rank gets the full result.

    * **Layout.** Global positions follow build order, then add order, exactly
      as in one :class:`HipFlatIPIndex` (so results are equal id for id).
      ``build`` keeps rank r's contiguous slice ``shard_range(N, world, r)``;
      each ``add`` of m rows appends to every rank the slice
      ``shard_range(m, world, r)`` of the new global rows, so shards stay
      balanced. A rank's rows stay in increasing global order (an ``int64``
      position map on the device once an add made them non-contiguous), so the
      kernels' lower-id-wins tie rule holds globally.
    * **Search** (:func:`rtrec_amd.dist.sharded.sharded_topk_global`): one
      corpus-wide threshold per query from the ranks' shard samples, each
      rank's rows at or above it, all-to-all + owner merge
      (``rt_topk_merge``), one all-gather of the merged slices (``layout="all"``,
      the IndexBase ``search``) — or each rank only its slice of the queries
      (``layout="owner"``, :meth:`search_tensors`, what ``bench.py`` times).
      Shapes without the 16-bit v4 plan (float32 storage, k > 128) take the
      plain form of the same exchange. Queries run in tiles of
      ``query_tile`` (65,536) rows.
    * **string ids**: the id map is replicated on every rank (host data).
      ``filter_ids`` over-fetches ``k_search = min(2k, N)`` like FaissIndex
      (retrieval.py:170-195); -1 padding is dropped; k <= 512.
    * **save/load**: each rank writes its own ``<path>.shard{r}of{W}.faiss``
      (IndexFlat layout) and ``.pos.npy`` (its global positions); rank 0 writes
      the ``<path>.pkl`` id maps. ``load`` on the same world size reads only
      this rank's files; on another world size (or from a single-GPU
      :class:`HipFlatIPIndex` save, ``<path>.faiss``) it re-shards.

    Config keys: those of :class:`HipFlatIPIndex` for the inner-product
    metrics ("cosine", "inner_product"), plus ``process_group`` (default: the
    default group; world 1 without one) and ``query_tile``.
    """

    MAX_K = 512  # rt_topk_merge: k_out <= 512

    def __init__(self, config: Optional[Dict[str, Any]] = None):
        self.config = dict(config or {})
        self.dimension = self.config.get("dimension", 128)
        self.index_factory = self.config.get("index_factory", "Flat")
        self.metric = self.config.get("metric", "cosine")
        self.nprobe = self.config.get("nprobe", 20)
        if self.metric not in ("cosine", "inner_product"):
            raise ValueError("the sharded index serves the inner-product metrics ('cosine', 'inner_product'); "
                             "IndexFlatL2 is the single-GPU HipFlatIPIndex")
        self.storage_dtype = _STORAGE[self.config.get("storage_dtype", "float32")]
        step = 4 if self.storage_dtype == torch.float32 else 8
        if not (0 < self.dimension <= MAX_DIM) or self.dimension % step:
            raise ValueError(f"dimension {self.dimension} unsupported: the MI355X index serves d % {step} == 0, "
                             f"d <= {MAX_DIM}")
        self.group = self.config.pop("process_group", None)
        self.query_tile = int(self.config.get("query_tile", 65536))
        dev = self.config.get("device")
        self.device = torch.device(dev) if dev is not None else None
        from ..dist import sharded as _sh
        self._sh = _sh
        self.world, self.rank = _sh._world(self.group)
        self._reset()

    # -- hooks (the CPU orchestration tests substitute these) ---------------
    def _dev(self) -> torch.device:
        if self.device is None:
            self.device = _default_device()
        return self.device

    def _renorm_(self, t: torch.Tensor) -> torch.Tensor:
        return kernels.l2_renorm_(t)

    def _ops(self, rows: torch.Tensor):
        return self._sh.ShardOps(rows, self.begin, self.gpos)

    def _merge(self, s, i, k):
        return kernels.topk_merge(s, i, k)

    # -- layout --------------------------------------------------------------
    def _reset(self):
        self.shard: Optional[torch.Tensor] = None  # [capacity, d] storage rows; first n_local valid
        self.n_local = 0
        self.begin = 0                             # global position of local row 0 (contiguous shard)
        self.gpos: Optional[torch.Tensor] = None   # int64 [n_local] global positions once non-contiguous
        self.shard_sizes: List[int] = [0] * self.world
        self.id_map: Dict[int, str] = {}
        self.reverse_id_map: Dict[str, int] = {}
        self._ids: List[Optional[str]] = []
        self._implicit_ids = False                 # build_shard without ids: id = str(position)
        self.current_size = 0

    def _prepare(self, x: Array) -> torch.Tensor:
        """Contiguous fp32 device copy (the index owns its vectors), Faiss
        renorm for the cosine metric (retrieval.py:82-86)."""
        t = torch.as_tensor(x) if not isinstance(x, torch.Tensor) else x
        if t.dim() == 1:
            t = t.reshape(1, -1)
        t = t.to(device=self._dev(), dtype=torch.float32, copy=True).contiguous()
        if t.shape[1] != self.dimension:
            raise ValueError(f"expected dimension {self.dimension}, got {t.shape[1]}")
        if self.metric == "cosine" and t.shape[0]:
            self._renorm_(t)
        return t

    def _append_local(self, rows: torch.Tensor, positions: Optional[torch.Tensor]):
        """Append prepared rows (their global positions: ``positions``, or the
        contiguous run after the current ones when None)."""
        rows = rows.to(self.storage_dtype)
        n_new = self.n_local + rows.shape[0]
        if self.shard is None or self.shard.shape[0] < n_new:
            cap = max(n_new, 2 * (self.shard.shape[0] if self.shard is not None else 0), 1024)
            buf = torch.empty((cap, self.dimension), dtype=self.storage_dtype, device=self._dev())
            if self.shard is not None and self.n_local:
                buf[: self.n_local].copy_(self.shard[: self.n_local])
            self.shard = buf
        self.shard[self.n_local:n_new].copy_(rows)
        if positions is not None:
            if self.gpos is None:
                self.gpos = torch.arange(self.begin, self.begin + self.n_local, dtype=torch.int64,
                                         device=self._dev())
            self.gpos = torch.cat([self.gpos, positions.to(device=self._dev(), dtype=torch.int64)])
        self.n_local = n_new

    def _set_ids(self, start: int, ids: List[str], n_rows: int):
        for i, item_id in enumerate(ids):
            self.id_map[start + i] = item_id
            self.reverse_id_map[item_id] = start + i
        self._ids.extend(list(ids)[:n_rows] + [None] * max(0, n_rows - len(ids)))

    # -- IndexBase -------------------------------------------------------------
    def build(self, embeddings: Array, ids: List[str]):
        """retrieval.py:70-139 (Flat): every rank passes the whole corpus and
        keeps its slice."""
        start = time.time()
        n = len(embeddings)
        self._reset()
        b, c = self._sh.shard_range(n, self.world, self.rank)
        self.begin = b
        self._append_local(self._prepare(embeddings[b:b + c]), None)
        self.shard_sizes = [self._sh.shard_range(n, self.world, r)[1] for r in range(self.world)]
        self._set_ids(0, ids, n)
        self.current_size = n
        logger.info("Sharded index built in %.2f seconds (%d of %d rows on rank %d)", time.time() - start, c, n,
                    self.rank)

    def build_shard(self, rows: Array, n_total: int, ids: Optional[List[str]] = None, prepared: bool = False):
        """Rank-local build: this rank passes only ITS slice
        ``shard_range(n_total, world, rank)`` of the corpus (e.g. rows that
        already live on its GPU). ``prepared``: the rows are already
        normalised (no renorm)."""
        self._reset()
        b, c = self._sh.shard_range(n_total, self.world, self.rank)
        if len(rows) != c:
            raise ValueError(f"rank {self.rank} holds {len(rows)} rows, shard_range says {c}")
        self.begin = b
        if prepared:
            t = rows if isinstance(rows, torch.Tensor) else torch.as_tensor(rows)
            self._append_local(t.to(self._dev()), None)
        else:
            self._append_local(self._prepare(rows), None)
        self.shard_sizes = [self._sh.shard_range(n_total, self.world, r)[1] for r in range(self.world)]
        if ids is None:  # string ids = positions, materialised only when needed (add / save / load)
            self._implicit_ids = True
        else:
            self._set_ids(0, ids, n_total)
        self.current_size = int(n_total)
        return self

    def _materialize_ids(self):
        if self._implicit_ids:
            self._implicit_ids = False
            self._set_ids(0, [str(i) for i in range(self.current_size)], self.current_size)

    def add(self, embeddings: Array, ids: List[str]):
        """retrieval.py:199-226: every rank passes the whole batch; the new
        global rows current_size.. are spread over the ranks (shard_range of
        the batch), each rank appending its slice."""
        if self.shard is None:
            raise ValueError("Index not built yet")
        self._materialize_ids()
        m = len(embeddings)
        b, c = self._sh.shard_range(m, self.world, self.rank)
        pos = torch.arange(self.current_size + b, self.current_size + b + c, dtype=torch.int64)
        self._append_local(self._prepare(embeddings[b:b + c]), pos)
        self.shard_sizes = [s + self._sh.shard_range(m, self.world, r)[1] for r, s in enumerate(self.shard_sizes)]
        self._set_ids(self.current_size, ids, m)
        self.current_size += m
        logger.info("Added %d items to index. Total size: %d", m, self.current_size)

    def update(self, embeddings: Array, ids: List[str]):
        logger.warning("Flat index doesn't support direct updates. Consider periodic rebuilds.")

    def remove(self, ids: List[str]):
        logger.warning("Flat index doesn't support removal. Consider periodic rebuilds.")

    def search_tensors(self, query_embeddings: Array, k: int, layout: str = "all", prepared: bool = False
                       ) -> Tuple[torch.Tensor, torch.Tensor]:
        """(scores [nq, k], global positions [nq, k]) with (-FLT_MAX, -1)
        padding. ``layout="all"``: every rank gets every query's result;
        ``"owner"``: each rank gets its slice ``shard_range(tile, world, rank)``
        of every query tile (nq % world == 0). ``prepared``: the queries are a
        device tensor already normalised and in the storage dtype (no copy)."""
        if self.shard is None:
            raise ValueError("Index not built yet")
        if not 0 < k <= self.MAX_K:
            raise ValueError(f"k={k}: the sharded index returns 1..{self.MAX_K} results per query")
        if layout not in ("all", "owner"):
            raise ValueError(f"layout {layout!r}")
        if prepared:
            q = query_embeddings
            if q.dtype != self.storage_dtype or q.dim() != 2 or q.shape[1] != self.dimension:
                raise ValueError("prepared queries must be [nq, dimension] in the storage dtype")
        else:
            q = self._prepare(query_embeddings).to(self.storage_dtype)
        owner = layout == "owner"
        if owner and q.shape[0] % self.world:
            raise ValueError(f"{q.shape[0]} queries do not split over {self.world} ranks")
        tile = max(self.query_tile - self.query_tile % self.world, self.world)
        ops = self._ops(self.shard[: self.n_local])
        parts_s, parts_i = [], []
        for t0 in range(0, max(q.shape[0], 1), tile):
            qt = q[t0:t0 + tile]
            if qt.shape[0] == 0:
                break
            s, i = self._sh.sharded_topk_global(qt, k, self.current_size, ops, self._merge, self.group,
                                                owner=owner, shard_rows=self.shard_sizes)
            parts_s.append(s)
            parts_i.append(i)
        if not parts_s:
            return (torch.empty((0, k), dtype=torch.float32, device=q.device),
                    torch.empty((0, k), dtype=torch.int64, device=q.device))
        if len(parts_s) == 1:
            return parts_s[0], parts_i[0]
        return torch.cat(parts_s), torch.cat(parts_i)

    def search(self, query_embeddings: Array, k: int = 10,
               filter_ids: Optional[List[str]] = None) -> Tuple[List[List[str]], List[List[float]]]:
        """retrieval.py:141-197 on every rank (collective)."""
        if self.shard is None:
            raise ValueError("Index not built yet")
        k_search = min(k * 2, self.current_size) if filter_ids else k
        if k_search <= 0:
            n = 1 if np.ndim(query_embeddings) == 1 else len(query_embeddings)
            return [[] for _ in range(n)], [[] for _ in range(n)]
        scores, pos = self.search_tensors(query_embeddings, k_search)
        id_map = _PositionIds(self.current_size) if self._implicit_ids else self.id_map
        return _lists_from_positions(scores.cpu().numpy(), pos.cpu().numpy(), id_map, k, filter_ids)

    def vectors(self) -> np.ndarray:
        """This rank's rows (fp32, global order)."""
        if self.shard is None:
            return np.zeros((0, self.dimension), np.float32)
        return self.shard[: self.n_local].float().cpu().numpy()

    def positions(self) -> np.ndarray:
        """Global positions of this rank's rows."""
        if self.gpos is not None:
            return self.gpos.cpu().numpy()
        return np.arange(self.begin, self.begin + self.n_local, dtype=np.int64)

    def _shard_files(self, path: Path, r: int, w: int) -> Tuple[Path, Path]:
        """(rows .faiss, positions .npy) of shard r of w, next to ``path``."""
        stem = path.with_suffix("").name
        return (path.with_name(f"{stem}.shard{r}of{w}.faiss"), path.with_name(f"{stem}.shard{r}of{w}.pos.npy"))

    def _barrier(self):
        if self.world > 1:
            import torch.distributed as dist
            dist.barrier(group=self.group)

    def save(self, path: str):
        """Per-shard save: ``<path>.shard{r}of{W}.faiss`` + ``.pos.npy`` on every
        rank, ``<path>.pkl`` (id maps, layout) from rank 0 (retrieval.py:248-273)."""
        if self.shard is None:
            raise ValueError("No index to save")
        self._materialize_ids()
        path = Path(path)
        path.parent.mkdir(parents=True, exist_ok=True)
        fx, fp = self._shard_files(path, self.rank, self.world)
        write_flat_index(fx, self.vectors(), True)
        with open(fp, "wb") as f:
            np.save(f, self.positions(), allow_pickle=False)
        if self.rank == 0:
            with open(path.with_suffix(".pkl"), "wb") as f:
                pickle.dump({"id_map": self.id_map, "reverse_id_map": self.reverse_id_map,
                             "current_size": self.current_size, "config": self.config,
                             "world": self.world, "shard_sizes": self.shard_sizes}, f)
        self._barrier()
        logger.info("Saved shard %d of %d to %s", self.rank, self.world, fx)

    def load(self, path: str):
        """retrieval.py:275-299. Same world size: this rank's shard files only;
        another world size, or a single-GPU save (``<path>.faiss``): the rows
        are re-sharded by global position."""
        path = Path(path)
        with open(path.with_suffix(".pkl"), "rb") as f:
            data = pickle.load(f)  # files this package wrote
        n = int(data["current_size"])
        saved_world = data.get("world")
        self._reset()
        cfg = data.get("config", {})
        self.metric = cfg.get("metric", self.metric)
        if saved_world == self.world:
            fx, fp = self._shard_files(path, self.rank, self.world)
            vecs, _ = read_flat_index(fx)
            pos = np.load(fp, allow_pickle=False)
            self.shard_sizes = [int(s) for s in data["shard_sizes"]]
        else:
            if saved_world is None:  # a HipFlatIPIndex save: the whole corpus in one file
                full, _ = read_flat_index(path.with_suffix(".faiss"))
            else:
                full = np.zeros((n, self.dimension), np.float32)
                for r in range(saved_world):
                    fx, fp = self._shard_files(path, r, saved_world)
                    v, _ = read_flat_index(fx)
                    full[np.load(fp, allow_pickle=False)] = v
            b, c = self._sh.shard_range(n, self.world, self.rank)
            vecs, pos = full[b:b + c], np.arange(b, b + c, dtype=np.int64)
            self.shard_sizes = [self._sh.shard_range(n, self.world, r)[1] for r in range(self.world)]
        if vecs.shape[1] != self.dimension:
            raise ValueError(f"{path}: dimension {vecs.shape[1]} != {self.dimension}")
        contiguous = pos.size == 0 or bool(np.all(np.diff(pos) == 1))
        self.begin = int(pos[0]) if pos.size else int(sum(self.shard_sizes[:self.rank]))
        self._append_local(torch.from_numpy(vecs).to(self._dev()),  # stored rows: no second renorm
                           None if contiguous else torch.from_numpy(pos))
        self.id_map = data["id_map"]
        self.reverse_id_map = data["reverse_id_map"]
        self._ids = [self.id_map.get(i) for i in range(n)]
        self.current_size = n
        logger.info("Loaded shard %d of %d from %s (%d of %d rows)", self.rank, self.world, path, self.n_local, n)


class _PositionIds:
    """id_map of an index built without ids: position p -> str(p)."""

    def __init__(self, n: int):
        self.n = n

    def __contains__(self, p) -> bool:
        return 0 <= p < self.n

    def __getitem__(self, p) -> str:
        return str(p)


def _lists_from_positions(scores: np.ndarray, pos: np.ndarray, id_map: Dict[int, str], k: int,
                          filter_ids: Optional[List[str]]) -> Tuple[List[List[str]], List[List[float]]]:
    """retrieval.py:176-195: positions -> string ids, -1 padding dropped, the
    filter applied, at most k per query."""
    allowed = set(filter_ids) if filter_ids is not None else None
    batch_ids, batch_scores = [], []
    for i in range(pos.shape[0]):
        item_ids, item_scores = [], []
        for j in range(pos.shape[1]):
            p = int(pos[i, j])
            if p >= 0 and p in id_map:
                item_id = id_map[p]
                if allowed is None or item_id in allowed:
                    item_ids.append(item_id)
                    item_scores.append(float(scores[i, j]))
                    if len(item_ids) >= k:
                        break
        batch_ids.append(item_ids)
        batch_scores.append(item_scores)
    return batch_ids, batch_scores


# Backwards-compatible name: configs with index_type "faiss" get the exact
# HBM-resident index (Faiss-CPU is not part of the MI355X build).
FaissIndex = HipFlatIPIndex

_INDEX_TYPES = {"hip_flat": HipFlatIPIndex, "faiss": HipFlatIPIndex, "hip_flat_sharded": HipShardedFlatIPIndex}


def register_index(name: str, cls):
    """Plugin hook: make ``RetrievalEngine(config)`` accept ``index_type=name``."""
    _INDEX_TYPES[name] = cls


class RetrievalEngine:
    """High-level retrieval engine with md5 query cache and metrics
    (retrieval.py:505-692)."""

    def __init__(self, config: Dict[str, Any]):
        self.config = config
        self.index_type = config.get("index_type", "faiss")
        self.top_k = config.get("top_k", 100)
        self.update_interval = config.get("update_interval_seconds", 300)
        self.index = self._create_index()
        self.cache: Dict[str, Dict[str, Any]] = {}
        self.cache_ttl = config.get("cache_ttl", 300)
        self.last_cache_clear = time.time()
        self.total_queries = 0
        self.cache_hits = 0
        self.total_latency = 0.0

    def _create_index(self) -> IndexBase:
        """retrieval.py:532-544 string dispatch (+ the "hip_flat" type)."""
        index_config = dict(self.config.get(self.index_type, {}) or {})
        index_config["dimension"] = self.config.get("embedding_dim", 128)
        cls = _INDEX_TYPES.get(self.index_type)
        if cls is None:
            raise ValueError(f"Unknown index type: {self.index_type}")
        return cls(index_config)

    def build_index(self, embeddings: Array, ids: List[str]):
        self.index.build(embeddings, ids)
        self.cache.clear()
        logger.info("Built index with %d items", len(embeddings))

    def retrieve(self, query_embeddings: Array, k: Optional[int] = None,
                 filter_ids: Optional[List[str]] = None, use_cache: bool = True
                 ) -> Tuple[List[List[str]], List[List[float]], Dict[str, Any]]:
        start = time.time()
        k = k or self.top_k
        cache_key = None
        if use_cache and filter_ids is None:
            qb = query_embeddings.detach().cpu().numpy().tobytes() if isinstance(query_embeddings, torch.Tensor) \
                else np.asarray(query_embeddings).tobytes()
            cache_key = hashlib.md5(qb).hexdigest()
            entry = self.cache.get(cache_key)
            if entry is not None and time.time() - entry["timestamp"] < self.cache_ttl:
                self.cache_hits += 1
                latency = time.time() - start
                self.total_queries += 1
                self.total_latency += latency
                return entry["ids"], entry["scores"], {"latency_ms": latency * 1000, "cache_hit": True}
        item_ids, scores = self.index.search(query_embeddings, k, filter_ids)
        if use_cache and cache_key:
            self.cache[cache_key] = {"ids": item_ids, "scores": scores, "timestamp": time.time()}
            if time.time() - self.last_cache_clear > self.cache_ttl:
                self._clear_expired_cache()
        latency = time.time() - start
        self.total_queries += 1
        self.total_latency += latency
        flat = [s for sl in scores for s in sl]
        metrics = {"latency_ms": latency * 1000, "cache_hit": False,
                   "num_results": sum(len(x) for x in item_ids),
                   "avg_score": float(np.mean(flat)) if flat else float("nan")}
        return item_ids, scores, metrics

    def update_index(self, new_embeddings: Array, new_ids: List[str]):
        self.index.add(new_embeddings, new_ids)
        self.cache.clear()

    def _clear_expired_cache(self):
        now = time.time()
        for key in [k for k, e in self.cache.items() if now - e["timestamp"] > self.cache_ttl]:
            del self.cache[key]
        self.last_cache_clear = now

    def get_metrics(self) -> Dict[str, Any]:
        return {
            "total_queries": self.total_queries,
            "avg_latency_ms": self.total_latency / max(self.total_queries, 1) * 1000,
            "cache_hit_rate": self.cache_hits / max(self.total_queries, 1),
            "cache_size": len(self.cache),
            "index_size": self.index.current_size,
            "index_type": self.index_type,
        }

    def save(self, path: str):
        self.index.save(path)

    def load(self, path: str):
        self.index.load(path)
        self.cache.clear()
