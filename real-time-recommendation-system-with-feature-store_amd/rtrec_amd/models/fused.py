"""Host-side executor of the fused tower MLP kernels (rt_linear_fwd_f32 /
rt_linear_bwd_f32) and the flat parameter slab.

A tower's ``mlp`` (src/models/two_tower.py:56-72: [Linear → act → BatchNorm1d →
Dropout] × L → Linear) is run as L+1 kernel launches forward and 2(L+1)
backward; the row gather of the input features (layer 1), BatchNorm (batch
statistics finalised from fp64 column sums), activation, dropout and the final
F.normalize are fused into those launches. Parameter gradients are
accumulated straight into one flat fp32 grad slab (views are the params'
``.grad``), so the optimiser is one fused clip+Adam kernel.
"""
from __future__ import annotations

import ctypes
import itertools
import os
from dataclasses import dataclass, field
from typing import List, Optional

import torch
import torch.nn as nn

from .. import native
from ..native import LinearBwdArgs, LinearFwdArgs, call, ptr
from ..profiling import TIMER

ACT_CODE = {nn.ReLU: 0, nn.GELU: 1, nn.LeakyReLU: 2, nn.Tanh: 3, nn.Sigmoid: 4}
ACT_NONE = 5

_seed_counter = itertools.count(1)


def act_code(mod: Optional[nn.Module]) -> int:
    if mod is None:
        return ACT_NONE
    for cls, code in ACT_CODE.items():
        if isinstance(mod, cls):
            if cls is nn.LeakyReLU and abs(mod.negative_slope - 0.1) > 1e-12:
                raise NotImplementedError("LeakyReLU slope other than 0.1 (two_tower.py:82)")
            return code
    raise NotImplementedError(f"activation {type(mod).__name__}")


@dataclass
class Block:
    """One Linear plus the (optional) act/BN/dropout that FOLLOW it."""
    linear: nn.Linear
    act: int = ACT_NONE
    bn: Optional[nn.BatchNorm1d] = None
    drop: Optional[nn.Dropout] = None

    def drop_p(self) -> float:
        return float(self.drop.p) if (self.drop is not None and self.drop.training and self.drop.p > 0) else 0.0

    def bn_mode(self) -> int:
        """prologue/grad mode of this block's BN for the consumer: 1 train, 2 eval, 3 none."""
        if self.bn is None:
            return 3
        return 1 if self.bn.training else 2


def blocks_from_sequential(seq: nn.Sequential) -> List[Block]:
    """[Linear, act, BN, Dropout]*L + Linear (two_tower.py:60-70) or the content
    projection Linear, ReLU, Dropout, Linear (:185-190)."""
    mods = list(seq)
    blocks: List[Block] = []
    i = 0
    while i < len(mods):
        lin = mods[i]
        if not isinstance(lin, nn.Linear):
            raise NotImplementedError(f"unexpected module {type(lin).__name__} at {i}")
        b = Block(lin)
        i += 1
        if i < len(mods) and not isinstance(mods[i], (nn.Linear, nn.BatchNorm1d, nn.Dropout)):
            b.act = act_code(mods[i])
            i += 1
        if i < len(mods) and isinstance(mods[i], nn.BatchNorm1d):
            b.bn = mods[i]
            i += 1
        if i < len(mods) and isinstance(mods[i], nn.Dropout):
            b.drop = mods[i]
            i += 1
        blocks.append(b)
    return blocks


# ---------------------------------------------------------------------------
# parameter slab
# ---------------------------------------------------------------------------
class ParamSlab:
    """All parameters of a module in ONE contiguous fp32 device buffer (plus a
    grad slab). Params become views (``p.data``), and ``p.grad`` is pinned to the
    grad-slab view whenever the kernels need it."""

    def __init__(self, module: nn.Module):
        self.module = module
        self.params: List[nn.Parameter] = []
        self.data: Optional[torch.Tensor] = None
        self.grad: Optional[torch.Tensor] = None
        self.offsets: List[int] = []
        self.offsets_dev: Optional[torch.Tensor] = None
        # bumped whenever something outside the fused step may have written the
        # grad slab (autograd backward through attach_grads, a slab rebuild);
        # FusedTrainStep re-zeroes the slab before its next step when it changes
        self.grad_gen = 0

    def _valid(self) -> bool:
        ps = [p for p in self.module.parameters()]
        if self.data is None or len(ps) != len(self.params) or any(a is not b for a, b in zip(ps, self.params)):
            return False
        base = self.data.data_ptr()
        for p, off in zip(self.params, self.offsets):
            if p.device != self.data.device or p.data_ptr() != base + off * 4:
                return False
        return True

    def ensure(self) -> "ParamSlab":
        if self._valid():
            return self
        ps = list(self.module.parameters())
        if not ps:
            raise ValueError("module has no parameters")
        dev = ps[0].device
        for p in ps:
            if p.dtype != torch.float32 or p.device != dev:
                raise TypeError("parameter slab needs fp32 parameters on one device")
        sizes = [p.numel() for p in ps]
        # 16-byte aligned starts (vector loads in the kernels)
        offs, cur = [], 0
        for s in sizes:
            offs.append(cur)
            cur += (s + 3) // 4 * 4
        data = torch.zeros(cur, dtype=torch.float32, device=dev)
        grad = torch.zeros(cur, dtype=torch.float32, device=dev)
        with torch.no_grad():
            for p, o, s in zip(ps, offs, sizes):
                data[o:o + s].copy_(p.data.reshape(-1))
        for p, o, s in zip(ps, offs, sizes):
            p.data = data[o:o + s].view(p.shape)
            old = p.grad
            p.grad = grad[o:o + s].view(p.shape)
            if old is not None:
                p.grad.copy_(old)
        self.params, self.offsets, self.data, self.grad = ps, offs, data, grad
        self.grad_gen += 1
        self.__dict__["_grad_views"] = {}
        ends = [o + s for o, s in zip(offs, sizes)]
        self.bounds = list(zip(offs, ends))
        self.offsets_dev = None
        return self

    def attach_grads(self):
        """Make every param's .grad the slab view again (after zero_grad(set_to_none)).
        Called by every autograd backward that accumulates into the slab."""
        self.ensure()
        self.grad_gen += 1
        for p, (o, e) in zip(self.params, self.bounds):
            view = self.grad[o:e]
            if p.grad is None:
                view.zero_()
                p.grad = view.view(p.shape)
            elif p.grad.data_ptr() != view.data_ptr():
                view.copy_(p.grad.reshape(-1))
                p.grad = view.view(p.shape)

    def grad_of(self, p: torch.Tensor) -> torch.Tensor:
        cache = self.__dict__.setdefault("_grad_views", {})
        v = cache.get(id(p))
        if v is not None and v[0] is p and v[1].data_ptr() >= self.grad.data_ptr():
            return v[1]
        for q, (o, e) in zip(self.params, self.bounds):
            if q is p:
                view = self.grad[o:e].view(p.shape)
                cache[id(p)] = (p, view)
                return view
        raise KeyError("parameter not in slab")

    def tensor_offsets(self) -> torch.Tensor:
        """Device int64 [n+1] boundaries (per-tensor grad norms; the alignment
        padding between tensors is zero in both slabs)."""
        if self.offsets_dev is None:
            b = [o for o, _ in self.bounds] + [self.bounds[-1][1]]
            self.offsets_dev = torch.tensor(b, dtype=torch.int64, device=self.data.device)
        return self.offsets_dev


# ---------------------------------------------------------------------------
# chain executor
# ---------------------------------------------------------------------------
@dataclass
class ChainCtx:
    m: int
    src: torch.Tensor
    ids: Optional[torch.Tensor]
    zs: List[Optional[torch.Tensor]] = field(default_factory=list)
    save_mean: List[Optional[torch.Tensor]] = field(default_factory=list)
    save_invstd: List[Optional[torch.Tensor]] = field(default_factory=list)
    seeds: List[int] = field(default_factory=list)
    drop_ps: List[float] = field(default_factory=list)
    bn_modes: List[int] = field(default_factory=list)
    out: Optional[torch.Tensor] = None
    norms: Optional[torch.Tensor] = None
    normalize: bool = True
    seg_split: int = 0  # > 0: rows [0, seg_split) and [seg_split, m) are separate BN batches
    wts: List[Optional[torch.Tensor]] = field(default_factory=list)  # Wᵀ of each Linear (fwd writes, dz reads)
    # split pieces of each Linear's W ([3][n][k] bf16: the previous launch writes, the
    # Linear's own forward reads) and of its Wᵀ ([3][k][n]: the forward writes, dz reads)
    w_planes: List[Optional[torch.Tensor]] = field(default_factory=list)
    wt_planes: List[Optional[torch.Tensor]] = field(default_factory=list)
    ains: List[Optional[torch.Tensor]] = field(default_factory=list)  # transformed inputs (fwd writes, dW reads)


def _stream(t: torch.Tensor):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


# BN sums are [slots][2][width] fp64 (include/rtrec_hip.h RT_STAT_SLOTS, 8 in
# this build); the arenas are sized for 16, an upper bound of every library
# variant's slot count, so a variant build never writes past them
STAT_SLOTS = 16
# dbias slots are [RT_STAT_SLOTS + 1][n]: row RT_STAT_SLOTS holds the fused-dz dW
# launch's per-tile tickets, so a region of STAT_SLOTS + 1 rows covers every variant
DBIAS_ROWS = STAT_SLOTS + 1
# BatchNorm batch statistics finalised once by the producing forward launch
# (rt_linear_fwd_args.fin_*: its last block, found by a ticket) instead of by
# every block of the consuming launch. Off by default: the consumer's slot
# reads overlap its A-tile loads, while the producer's ticket and serial tail
# cost more — C2 step 0.2392 -> 0.2505 ms in a same-box A/B
# (profiles/r05_c2_ab_bn_final.txt). RTREC_BN_FINAL=1 turns it on.
FINALIZE_BN_IN_PRODUCER = os.environ.get("RTREC_BN_FINAL", "0") == "1"
# Split-weight planes (DESIGN.md §5 note i): each weight's three bf16 pieces are
# written once per chain by a side task of the launch before the one that uses
# them (rt_linear_fwd_args.next_w_planes for the forward's k-loop, wt_planes_out
# for the dz launch's dA) instead of being split in registers by every block.
# Bit-identical either way (tests/test_gpu_wplanes.py). Off by default: the
# k-loops are bound by their W fragment loads, not by the split VALU, and three
# 16-byte piece loads per k-block cost more than two float4 loads plus the split
# — C2 step 0.2428 -> 0.2563 ms in a same-box A/B (profiles/r06_c2_ab_wplanes.txt).
# RTREC_W_PLANES=1 turns it on.
# RTREC_W_PLANES=fwd / =dz enable one side only (A/B).
_WPL = os.environ.get("RTREC_W_PLANES", "0")
SPLIT_W_PLANES = _WPL in ("1", "fwd", "dz")
SPLIT_W_PLANES_FWD = _WPL in ("1", "fwd")
SPLIT_W_PLANES_DZ = _WPL in ("1", "dz")


def stats_arena_size(blocks: List[Block], n_seg: int = 1) -> int:
    """fp64 words of BN column sums one forward (or backward) of the chain needs,
    plus the dbias slots of every Linear ([DBIAS_ROWS][n], backward)."""
    return max(1, n_seg * STAT_SLOTS * 2 * sum(b.linear.out_features for b in blocks[:-1])
               + DBIAS_ROWS * sum(b.linear.out_features for b in blocks))


def _zero_on_entry(layer, zero_buf: Optional[torch.Tensor]):
    """The launch clears ``zero_buf`` (fp64) before its own work (rt_linear_fwd_args.zero_buf)."""
    if zero_buf is not None:
        layer.zero_buf = zero_buf.data_ptr()
        layer.zero_words = zero_buf.numel()


def chain_forward(blocks: List[Block], src: torch.Tensor, ids: Optional[torch.Tensor] = None,
                  normalize: bool = True, seed_offset: Optional[torch.Tensor] = None,
                  stats_arena: Optional[torch.Tensor] = None, seg_split: int = 0,
                  zero_buf: Optional[torch.Tensor] = None, seed_base: Optional[int] = None) -> ChainCtx:
    """Run the block chain (see ``_forward_plan`` for the arguments)."""
    ctx, layers = _forward_plan(blocks, src, ids, normalize, seed_offset, stats_arena, seg_split, seed_base)
    _zero_on_entry(layers[0], zero_buf)
    st = _stream(src)
    for a in layers:
        _launch_fwd([a], st)
    return ctx


def chain_forward_pair(first: tuple, second: tuple, zero_buf: Optional[torch.Tensor] = None) -> tuple:
    """Two independent chains (e.g. the item and the user tower), each given as
    the ``chain_forward`` positional arguments; layer l of both runs as ONE
    launch (``rt_linear_fwd_f32_multi``) when the chains have the same depth.
    ``zero_buf`` is cleared by the first launch. Returns the two ChainCtx."""
    c1, l1 = _forward_plan(*first)
    c2, l2 = _forward_plan(*second)
    _zero_on_entry(l1[0], zero_buf)
    st = _stream(first[1])
    if len(l1) == len(l2):
        for a, b in zip(l1, l2):
            _launch_fwd([a, b], st)
    else:
        for a in l1 + l2:
            _launch_fwd([a], st)
    return c1, c2


def _launch_fwd(group: list, st) -> None:
    flops = sum(2.0 * a.m * a.k * a.n for a in group)
    nbytes = sum(4.0 * (a.m * a.k + a.n * a.k + a.m * a.n) for a in group)
    with TIMER.region("linear_fwd", flops=flops, bytes_=nbytes):
        if len(group) == 1:
            call("rt_linear_fwd_f32", ctypes.byref(group[0]), st)
        else:
            arr = (LinearFwdArgs * len(group))(*group)
            call("rt_linear_fwd_f32_multi", arr, len(group), st)


def layer_seed(seed_base: int, layer: int) -> int:
    """Dropout seed of one layer of a chain with a fixed ``seed_base``
    (splitmix64 of the pair): the kernel adds the device step counter
    (``seed_offset``), so the masks change every step while an eager step and
    a graph replay of the same step draw the same masks."""
    z = (seed_base * 0x100000001B3 + (layer + 1) * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return z ^ (z >> 31)


def _forward_plan(blocks: List[Block], src: torch.Tensor, ids: Optional[torch.Tensor] = None,
                  normalize: bool = True, seed_offset: Optional[torch.Tensor] = None,
                  stats_arena: Optional[torch.Tensor] = None, seg_split: int = 0,
                  seed_base: Optional[int] = None):
    """Allocate the chain's activations and build its per-layer launch
    arguments (launched by the callers above). ``src`` is the dense input [rows, k0] (fp32) or a
    feature table when ``ids`` selects its rows (fused gather). ``seg_split`` > 0
    runs two tower calls in one chain: rows [0, seg_split) and [seg_split, m)
    are separate BatchNorm batches (running stats updated in that order).
    ``seed_base``: fixed per-layer dropout seeds (``layer_seed``) instead of a
    fresh host seed per call."""
    native.require_device(src, what="tower forward")
    if src.dtype != torch.float32:
        raise TypeError("tower input must be fp32 (the reference towers are fp32)")
    src = src.contiguous()
    m = int(ids.numel()) if ids is not None else int(src.shape[0])
    if ids is not None:
        ids = ids.contiguous().to(torch.int64)
    dev = src.device
    L = len(blocks) - 1
    k0 = blocks[0].linear.in_features
    if src.dim() != 2 or src.shape[1] != k0:
        # what F.linear raises for the same mismatch
        raise RuntimeError(f"mat1 and mat2 shapes cannot be multiplied ({m}x{src.shape[-1]} and "
                           f"{k0}x{blocks[0].linear.out_features})")
    n_seg = 2 if seg_split else 1
    if seg_split and (seg_split % 32 != 0 or not 0 < seg_split < m):
        raise ValueError("seg_split must be a multiple of 32 inside (0, m)")
    seg_rows = [seg_split, m - seg_split] if seg_split else [m]
    for b in blocks[:-1]:
        if b.bn is not None and b.bn.training and min(seg_rows) <= 1:
            raise ValueError("Expected more than 1 value per channel when training (BatchNorm1d)")
    ctx = ChainCtx(m=m, src=src, ids=ids, normalize=normalize, seg_split=seg_split)
    # one fp64 arena for all BN column sums of this call
    widths = [b.linear.out_features for b in blocks[:-1]]
    if stats_arena is None:  # caller-provided arenas are zeroed by the caller (one memset per step)
        stats_arena = torch.zeros(stats_arena_size(blocks, n_seg), dtype=torch.float64, device=dev)
    stats, off = [], 0
    for wdt in widths:
        stats.append(stats_arena[off:off + n_seg * STAT_SLOTS * 2 * wdt])
        off += n_seg * STAT_SLOTS * 2 * wdt
    layers = []
    cur_src, cur_ids, ld = src, ids, src.shape[1]
    for li, b in enumerate(blocks):
        lin = b.linear
        a = LinearFwdArgs()
        a.src = cur_src.data_ptr()
        a.src_rows = cur_src.shape[0]
        a.ld_src = ld
        a.ids = cur_ids.data_ptr() if cur_ids is not None else None
        a.m = m
        a.k = lin.in_features
        a.n = lin.out_features
        a.w = lin.weight.data_ptr()
        a.bias = lin.bias.data_ptr() if lin.bias is not None else None
        a.seed_offset = seed_offset.data_ptr() if seed_offset is not None else None
        a.seg_split = seg_split
        if li == 0:
            a.prev_mode = 0
        else:
            pb = blocks[li - 1]
            a.prev_mode = pb.bn_mode()
            a.prev_act = pb.act
            a.drop_p = pb.drop_p()
            a.drop_seed = ctx.seeds[li - 1]
            if pb.bn is not None:
                a.prev_stats = stats[li - 1].data_ptr()
                a.bn_gamma = pb.bn.weight.data_ptr()
                a.bn_beta = pb.bn.bias.data_ptr()
                a.running_mean = pb.bn.running_mean.data_ptr()
                a.running_var = pb.bn.running_var.data_ptr()
                sm = torch.empty(n_seg * lin.in_features, dtype=torch.float32, device=dev)
                si = torch.empty(n_seg * lin.in_features, dtype=torch.float32, device=dev)
                ctx.save_mean[li - 1], ctx.save_invstd[li - 1] = sm, si
                a.save_mean = sm.data_ptr()
                a.save_invstd = si.data_ptr()
                a.bn_eps = float(pb.bn.eps)
                a.bn_momentum = float(pb.bn.momentum if pb.bn.momentum is not None else 0.1)
                if pb.bn.training and pb.bn.num_batches_tracked is not None:
                    a.num_batches_tracked = pb.bn.num_batches_tracked.data_ptr()  # +1 in-kernel
                prod = layers[li - 1]
                if a.prev_mode == 1 and prod.stats_out and FINALIZE_BN_IN_PRODUCER:
                    # the producing launch's last block derives mean / invstd and the
                    # running-stat updates once (rt_linear_fwd_args.fin_*); this launch
                    # reads them (prev_final)
                    prod.fin_save_mean, prod.fin_save_invstd = a.save_mean, a.save_invstd
                    prod.fin_running_mean, prod.fin_running_var = a.running_mean, a.running_var
                    prod.fin_num_batches_tracked = a.num_batches_tracked
                    prod.fin_eps, prod.fin_momentum = a.bn_eps, a.bn_momentum
                    a.prev_final = 1
        a.act = b.act
        # Wᵀ of this Linear for its backward's dA (layers past the first: their
        # dz launch computes the previous block's gradient); training forwards
        # only — eval / serving forwards have no backward to read it. With
        # SPLIT_W_PLANES the forward writes Wᵀ's split pieces instead (n % 8 == 0).
        wt = wtp = None
        if li > 0 and lin.training:
            if SPLIT_W_PLANES and SPLIT_W_PLANES_DZ and lin.out_features % 8 == 0:
                wtp = torch.empty((3, lin.in_features, lin.out_features), dtype=torch.int16, device=dev)
                a.wt_planes_out = wtp.data_ptr()
            else:
                wt = torch.empty((lin.in_features, lin.out_features), dtype=torch.float32, device=dev)
                a.wt_out = wt.data_ptr()
        ctx.wts.append(wt)
        ctx.wt_planes.append(wtp)
        # W's split pieces for this launch's k-loop, written by the previous
        # launch of the chain (layers past the first; k % 8 == 0, n <= 128)
        wp = None
        if SPLIT_W_PLANES and SPLIT_W_PLANES_FWD and li > 0 and lin.in_features % 8 == 0 and lin.out_features <= 128:
            wp = torch.empty((3, lin.out_features, lin.in_features), dtype=torch.int16, device=dev)
            prev = layers[li - 1]
            prev.next_w = lin.weight.data_ptr()
            prev.next_w_planes = wp.data_ptr()
            prev.next_n, prev.next_k = lin.out_features, lin.in_features
            a.w_planes = wp.data_ptr()
        ctx.w_planes.append(wp)
        # training: the launch also writes the transformed input it stages (act →
        # BN → dropout of the previous block), which this Linear's dW launch then
        # reads as is instead of recomputing it (rt_linear_fwd_args.a_out / a_in)
        ain = None
        if li > 0 and lin.training and lin.in_features % 4 == 0:
            ain = torch.empty((m, lin.in_features), dtype=torch.float32, device=dev)
            a.a_out = ain.data_ptr()
        ctx.ains.append(ain)
        if li < L:
            z = torch.empty((m, lin.out_features), dtype=torch.float32, device=dev)
            a.z_out = z.data_ptr()
            if b.bn is not None and b.bn.training:
                a.stats_out = stats[li].data_ptr()
            ctx.zs.append(z)
            ctx.save_mean.append(None)
            ctx.save_invstd.append(None)
            ctx.seeds.append(layer_seed(seed_base, li) if seed_base is not None else
                             next(_seed_counter) * 0x9E3779B97F4A7C15 & 0xFFFFFFFFFFFFFFFF)
            ctx.drop_ps.append(b.drop_p())
            ctx.bn_modes.append(b.bn_mode())
            cur_src, cur_ids, ld = z, None, lin.out_features
        else:
            out = torch.empty((m, lin.out_features), dtype=torch.float32, device=dev)
            if normalize:
                norms = torch.empty(m, dtype=torch.float32, device=dev)
                a.l2_out = out.data_ptr()
                a.norms_out = norms.data_ptr()
                ctx.norms = norms
            else:
                a.z_out = out.data_ptr()
            ctx.out = out
        layers.append(a)
    return ctx, layers


def chain_backward(blocks: List[Block], ctx: ChainCtx, dout: torch.Tensor, slab: ParamSlab,
                   want_dsrc: bool = False, seed_offset: Optional[torch.Tensor] = None,
                   stats_arena: Optional[torch.Tensor] = None, attach: bool = True) -> Optional[torch.Tensor]:
    """Backward through the chain; parameter grads are atomically accumulated
    into the slab. Returns d src (dense input) when ``want_dsrc``."""
    layers, dsrc, keep = _backward_plan(blocks, ctx, dout, slab, want_dsrc, seed_offset, stats_arena, attach)
    st = _stream(dout)
    groups = [[a] for a in layers]
    keep += _plan_partials(groups, dout.device)
    for g in groups:  # per Linear: dz (+dA) then dW (+dbias), timed separately (bench roofline)
        _launch_bwd(g, st)
    return dsrc


def chain_backward_pair(first: tuple, second: tuple) -> None:
    """Backward of two independent chains (``chain_backward`` positional
    arguments each, no dsrc); layer l of both runs as ONE dz launch and ONE dW
    launch (``rt_linear_bwd_*_f32_multi``) when the depths match."""
    # keep1/keep2 hold the planned buffers until every launch is enqueued
    l1, _, keep1 = _backward_plan(*first)
    l2, _, keep2 = _backward_plan(*second)
    st = _stream(first[2])
    if len(l1) == len(l2):
        groups = [[a, b] for a, b in zip(l1, l2)]
        keep1 += _plan_partials(groups, first[2].device)
    else:
        groups = [[a] for a in l1 + l2]
    for g in groups:
        _launch_bwd(g, st)


def _plan_partials(groups: list, dev) -> list:
    """Launch groups in execution order: every dW launch but the last STORES its
    row-split tile sums (rt_linear_bwd_args.dw_part) instead of adding them
    with fp32 atomics, and the next group's first launch (its dz, or its dW
    when that layer's dz is fused) folds them into the gradient (fold_*): the
    atomics were bound by their bytes (≈ 11 MB per C2 step at ≈ 1.3 TB/s).
    Returns the partial buffers (kept alive by the caller)."""
    lib = native.lib()
    if not hasattr(lib, "rt_linear_bwd_dw_splits"):
        return []
    keep = []
    for gi in range(len(groups) - 1):
        grp, nxt = groups[gi], groups[gi + 1]
        if len(grp) != len(nxt):
            continue
        arr = (LinearBwdArgs * len(grp))(*grp)
        splits = (ctypes.c_int64 * len(grp))()
        if lib.rt_linear_bwd_dw_splits(arr, len(grp), splits) != 0:
            continue
        narr = (LinearBwdArgs * len(nxt))(*nxt)
        fold_in = 1 if lib.rt_linear_bwd_dz_fused(narr, len(nxt)) else 0
        for a, b, sp in zip(grp, nxt, splits):
            words = a.n * a.k
            if sp < 1 or words % 4 or b.fold_src:
                continue
            part = torch.empty(sp * words, dtype=torch.float32, device=dev)
            keep.append(part)
            a.dw_part = part.data_ptr()
            b.fold_src, b.fold_dst, b.fold_words = part.data_ptr(), a.dw, words
            b.fold_splits, b.fold_in = sp, fold_in
    return keep


def _launch_bwd(group: list, st) -> None:
    da = [a.g_prev is not None or a.dsrc is not None for a in group]
    flops = sum((2.0 if d else 0.0) * a.m * a.k * a.n for a, d in zip(group, da))
    nbytes = sum(4.0 * (3 * a.m * a.n + (2 * a.m * a.k if d else 0) + a.n * a.k) for a, d in zip(group, da))
    arr = (LinearBwdArgs * len(group))(*group)
    lib = native.lib()
    fused = hasattr(lib, "rt_linear_bwd_dz_fused") and lib.rt_linear_bwd_dz_fused(arr, len(group))
    if not fused:  # else the dW launch computes dz (older library builds: always the dz launch)
        with TIMER.region("linear_bwd_dz", flops=flops, bytes_=nbytes):
            call("rt_linear_bwd_dz_f32_multi", arr, len(group), st)
    with TIMER.region("linear_bwd_dw", flops=sum(2.0 * a.m * a.k * a.n for a in group),
                      bytes_=sum(4.0 * (a.m * a.n + a.m * a.k + a.n * a.k) for a in group)):
        call("rt_linear_bwd_dw_f32_multi", arr, len(group), st)


def _backward_plan(blocks: List[Block], ctx: ChainCtx, dout: torch.Tensor, slab: ParamSlab,
                   want_dsrc: bool = False, seed_offset: Optional[torch.Tensor] = None,
                   stats_arena: Optional[torch.Tensor] = None, attach: bool = True):
    """Per-Linear backward launch arguments, last layer first, the d src buffer
    (or None), and the buffers allocated here (the caller keeps them alive until
    the launches are enqueued, so no later allocation can reuse them early)."""
    dev = dout.device
    dout = dout.contiguous()
    m = ctx.m
    L = len(blocks) - 1
    if attach:
        slab.attach_grads()
    # one dz buffer per layer (no write-after-read ordering between layer l's dW
    # and layer l-1's dz; 0.3 % of the C2 step in a same-box A/B)
    dz_bufs = [torch.empty((m, b.linear.out_features), dtype=torch.float32, device=dev) for b in blocks]
    layers = []
    widths = [b.linear.out_features for b in blocks[:-1]]
    n_seg = 2 if ctx.seg_split else 1
    gst_arena = stats_arena if stats_arena is not None else \
        torch.zeros(stats_arena_size(blocks, n_seg), dtype=torch.float64, device=dev)
    gstats, off = [], 0
    for wdt in widths:
        gstats.append(gst_arena[off:off + n_seg * STAT_SLOTS * 2 * wdt])
        off += n_seg * STAT_SLOTS * 2 * wdt
    bslots = []  # dbias slots of Linear li (both BN segments add into the same slots)
    for b in blocks:
        bslots.append(gst_arena[off:off + DBIAS_ROWS * b.linear.out_features])
        off += DBIAS_ROWS * b.linear.out_features
    gs: List[Optional[torch.Tensor]] = [None] * L
    dsrc = torch.empty((m, blocks[0].linear.in_features), dtype=torch.float32, device=dev) if want_dsrc else None
    keep = [dout, gst_arena] + dz_bufs
    for li in range(L, -1, -1):
        b = blocks[li]
        lin = b.linear
        a = LinearBwdArgs()
        a.m, a.k, a.n = m, lin.in_features, lin.out_features
        a.w = lin.weight.data_ptr()
        a.dw = slab.grad_of(lin.weight).data_ptr()
        a.dbias = slab.grad_of(lin.bias).data_ptr() if lin.bias is not None else None
        a.dbias_slots = bslots[li].data_ptr() if lin.bias is not None else None
        a.dz_ws = dz_bufs[li].data_ptr()
        a.seed_offset = seed_offset.data_ptr() if seed_offset is not None else None
        a.seg_split = ctx.seg_split
        if li == L:
            if ctx.normalize:
                a.grad_mode = 0
                a.dout = dout.data_ptr()
                a.l2_out = ctx.out.data_ptr()
                a.norms = ctx.norms.data_ptr()
            else:
                a.grad_mode = 3
                a.g = dout.data_ptr()
                a.z = dout.data_ptr()
                a.act = ACT_NONE
        else:
            a.grad_mode = ctx.bn_modes[li]
            a.g = gs[li].data_ptr()
            a.z = ctx.zs[li].data_ptr()
            a.act = b.act
            if b.bn is not None:
                a.g_stats = gstats[li].data_ptr()
                a.save_mean = ctx.save_mean[li].data_ptr()
                a.save_invstd = ctx.save_invstd[li].data_ptr()
                a.bn_gamma = b.bn.weight.data_ptr()
                a.dgamma = slab.grad_of(b.bn.weight).data_ptr()
                a.dbeta = slab.grad_of(b.bn.bias).data_ptr()
        # input of this linear (recomputed by the same prologue as forward)
        if li == 0 and not want_dsrc:
            a.fuse_dz = 1  # no dA: the dW launch computes dz (the dz launch becomes a no-op)
        if li == 0:
            a.src = ctx.src.data_ptr()
            a.src_rows = ctx.src.shape[0]
            a.ld_src = ctx.src.shape[1]
            a.ids = ctx.ids.data_ptr() if ctx.ids is not None else None
            a.prev_mode = 0
            if want_dsrc:
                if ctx.ids is not None:
                    raise NotImplementedError("input gradient through a fused gather")
                a.dsrc = dsrc.data_ptr()
        else:
            pb = blocks[li - 1]
            a.src = ctx.zs[li - 1].data_ptr()
            a.src_rows = m
            a.ld_src = pb.linear.out_features
            a.prev_mode = ctx.bn_modes[li - 1]
            a.prev_act = pb.act
            a.prev_drop_p = ctx.drop_ps[li - 1]
            a.prev_drop_seed = ctx.seeds[li - 1]
            if pb.bn is not None:
                a.prev_mean = ctx.save_mean[li - 1].data_ptr()
                a.prev_invstd = ctx.save_invstd[li - 1].data_ptr()
                a.prev_gamma = pb.bn.weight.data_ptr()
                a.prev_beta = pb.bn.bias.data_ptr()
                a.g_prev_stats = gstats[li - 1].data_ptr()
            g = torch.empty((m, pb.linear.out_features), dtype=torch.float32, device=dev)
            gs[li - 1] = g
            keep.append(g)
            a.g_prev = g.data_ptr()
            if li < len(ctx.wts) and ctx.wts[li] is not None:
                a.wt = ctx.wts[li].data_ptr()
            if li < len(ctx.wt_planes) and ctx.wt_planes[li] is not None:
                a.wt_planes = ctx.wt_planes[li].data_ptr()
            if li < len(ctx.ains) and ctx.ains[li] is not None:
                a.a_in = ctx.ains[li].data_ptr()
        layers.append(a)
    return layers, dsrc, keep
