"""ctypes binding of librtrec_hip.so (the C ABI declared in include/rtrec_hip.h).

The library is built in-tree by ``make -C real-time-recommendation-system-with-feature-store_amd``
(``__graft_entry__.build()``). There is no fallback: if the library is missing
or fails to load, every compute entry point raises :class:`NativeUnavailable`.
``torch`` is imported first so the HIP runtime torch ships is the one the
library binds to (both carry the soname ``libamdhip64.so.7``).
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

import torch  # noqa: F401  (must precede the CDLL: shared HIP runtime)

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("RTREC_HIP_LIB", os.path.join(PKG_DIR, "lib", "librtrec_hip.so"))

RT_F32, RT_F16, RT_BF16 = 0, 1, 2
ACTS = {"relu": 0, "gelu": 1, "leaky_relu": 2, "tanh": 3, "sigmoid": 4, "none": 5}

c_i64 = ctypes.c_int64
c_int = ctypes.c_int
c_f32 = ctypes.c_float
c_u64 = ctypes.c_uint64
c_size = ctypes.c_size_t
vp = ctypes.c_void_p


class NativeUnavailable(RuntimeError):
    """librtrec_hip.so is missing or unusable (no CPU fallback exists)."""


class RTError(RuntimeError):
    """A C-ABI call returned a non-zero rt_status."""

    def __init__(self, what: str, status: int, message: str):
        super().__init__(f"{what} failed: {message} (status {status})")
        self.status = status


class LinearFwdArgs(ctypes.Structure):
    _fields_ = [
        ("src", vp), ("src_rows", c_i64), ("ld_src", c_int), ("ids", vp), ("m", c_i64), ("k", c_int),
        ("n", c_int), ("w", vp), ("bias", vp),
        ("prev_mode", c_int), ("prev_act", c_int), ("prev_stats", vp), ("bn_gamma", vp), ("bn_beta", vp),
        ("running_mean", vp), ("running_var", vp), ("save_mean", vp), ("save_invstd", vp),
        ("bn_eps", c_f32), ("bn_momentum", c_f32), ("drop_p", c_f32), ("drop_seed", c_u64),
        ("seed_offset", vp), ("z_out", vp), ("act", c_int), ("stats_out", vp), ("l2_out", vp), ("norms_out", vp),
        ("num_batches_tracked", vp), ("seg_split", c_i64), ("zero_buf", vp), ("zero_words", c_i64),
        ("wt_out", vp), ("a_out", vp),
        ("fin_save_mean", vp), ("fin_save_invstd", vp), ("fin_running_mean", vp), ("fin_running_var", vp),
        ("fin_num_batches_tracked", vp), ("fin_eps", c_f32), ("fin_momentum", c_f32), ("prev_final", c_int),
        ("w_planes", vp), ("wt_planes_out", vp), ("next_w", vp), ("next_w_planes", vp), ("next_n", c_int),
        ("next_k", c_int),
    ]


class LinearBwdArgs(ctypes.Structure):
    _fields_ = [
        ("m", c_i64), ("k", c_int), ("n", c_int), ("w", vp), ("dw", vp), ("dbias", vp), ("dz_ws", vp),
        ("grad_mode", c_int), ("dout", vp), ("l2_out", vp), ("norms", vp),
        ("g", vp), ("z", vp), ("act", c_int), ("g_stats", vp), ("save_mean", vp), ("save_invstd", vp),
        ("bn_gamma", vp), ("dgamma", vp), ("dbeta", vp),
        ("src", vp), ("src_rows", c_i64), ("ld_src", c_int), ("ids", vp),
        ("prev_mode", c_int), ("prev_act", c_int), ("prev_mean", vp), ("prev_invstd", vp),
        ("prev_gamma", vp), ("prev_beta", vp), ("prev_drop_p", c_f32), ("prev_drop_seed", c_u64),
        ("seed_offset", vp), ("g_prev", vp), ("g_prev_stats", vp), ("dsrc", vp), ("seg_split", c_i64),
        ("dbias_slots", vp), ("wt", vp), ("fuse_dz", c_int), ("a_in", vp), ("dw_part", vp),
        ("fold_src", vp), ("fold_dst", vp), ("fold_words", c_i64), ("fold_splits", c_int), ("fold_in", c_int),
        ("wt_planes", vp),
    ]


# name -> (restype, argtypes); mirrors include/rtrec_hip.h one-to-one
SIGNATURES = {
    "rt_abi_version": (c_int, []),
    "rt_status_string": (ctypes.c_char_p, [c_int]),
    "rt_last_error": (ctypes.c_char_p, []),
    "rt_gather_rows": (c_int, [vp, c_i64, c_i64, c_i64, vp, c_i64, vp, vp, vp]),
    "rt_scatter_add_rows_f32": (c_int, [vp, c_i64, c_int, vp, c_i64, vp, c_i64, vp]),
    "rt_l2_renorm_f32": (c_int, [vp, c_i64, c_int, vp]),
    "rt_flatip_topk_workspace_bytes": (c_size, [c_i64, c_i64, c_int, c_int, c_int]),
    "rt_flatip_topk": (c_int, [vp, c_i64, vp, c_i64, c_int, c_int, c_int, vp, c_i64, c_i64, vp, vp, vp,
                               c_size, vp]),
    "rt_topk_merge": (c_int, [vp, vp, c_i64, c_int, c_int, c_int, vp, vp, vp]),
    "rt_flatip_topk_tuning": (c_int, [c_int, c_int, c_int]),
    "rt_flatip_topk_shard_workspace_bytes": (c_size, [c_i64, c_i64, c_int, c_int, c_int]),
    "rt_flatip_topk_shard_plan": (c_int, [c_i64, c_i64, c_int, c_int, c_int, c_int, vp]),
    "rt_flatip_topk_shard_sample": (c_int, [vp, c_i64, vp, c_i64, c_int, c_int, c_int, c_int, vp, vp, vp, c_size,
                                            vp]),
    "rt_topk_sample_rank": (c_int, [c_int, c_i64, c_i64, vp]),
    "rt_topk_sample_threshold": (c_int, [vp, c_int, c_i64, c_int, vp, vp]),
    "rt_flatip_topk_shard_search": (c_int, [vp, c_i64, vp, c_i64, c_int, c_int, c_int, vp, c_i64, vp, vp, vp,
                                            c_size, vp]),
    "rt_sample_negatives": (c_int, [vp, vp, c_i64, vp, c_i64, c_i64, c_int, c_u64, vp, vp, vp]),
    "rt_feeder_batch": (c_int, [vp, vp, vp, vp, c_i64, vp, vp, vp]),
    "rt_feeder_commit": (c_int, [vp, vp, c_i64, vp, vp]),
    "rt_linear_fwd_f32": (c_int, [ctypes.POINTER(LinearFwdArgs), vp]),
    "rt_linear_bwd_f32": (c_int, [ctypes.POINTER(LinearBwdArgs), vp]),
    "rt_linear_bwd_dz_f32": (c_int, [ctypes.POINTER(LinearBwdArgs), vp]),
    "rt_linear_bwd_dz_fused": (c_int, [ctypes.POINTER(LinearBwdArgs), c_int]),
    "rt_linear_bwd_dw_splits": (c_int, [ctypes.POINTER(LinearBwdArgs), c_int, ctypes.POINTER(c_i64)]),
    "rt_linear_bwd_dw_f32": (c_int, [ctypes.POINTER(LinearBwdArgs), vp]),
    "rt_linear_fwd_f32_multi": (c_int, [ctypes.POINTER(LinearFwdArgs), c_int, vp]),
    "rt_linear_bwd_dz_f32_multi": (c_int, [ctypes.POINTER(LinearBwdArgs), c_int, vp]),
    "rt_linear_bwd_dw_f32_multi": (c_int, [ctypes.POINTER(LinearBwdArgs), c_int, vp]),
    "rt_twotower_loss_workspace_bytes": (c_size, [c_i64, c_int]),
    "rt_twotower_loss_fwd_bwd": (c_int, [vp, vp, vp, c_int, c_i64, c_int, c_int, c_f32, vp, vp, c_f32,
                                         c_f32, vp, vp, vp, vp, vp, vp, vp, c_size, vp]),
    "rt_twotower_loss_fwd": (c_int, [vp, vp, vp, c_int, c_i64, c_int, c_int, c_f32, vp, vp, c_f32, c_f32,
                                     vp, vp, c_size, vp]),
    "rt_inbatch_loss_workspace_bytes": (c_size, [c_i64, c_i64, c_int]),
    "rt_inbatch_loss_fwd_bwd": (c_int, [vp, vp, c_int, c_i64, c_i64, c_int, c_i64, c_f32, vp, vp, vp, vp, c_size, vp]),
    "rt_similarity_f32": (c_int, [vp, vp, c_i64, c_int, c_f32, vp, vp, vp, vp]),
    "rt_grad_sqnorm": (c_int, [vp, vp, c_int, vp, vp, vp, vp]),
    "rt_clip_adam_step": (c_int, [vp, vp, vp, vp, c_i64, vp, c_int, c_f32, c_f32, vp, c_f32, c_f32, c_f32,
                                  c_f32, c_int, vp, vp, c_i64, vp]),
    "rt_l2_augment_f32": (c_int, [vp, c_i64, c_int, vp, c_int, c_int, vp]),
    "rt_l2_finish_f32": (c_int, [vp, c_int, vp, c_int, c_int, c_i64, c_int, vp, vp, c_int, vp, vp, vp, c_i64, vp]),
    "rt_exclusion_bitmap": (c_int, [vp, vp, c_i64, vp, c_i64, c_i64, vp, c_i64, vp]),
    "rt_rank_metrics": (c_int, [vp, c_i64, c_int, vp, vp, vp, c_i64, vp, vp, vp, c_i64, vp, c_int, c_i64, vp, vp,
                                vp, vp]),
    "rt_rank_metrics_reduce": (c_int, [vp, vp, c_i64, c_int, vp, c_i64, vp, vp]),
}

RT_METRICS_MAX_K = 16

_lib = None
_lock = threading.Lock()
_load_error: Optional[str] = None
MISSING: list = []  # ABI symbols the loaded library does not export


def lib():
    """Load (once) and return the CDLL; raise NativeUnavailable otherwise."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            _load_error = (f"{LIB_PATH} not found — build it with "
                           f"`make -C {PKG_DIR}` (or __graft_entry__.build())")
            raise NativeUnavailable(_load_error)
        try:
            handle = ctypes.CDLL(LIB_PATH)
        except OSError as e:  # pragma: no cover - depends on the box
            _load_error = f"cannot load {LIB_PATH}: {e}"
            raise NativeUnavailable(_load_error) from e
        for name, (res, args) in SIGNATURES.items():
            if not hasattr(handle, name):
                MISSING.append(name)
                continue
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
        return _lib


def available() -> bool:
    try:
        lib()
        return True
    except NativeUnavailable:
        return False


def call(name: str, *args) -> int:
    """Invoke an rt_* entry point and raise RTError on a non-zero status."""
    fn = getattr(lib(), name)
    rc = fn(*args)
    if rc != 0:
        msg = lib().rt_status_string(rc).decode()
        last = lib().rt_last_error().decode()
        raise RTError(name, rc, msg + (f" [{last}]" if last else ""))
    return rc


def ptr(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_of(t: torch.Tensor):
    """hipStream_t of torch's current stream on ``t``'s device."""
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def require_device(*tensors: torch.Tensor, what: str = "rtrec kernel"):
    """The HIP path is the only path: CPU tensors are an error, not a fallback."""
    for t in tensors:
        if t is not None and t.device.type != "cuda":
            raise RuntimeError(f"{what}: expected a ROCm (cuda) device tensor, got {t.device}; "
                               "this MI355X build has no CPU fallback")
    lib()


def dtype_code(dt: torch.dtype) -> int:
    if dt == torch.float32:
        return RT_F32
    if dt == torch.float16:
        return RT_F16
    if dt == torch.bfloat16:
        return RT_BF16
    raise TypeError(f"unsupported dtype {dt}")
