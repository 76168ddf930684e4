"""ctypes binding of libfibinet_hip.so (the C-ABI declared in include/fibinet.h).

The library is loaded once; a missing or un-loadable library raises immediately -- there is
no CPU fallback anywhere in the product path.  Every call goes through :func:`call`, which
raises ``RuntimeError`` with ``fbn_last_error()`` on a non-zero return code.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FBN_LIB_PATH") or os.path.join(_HERE, "libfibinet_hip.so")   # override: tuning tools

P = ctypes.c_void_p
I = ctypes.c_int
LL = ctypes.c_longlong
F = ctypes.c_float
D = ctypes.c_double
SZ = ctypes.c_size_t
U = ctypes.c_uint

# name -> (restype, argtypes); the single source of truth mirrored by include/fibinet.h
SIGNATURES = {
    "fbn_version": (I, []),
    "fbn_last_error": (ctypes.c_char_p, []),
    "fbn_device_ok": (I, []),
    "fbn_gemm_workspace_size": (SZ, [I, I, I, I]),
    "fbn_gemm": (I, [P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, I, I, I, F, I, I, I, P, P, SZ, P]),
    "fbn_gemm_split": (I, [P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, F, P, P, SZ, P, I, I, P, I, I, P]),
    "fbn_gemm_bf16out": (I, [P, P, P, I, I, I, I, I, I, I, I, P]),
    "fbn_gemm_bn_bwd_part_supported": (I, [I, I, I, I, I, I, I]),
    "fbn_gemm_bn_bwd_part": (I, [P, P, P, I, I, I, I, I, I, I, I, P, P, P, F, P, P]),
    "fbn_bn_tile_stats": (I, [P, I, I, P, P, P]),
    "fbn_bn_tile_moments": (I, [P, I, I, P, P]),
    "fbn_bn_moments_finalize": (I, [P, D, I, P, P, P, P, F, F, I, P]),
    "fbn_bn_tile_finalize": (I, [P, I, I, D, P, P, P, P, F, F, I, P]),
    "fbn_bn_colpart_size": (SZ, [I, I]),
    "fbn_row_chunks": (I, [I]),
    "fbn_bn_bwd_chunks": (I, [I, I]),
    "fbn_bn_bwd_fused": (I, [P, P, P, P, P, F, P, P, P, P, I, I, D, P, P, P, P, P, P, P, P, P]),
    "fbn_colsum_partial": (I, [P, I, I, I, P, P]),
    "fbn_sum_jobs": (I, [P, I, P]),
    "fbn_sum_jobs2": (I, [P, I, P, I, P]),
    "fbn_gemm_slabs_size": (SZ, [I, I, I]),
    "fbn_gemm_slabs": (I, [P, P, I, I, I, I, I, I, I, P, SZ, P, I, I, P, I, I, P, P]),
    "fbn_gemm_slabs_split": (I, [I, I, I]),
    "fbn_gemm_slabs_group": (I, [P, I, P]),
    "fbn_gemm_slabs_group_split": (I, [I, I, I]),
    "fbn_fields_fwd": (I, [P, P, P, P, P, P, P, F, P, I, P, LL, P, P, P, P, P, I, P, P, P, P, I, I, P, P, P, P, P, I, I, I, I,
                           P]),
    "fbn_fields_fwd_hot": (I, [P, P, P, P, P, P, P, F, P, I, P, LL, P, P, P, P, I, P, P, P, P, I, I, P, P, P, P, P,
                               I, I, I, P, P, I, P]),
    "fbn_hot_rows": (I, [P, P, I, I, LL, P, P, P, I, I, I, P]),
    "fbn_fields_bwd_partials_size": (I, [I, I, I]),
    "fbn_fields_bwd_grid": (I, [I, I]),
    "fbn_fields_bwd": (I, [P, P, P, P, P, P, P, F, P, P, P, I, I, P, P, P, P, P, P, P, P, P, P, P, P, LL, P, P, I, I,
                           I, I, P]),
    "fbn_pairs_fwd": (I, [P, P, P, P, I, I, I, I, I, P]),
    "fbn_pairs_bwd": (I, [P, P, P, P, P, P, P, I, I, I, I, P]),
    "fbn_bn_workspace_size": (SZ, [I, I]),
    "fbn_bn_stats_pass": (I, [P, I, I, P, P, P, P]),
    "fbn_bn_mean": (I, [P, D, I, P, P]),
    "fbn_bn_finalize": (I, [P, P, D, I, P, P, P, P, F, F, I, P]),
    "fbn_bn_stats": (I, [P, I, I, P, P, P, P, F, F, I, P, P]),
    "fbn_bn_eval_params": (I, [P, P, P, P, I, F, P]),
    "fbn_bn_act_fwd": (I, [P, P, I, I, P, P, P, P, F, P, U, P, P, P, P]),
    "fbn_bn_act_head_fwd": (I, [P, P, I, I, P, P, P, P, F, P, U, P, P, P, P, P, P, P, P, P, F, P, F, P]),
    "fbn_bn_bwd_reduce": (I, [P, P, P, P, F, P, P, I, I, P, P, P]),
    "fbn_bn_bwd_apply": (I, [P, P, P, P, F, P, P, P, P, I, I, P, D, P, P, P, P, P, P, P]),
    "fbn_convert_bf16": (I, [P, I, P]),
    "fbn_bn_bwd": (I, [P, P, P, P, F, P, P, P, P, I, I, P, P, P, P, P, P]),
    "fbn_colsum_workspace_size": (SZ, [I, I]),
    "fbn_colsum": (I, [P, I, I, I, P, F, P, P]),
    "fbn_head_fwd": (I, [P, P, P, I, I, P, P, P, P, P, F, P]),
    "fbn_sigmoid_bwd": (I, [P, P, P, I, P]),
    "fbn_outer": (I, [P, P, P, I, I, P]),
    "fbn_sum": (I, [P, I, P, F, P]),
    "fbn_sumsq": (I, [P, LL, P, I, P, P]),
    "fbn_clip_coef": (I, [P, F, P, P, P]),
    "fbn_adam_dense": (I, [P, P, P, P, LL, P, P, P, F, F, F, P, F, P, P, P]),
    "fbn_sparse_fixup": (I, [P, P, P, I, I, LL, I, P, P, P, P, I, I, P]),
    "fbn_sumsq_sparse": (I, [P, P, P, I, I, I, P, P]),
    "fbn_sparse_fixup_dup": (I, [P, I, P, P, P, I, I, P]),
    "fbn_sumsq_sparse_norms": (I, [P, P, P, P, I, I, I, P, P, P, LL, P]),
    "fbn_sparse_fold_fx": (I, [P, P, I, P, P, I, I, P, P]),
    "fbn_adam_table": (I, [P, P, P, LL, I, P, P, P, P, I, P, P, P, F, F, F, I, P]),
    "fbn_adam_touched": (I, [P, P, P, I, P, P, P, P, I, I, P, P, P, F, F, F, P, P]),
    "fbn_adam_catchup": (I, [P, P, P, LL, I, P, I, P, I, I, P, P, P, F, F, F, P, P, P, LL, I, I, P]),
    "fbn_adam_claim_catchup": (I, [P, P, I, I, LL, P, P, P, P, P, P, P, P, LL, I, I, P, P, P, F, F, F, P, P, P, LL, I,
                                   I, P]),
    "fbn_adam_claim_catchup_conv": (I, [P, P, I, I, LL, P, P, P, P, P, P, P, P, LL, I, I, P, P, P, F, F, F, P, P, P,
                                        LL, I, I, P, I, P]),
    "fbn_adam_flush": (I, [P, P, P, LL, I, P, P, P, F, F, F, P, P, P, LL, I, I, P]),
    "fbn_adam_prefetch_rows": (I, [P, I, I, LL, P, P, P, P, I, P, P, P, F, F, F, P, P, P, LL, I, I, P]),
    "fbn_adam_prefetch": (I, [P, P, I, I, LL, P, P, P, P, P, I, P, P, P, F, F, F, P, P, P, LL, I, I, P]),
    "fbn_adam_selftest": (I, [I, ctypes.c_uint, P, P]),
    "fbn_adam_step_tail": (I, [P, P, P, P, LL, P, F, P, P, P, P, P, I, P, P, P, P, I, I, P, P, F, F, F, P, P, P, P, I,
                               LL, I, P, P, P, P, I, P, P]),
    "fbn_adam_commit": (I, [P, P, P, I, P, P, P, P, I, I, P, P, P, F, F, F, P, P, P, P, I, I, P]),
    "fbn_claim_rows": (I, [P, P, I, I, LL, P, P, P, P, P]),
    "fbn_pack_extras": (I, [P, P, P, P]),
    "fbn_unpack_extras": (I, [P, P, P, P]),
    "fbn_step_end": (I, [P, P, P, P, P, I, P, P]),
    "fbn_route": (I, [P, P, I, I, LL, LL, I, P, P, P, P, P, P, P]),
    "fbn_owner_claim": (I, [P, I, P, P, I, P]),
    "fbn_owner_gather": (I, [P, I, P, P, P, P, I, I, I, P]),
    "fbn_widen_bf16": (I, [P, P, LL, P]),
    "fbn_pad_routes": (I, [P, P, P, I, I, P, P]),
    "fbn_compact_routes": (I, [P, I, I, P, P, P]),
    "fbn_copy_jobs": (I, [P, P, P, I, P]),
    "fbn_bilinear_supported": (I, [I]),
    "fbn_bilinear_fwd": (I, [P, P, P, I, I, I, P]),
    "fbn_bilinear_bwd": (I, [P, I, I, P, P, P, P, P, I, I, P]),
    "fbn_collate": (I, [P, I, P, P, I, I, P, P, P, P, P, LL, P, P, I, P, P, P, P, P, P, P, P, P]),
    "fbn_collate_zero_if": (I, [P, LL, P, P]),
}

_lib: Optional[ctypes.CDLL] = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} is missing: build it with `python -m ctr_recommendation_amd.build` "
                "(the FiBiNET path has no CPU fallback)")
        h = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(h, name)
            fn.restype = res
            fn.argtypes = args
        _lib = h
    return _lib


_fns = {}
_UNCHECKED = ("fbn_version", "fbn_device_ok")


def call(name: str, *args) -> int:
    f = _fns.get(name)
    if f is None:                  # bound ctypes function, looked up once (host time per step)
        f = _fns[name] = getattr(lib(), name)
    rc = f(*args)
    if rc and isinstance(rc, int) and name not in _UNCHECKED and not name.endswith(("_size", "_grid")):
        msg = lib().fbn_last_error().decode(errors="replace")
        raise RuntimeError(f"{name} failed (code {rc}): {msg}")
    return rc


def ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_handle(device: Optional[torch.device] = None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def require_hip(t: torch.Tensor, what: str = "input") -> None:
    if t.device.type != "cuda":
        raise RuntimeError(
            f"{what} is on {t.device}; the MI355X FiBiNET path runs only on a HIP device "
            "(no CPU fallback: move the model and batch with .to('cuda'))")
