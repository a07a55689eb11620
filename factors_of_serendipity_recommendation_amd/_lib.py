"""ctypes binding of liblgx.so (the C ABI declared in include/lgx.h).

The library is built in-tree (``csrc/Makefile`` -> ``liblgx.so`` next to this file).  There is no
fallback: if the shared object is missing or a call fails, a RuntimeError is raised.  torch is
imported first so that liblgx.so binds to the HIP runtime torch already loaded (both carry the
SONAME libamdhip64.so.7) instead of pulling in a second copy.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import torch  # noqa: F401  (must be loaded before liblgx.so, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liblgx.so")
CSRC = os.path.join(_HERE, "csrc")

LGX_OK = 0
LGX_DTYPE_F32 = 0
LGX_DTYPE_BF16 = 1
LGX_LAYER_PLAIN, LGX_LAYER_FIRST, LGX_LAYER_MID, LGX_LAYER_LAST, LGX_LAYER_ONLY, LGX_LAYER_PARTIAL, LGX_LAYER_STACK = range(7)
LGX_REDUCE_MAX, LGX_REDUCE_SUM = 0, 1
LGX_STRAT_EXACT = 1

_c_i64 = ctypes.c_int64
_c_int = ctypes.c_int
_c_float = ctypes.c_float
_vp = ctypes.c_void_p
_sz_p = ctypes.POINTER(ctypes.c_size_t)


class LgxPlan(ctypes.Structure):
    """Mirror of ``struct lgx_plan`` (include/lgx.h)."""

    _fields_ = [
        ("seg_row", _vp), ("seg_part", _vp), ("seg_slot", _vp),
        ("n_segs", _c_i64), ("seg_len", _c_i64),
        ("split_row", _vp), ("split_ptr", _vp),
        ("n_split", _c_i64), ("n_partials", _c_i64), ("partials", _vp),
    ]


class LgxCSR(ctypes.Structure):
    """Mirror of ``struct lgx_csr`` (include/lgx.h)."""

    _fields_ = [
        ("indptr", _vp), ("indices", _vp), ("vals", _vp),
        ("n_rows", _c_i64), ("n_cols", _c_i64), ("nnz", _c_i64),
        ("seg_row", _vp), ("seg_part", _vp), ("seg_slot", _vp),
        ("n_segs", _c_i64), ("seg_len", _c_i64),
        ("split_row", _vp), ("split_ptr", _vp),
        ("n_split", _c_i64), ("n_partials", _c_i64), ("partials", _vp),
        ("cb_row0", _c_i64), ("cb_n", _c_i64), ("cb_ptr", _vp),
        ("cb_plans", ctypes.POINTER(LgxPlan)), ("cb_carry", _vp),
    ]


# name -> (restype, argtypes); every entry point of include/lgx.h
SIGNATURES = {
    "lgx_version": (ctypes.c_char_p, []),
    "lgx_last_error": (ctypes.c_char_p, []),
    "lgx_device_info": (_c_int, [_c_int, ctypes.POINTER(_c_int), ctypes.POINTER(_c_int), ctypes.c_char_p, ctypes.c_size_t]),
    "lgx_build_norm_adj_workspace": (_c_int, [_c_i64, _c_i64, _c_i64, _sz_p]),
    "lgx_build_norm_adj": (_c_int, [_vp, _vp, _c_i64, _c_i64, _c_i64, _c_int, _vp, _vp, _vp, _vp, ctypes.c_size_t, _vp]),
    "lgx_csr_from_coo_rows": (_c_int, [_vp, _c_i64, _c_i64, _vp, _vp]),
    "lgx_propagate_layer": (_c_int, [ctypes.POINTER(LgxCSR), _vp, _vp, _vp, _vp, _vp, _c_i64, _c_int, _c_int,
                                     ctypes.c_float, _vp]),
    "lgx_spmm_csr": (_c_int, [ctypes.POINTER(LgxCSR), _vp, _vp, _c_i64, _c_int, _vp]),
    "lgx_propagate_layer_stack": (_c_int, [ctypes.POINTER(LgxCSR), _vp, _vp, _vp, _c_int, _vp, _c_i64, _c_int,
                                           ctypes.c_float, _vp]),
    "lgx_strat_labels": (_c_int, [_vp, _c_i64, _c_i64, _c_float, _c_float, _c_int, _vp, _vp, _vp, _vp, _vp]),
    "lgx_strat_select": (_c_int, [_vp, _c_i64, _c_i64, _vp, _c_int, _vp, ctypes.c_uint64, _vp, _c_int, _vp, _vp]),
    "lgx_spmm_kernel_name": (_c_int, [_c_i64, _c_int, _c_i64, ctypes.c_char_p, ctypes.c_size_t]),
    "lgx_score_topk_plan": (_c_int, [_c_i64, _c_i64, _c_i64, _c_int, _c_int, ctypes.c_char_p, ctypes.c_size_t]),
    "lgx_strat_select_ex": (_c_int, [_vp, _c_i64, _c_i64, _vp, _c_int, _vp, ctypes.c_uint64, _vp, _c_int, _vp,
                                     _c_int, _vp]),
    "lgx_strat_labels_fused": (_c_int, [_vp, _vp, _vp, _c_i64, _c_i64, _c_i64, _c_int, _c_float, _c_float, _c_int,
                                        _vp, _vp, _vp, _vp, _vp]),
    "lgx_strat_thresholds": (_c_int, [_c_float, _c_float, _c_int, _vp]),
    "lgx_strat_hist": (_c_int, [_vp, _c_i64, _c_i64, _c_int, _vp, _vp, _vp, _vp]),
    "lgx_strat_mask": (_c_int, [_vp, _c_i64, _c_i64, _c_int, _vp, _vp, _vp, _vp]),
    "lgx_parse_lines_workspace": (_c_int, [_c_i64, _sz_p]),
    "lgx_parse_lines_count": (_c_int, [_vp, _c_i64, _vp, ctypes.c_size_t, _vp, _vp]),
    "lgx_parse_lines_fill": (_c_int, [_vp, _c_i64, _vp, ctypes.c_size_t, _c_i64, _c_i64, _vp, _vp, _vp, _vp, _vp]),
    "lgx_sample_bpr": (_c_int, [_vp, _vp, _c_i64, _c_i64, _vp, _c_i64, _c_i64, _c_int, ctypes.c_uint64, _vp, _vp]),
    "lgx_bpr_loss_workspace": (_c_int, [_c_i64, _sz_p]),
    "lgx_bpr_loss_forward": (_c_int, [_vp, _vp, _vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _vp, _c_i64, _vp, _vp, _vp,
                                      _vp, ctypes.c_size_t, _vp]),
    "lgx_bpr_loss_backward": (_c_int, [_vp, _vp, _vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _vp, _c_i64, _vp, _vp, _vp,
                                       _vp, _vp, _vp, _vp]),
    "lgx_adam_step": (_c_int, [_vp, _vp, _vp, _vp, _c_i64, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                               ctypes.c_double, _c_i64, _vp]),
    "lgx_adam_step_dev": (_c_int, [_vp, _vp, _vp, _vp, _c_i64, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                   ctypes.c_double, _vp, _vp]),
    "lgx_list_dot_reduce": (_c_int, [_vp, _c_i64, _c_int, _c_i64, _vp, _vp, _vp, _vp, _c_int, _vp, _vp]),
    "lgx_layer_epilogue": (_c_int, [_vp, _c_i64, _vp, _vp, _vp, _vp, _c_i64, _c_int, _c_int, _c_float, _vp]),
    "lgx_sum_slabs": (_c_int, [_vp, _c_i64, _c_i64, _vp, _vp]),
    "lgx_propagate_workspace": (_c_int, [_c_i64, _c_i64, _c_int, _sz_p]),
    "lgx_propagate": (_c_int, [ctypes.POINTER(LgxCSR), _vp, _vp, _c_i64, _c_int, _c_int, _vp, ctypes.c_size_t, _vp]),
    "lgx_score_dense": (_c_int, [_vp, _vp, _vp, _c_i64, _c_i64, _c_i64, _c_int, _c_int, _vp, _vp]),
    "lgx_score_topk_workspace": (_c_int, [_c_i64, _c_i64, _c_int, _sz_p]),
    "lgx_score_minmax_workspace": (_c_int, [_c_i64, _c_i64, _sz_p]),
    "lgx_score_minmax": (_c_int, [_vp, _vp, _vp, _c_i64, _c_i64, _c_i64, _c_int, _vp, _vp, ctypes.c_size_t, _vp]),
    "lgx_score_topk": (_c_int, [_vp, _vp, _vp, _c_i64, _c_i64, _c_i64, _c_int, _vp, _vp, _c_int, ctypes.c_float,
                                _c_int, _vp, _vp, _vp, _vp, ctypes.c_size_t, _vp]),
    "lgx_topk_rows": (_c_int, [_vp, _c_i64, _c_i64, _c_i64, _c_int, _vp, _vp, _vp]),
    "lgx_foldout_metrics": (_c_int, [_vp, _c_i64, _c_int, _vp, _vp, _vp, _vp, _vp]),
    "lgx_column_mean_f32": (_c_int, [_vp, _c_i64, _c_i64, _vp, _vp]),
    "lgx_test_metrics_workspace": (_c_int, [_c_i64, _c_int, _sz_p]),
    "lgx_test_metrics": (_c_int, [_vp, _c_i64, _c_int, _vp, _vp, _vp, _vp, _c_int, _vp, _vp, _vp, ctypes.c_size_t, _vp]),
    "lgx_gather_scores": (_c_int, [_vp, _vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _c_i64, _vp, _vp]),
    "lgx_synth_edges": (_c_int, [ctypes.c_uint64, _vp, _c_i64, _vp, _vp, _c_i64, _c_i64, _vp, _vp, _vp]),
    "lgx_fill_normal": (_c_int, [_vp, _c_i64, ctypes.c_float, ctypes.c_uint64, _c_int, _vp]),
    "lgx_fill_normal_at": (_c_int, [_vp, _c_i64, _c_i64, ctypes.c_float, ctypes.c_uint64, _c_int, _vp]),
}

_lib = None
# development A/B only (tools/*.py --lib): load an older build that lacks newer entry points
ALLOW_MISSING = False


def build(force: bool = False, jobs: int = 8) -> str:
    """Compile liblgx.so for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
    cmd = ["make", "-s", f"-j{jobs}", "-C", CSRC]
    if force:
        subprocess.check_call(["make", "-s", "-C", CSRC, "clean"])
    subprocess.check_call(cmd)
    return LIB_PATH


def lib():
    """The loaded liblgx.so.  Raises if it was not built -- there is no CPU fallback."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"liblgx.so not found at {LIB_PATH}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc --offload-arch=gfx950)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if ALLOW_MISSING and not hasattr(L, name):
                continue
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc: int, what: str) -> None:
    if rc != LGX_OK:
        msg = lib().lgx_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (lgx status {rc}): {msg}")


def version() -> str:
    return lib().lgx_version().decode()
