"""ctypes bindings for the in-tree native libraries.

* ``libdml_hip.so`` — HIP kernels for gfx950 (forest build/predict, binning, scoring,
  linear-model kernels).  Loaded only when a GPU path runs; if a GPU is present and the
  library is missing or stale the import FAILS LOUDLY (there is no silent fallback).
* ``libdml_cpu.so`` — C++ runtime (CPU forest builder used for the no-GPU plumbing
  config and as the exactness oracle for the HIP builder; scheduler core; binning).

Both are built by ``cs230_distributed_machine_learning_amd.build`` (``__graft_entry__.build``).
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

from .. import build as _build

_lock = threading.Lock()
_hip = None
_cpu = None

c_i64 = ctypes.c_int64
c_i32 = ctypes.c_int32
c_vp = ctypes.c_void_p

POIS_TABLE = 12

TREESPEC_DTYPE = np.dtype(
    [
        ("seed", "<u8"),
        ("split", "<i4"),
        ("fit", "<i4"),
        ("max_depth", "<i4"),
        ("min_samples_split", "<i4"),
        ("min_samples_leaf", "<i4"),
        ("max_features", "<i4"),
        ("bootstrap", "<i4"),
        ("criterion", "<i4"),
        ("min_impurity_decrease", "<f4"),
        ("target", "<i4"),
        ("pois_cdf", "<u4", (POIS_TABLE,)),
        ("cw_mode", "<i4"),
        ("reserved", "<i4"),
        ("min_weight_frac", "<f8"),
        ("min_weight_leaf", "<f8"),
    ]
)


def _i64_struct(name: str, fields: list[str]):
    return type(name, (ctypes.Structure,), {"_fields_": [(f, c_i64) for f in fields]})


ForestArgs = _i64_struct(
    "ForestArgs",
    [
        "Xb", "ld", "n", "d",
        "ycls", "yreg", "n_classes", "is_reg",
        "roles", "n_splits",
        "specs", "T",
        "active_count", "row_off", "rows_total", "max_active",
        "nodes", "node_val", "pool_cap",
        "tree_W",
        "workspace", "workspace_bytes",
        "wave_max", "block_max", "chunk",
        "kg_wave", "kg_block", "kg_large", "slack_wave",
        "sub_max", "sub_cache_d",
        "n_nodes_out", "status_out", "levels_out", "large_rounds_out",
        "tier0_nodes", "tier1_nodes", "tier2_nodes", "tier3_nodes",
        "ystride", "XbT", "cw",
        "yq_e1", "yq_e2",
        "mono", "nbound", "fast_crit",
        "early_pred", "fit_done_level", "n_fits",
        "bigsub_max", "all_features", "sub_small", "root_counts", "root_counts_valid", "large_unit",
        "large_pack",
    ],
)

PredictArgs = _i64_struct(
    "PredictArgs",
    ["Xb", "ld", "nodes", "node_val", "VC", "is_reg", "n_classes", "fit_tree_off", "fit_row_off", "rows",
     "out_pred", "out_proba", "F", "max_rows", "d", "lds_pitch", "fit_row_off_host", "fit_skip", "fit_depth_cap",
     "toptab", "max_trees"],
)

ScoreArgs = _i64_struct("ScoreArgs", ["rows", "fit_row_off", "pred", "ycls", "yreg", "is_reg", "out", "F"])

# csrc/kernels/lr_mfma.hip argument blocks (MFMA logistic-regression objective)
LrFwdArgs = _i64_struct(
    "LrFwdArgs",
    ["xh", "xl", "xrows", "wh", "wl", "n", "Kp", "row_tiles", "col_tiles", "row_groups", "bias", "col_fit",
     "fit_col0", "fit_k", "fit_kind", "fit_split", "scale", "cw", "cwC", "y", "roles", "rh", "rl", "kr", "loss",
     "lpart", "col_info", "col_scale", "n_splits", "softmax_any", "row_base", "live", "w_zero", "ct_split", "rt_skip",
     "rt_stride"],
)
# csrc/kernels/gbrt.hip argument blocks (fused gradient-boosting stage kernels)
GbStageArgs = _i64_struct(
    "GbStageArgs",
    ["Xb", "ld", "n", "nodes", "node_val", "J", "K", "S", "tree_raw", "tree_loss", "tree_lr", "inbag", "grad",
     "ycls", "slot_sum", "slot_node", "slot_val", "raw", "XbT", "pct_any", "yreg", "slot_of", "sel_hist", "sel_state",
     "tree_q", "tree_delta", "phase"],
)
GbGradArgs = _i64_struct("GbGradArgs", ["n", "K", "A", "fit_raw", "fit_loss", "raw", "ycls", "yreg", "grad", "tgt",
                                        "fit_alpha", "fit_delta", "fit_train", "sel_hist", "sel_state"])
# csrc/kernels/forest_mae.hip (criterion="absolute_error" builder)
MaeArgs = _i64_struct(
    "MaeArgs",
    ["Xb", "ld", "n", "d", "yreg", "roles", "specs", "T", "perm", "yq_e1", "yq_e2", "counts", "row_off", "rows_a",
     "rows_b", "nodes", "vals", "nabs", "pool_cap", "open_a", "open_b", "open_cap", "counters", "tree_W",
     "n_nodes_out", "levels_out", "status_out", "big_a", "big_b", "big_cap", "res", "P", "big_rows"],
)
LrGradArgs = _i64_struct("LrGradArgs", ["rh", "rl", "unused", "xth", "xtl", "m_tiles", "n_tiles", "Kp", "S", "Kc", "out",
                                        "bk_off", "slab0", "mlive", "kskip"])


def _load(path: str) -> ctypes.CDLL:
    return ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)


def cpu_lib() -> ctypes.CDLL:
    """Load (building if needed) the C++ runtime library."""
    global _cpu
    with _lock:
        if _cpu is None:
            path = _build.build_cpu()   # rebuilds only when the sources' content changed
            lib = _load(path)
            lib.dml_cpu_sizeof_treespec.restype = c_i32
            if lib.dml_cpu_sizeof_treespec() != TREESPEC_DTYPE.itemsize:
                raise RuntimeError("TreeSpec layout mismatch between C++ and Python")
            lib.dml_cpu_forest_build.restype = c_vp
            lib.dml_cpu_forest_build.argtypes = [c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_i64,
                                                 c_i64, c_vp]
            lib.dml_cpu_forest_build_mono.restype = c_vp
            lib.dml_cpu_forest_build_mono.argtypes = [c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp,
                                                      c_i64, c_i64, c_vp, c_vp, c_i64, c_i64]
            lib.dml_reg_exponents.argtypes = [c_vp, c_i64, c_vp]
            lib.dml_cpu_forest_apply.argtypes = [c_vp, c_i64, c_i64, c_vp, c_i32, c_i32, c_vp]
            lib.dml_cpu_forest_refine.argtypes = [c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_i32, c_vp, c_vp, c_vp]
            lib.dml_cpu_forest_prune.argtypes = [c_vp, c_vp, c_i64, c_i32, c_i32, c_vp, c_vp, c_i32, c_vp]
            lib.dml_cpu_forest_num_nodes.restype = c_i64
            lib.dml_cpu_forest_num_nodes.argtypes = [c_vp]
            lib.dml_cpu_forest_export.argtypes = [c_vp, c_vp, c_vp]
            lib.dml_cpu_forest_free.argtypes = [c_vp]
            lib.dml_cpu_forest_predict.argtypes = [c_vp, c_i64, c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp,
                                                   c_i64, c_vp, c_vp, c_vp]
            lib.dml_cpu_bin.argtypes = [c_vp, c_i64, c_i64, c_vp, c_vp, c_i64]
            lib.dml_cpu_svm_sizeof_prob.restype = c_i32
            lib.dml_cpu_svm_smo.argtypes = [c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp]
            lib.dml_cpu_dp_sizeof_args.restype = c_i32
            lib.dml_cpu_dp_step.restype = c_i32
            lib.dml_cpu_dp_step.argtypes = [c_vp, c_i32]
            _cpu = lib
        return _cpu


def hip_lib() -> ctypes.CDLL:
    """Load the HIP kernel library; raises if it is absent (no silent fallback)."""
    global _hip
    with _lock:
        if _hip is None:
            path = os.environ.get("DML_HIP_LIB") or _build.HIP_LIB   # override: A/B kernel variants
            if not os.path.exists(path):
                raise RuntimeError(
                    f"HIP kernel library {path} is missing: run `python -m cs230_distributed_machine_learning_amd.build`"
                )
            lib = _load(path)
            lib.dml_forest_sizeof_treespec.restype = c_i32
            lib.dml_forest_sizeof_args.restype = c_i32
            if lib.dml_forest_sizeof_treespec() != TREESPEC_DTYPE.itemsize:
                raise RuntimeError("TreeSpec layout mismatch between HIP library and Python")
            if lib.dml_forest_sizeof_args() != ctypes.sizeof(ForestArgs):
                raise RuntimeError("ForestArgs layout mismatch between HIP library and Python")
            lib.dml_predict_sizeof_args.restype = c_i32
            if lib.dml_predict_sizeof_args() != ctypes.sizeof(PredictArgs):
                raise RuntimeError("PredictArgs layout mismatch between HIP library and Python")
            lib.dml_forest_last_error.restype = ctypes.c_char_p
            lib.dml_forest_last_error.argtypes = [ctypes.POINTER(c_i32)]
            lib.dml_forest_workspace_bytes.restype = c_i64
            lib.dml_forest_workspace_bytes.argtypes = [ctypes.POINTER(ForestArgs)]
            lib.dml_forest_count.restype = c_i32
            lib.dml_forest_count.argtypes = [ctypes.POINTER(ForestArgs), c_vp]
            lib.dml_forest_build.restype = c_i32
            lib.dml_forest_build.argtypes = [ctypes.POINTER(ForestArgs), c_vp]
            lib.dml_forest_predict.restype = c_i32
            lib.dml_forest_predict.argtypes = [ctypes.POINTER(PredictArgs), c_vp]
            lib.dml_forest_predict_fit.restype = c_i32
            lib.dml_forest_predict_fit.argtypes = [ctypes.POINTER(PredictArgs), c_i32, c_vp]
            lib.dml_scores.restype = c_i32
            lib.dml_scores.argtypes = [ctypes.POINTER(ScoreArgs), c_vp]
            lib.dml_bin.restype = c_i32
            lib.dml_bin.argtypes = [c_vp, c_i64, c_i64, c_vp, c_vp, c_i64, c_vp]
            _register_optional(lib)
            _hip = lib
        return _hip


def _register_optional(lib) -> None:
    """Signatures of kernels added in later files (absent symbols are skipped)."""
    table = {
        "dml_lr_link_grad": (c_i32, [c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_i64,
                                     c_vp, c_vp, c_vp]),
        "dml_lr_predict": (c_i32, [c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp]),
        "dml_knn_l2_mfma": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_i64, c_i32, c_vp,
                                    c_vp, c_vp]),
        "dml_knn": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_i64, c_i32, ctypes.c_float, c_i32, c_vp,
                            c_vp, c_vp]),
        "dml_knn_qpw": (c_i32, []),
        "dml_forest_apply": (c_i32, [c_vp, c_i64, c_i64, c_vp, c_i32, c_i32, c_vp, c_vp]),
        "dml_forest_prune": (c_i32, [c_vp, c_vp, c_i64, c_i32, c_i32, c_vp, c_vp, c_i32, c_i32, c_vp, c_i64, c_vp, c_vp]),
        "dml_svm_sizeof_prob": (c_i32, []),
        "dml_forest_set_lane": (c_i32, [c_i32]),
        "dml_forest_refine": (c_i32, [c_vp, c_i64, c_i64, c_i64, c_vp, c_i64, c_vp, c_i32, c_vp, c_vp, c_vp, c_vp,
                                      c_vp]),
        "dml_svm_smo_split": (c_i32, [c_vp, c_i64, c_vp, c_i64, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                      c_vp, c_vp, c_vp, c_i64, c_vp, c_i32, c_vp]),
        "dml_svm_split_limits": (c_i32, [c_vp, c_vp, c_vp]),
        "dml_svm_smo": (c_i32, [c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp]),
        "dml_split_moments": (c_i32, [c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_i64, c_i32, c_vp, c_i64, c_vp]),
        "dml_lr_mfma_tile": (c_i32, []),
        "dml_lr_mfma_fwd": (c_i32, [ctypes.POINTER(LrFwdArgs), c_vp]),
        "dml_lr_mfma_grad": (c_i32, [ctypes.POINTER(LrGradArgs), c_vp]),
        "dml_lr_v3_row_tile": (c_i32, []),
        "dml_lr_mfma_fwd3": (c_i32, [ctypes.POINTER(LrFwdArgs), c_vp]),
        "dml_lr_mfma_grad3": (c_i32, [ctypes.POINTER(LrGradArgs), c_vp]),
        "dml_split_hilo": (c_i32, [c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_i64, c_i32, c_vp, c_vp]),
        "dml_lr_sizeof_fwd_args": (c_i32, []),
        "dml_lr_sizeof_grad_args": (c_i32, []),
        "dml_dp_sizeof_args": (c_i32, []),
        "dml_dp_sizeof_slot": (c_i32, []),
        "dml_dp_step": (c_i32, [c_vp, c_i32, c_vp]),
        "dml_gb_sizeof_stage_args": (c_i32, []),
        "dml_gb_sizeof_grad_args": (c_i32, []),
        "dml_gb_stage": (c_i32, [ctypes.POINTER(GbStageArgs), c_vp]),
        "dml_gb_grad": (c_i32, [ctypes.POINTER(GbGradArgs), c_vp]),
        "dml_gb_huber_delta": (c_i32, [ctypes.POINTER(GbGradArgs), c_vp]),
        "dml_gb_stage_phase": (c_i32, [ctypes.POINTER(GbStageArgs), c_vp]),
        "dml_gb_sel_step": (c_i32, [ctypes.POINTER(GbStageArgs), c_i32, c_i32, c_vp]),
        "dml_gb_fit_sel_step": (c_i32, [ctypes.POINTER(GbGradArgs), c_i32, c_i32, c_vp]),
        "dml_exp_hist": (c_i32, [c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp]),
        "dml_forest_release_scratch": (c_i32, []),
        "dml_mae_sizeof_args": (c_i32, []),
        "dml_mae_sizeof_open": (c_i32, []),
        "dml_mae_sizeof_res": (c_i32, []),
        "dml_mae_count": (c_i32, [ctypes.POINTER(MaeArgs), c_vp]),
        "dml_mae_build": (c_i32, [ctypes.POINTER(MaeArgs), c_vp]),
    }
    for name, (res, args) in table.items():
        fn = getattr(lib, name, None)
        if fn is not None:
            fn.restype = res
            fn.argtypes = args
    if getattr(lib, "dml_gb_sizeof_stage_args", None) is not None:
        if (lib.dml_gb_sizeof_stage_args() != ctypes.sizeof(GbStageArgs)
                or lib.dml_gb_sizeof_grad_args() != ctypes.sizeof(GbGradArgs)):
            raise RuntimeError("GBRT stage argument layout mismatch between HIP library and Python")
    if getattr(lib, "dml_mae_sizeof_args", None) is not None and lib.dml_mae_sizeof_args() != ctypes.sizeof(MaeArgs):
        raise RuntimeError("MAE builder argument layout mismatch between HIP library and Python")
    if getattr(lib, "dml_lr_sizeof_fwd_args", None) is not None:
        if (lib.dml_lr_sizeof_fwd_args() != ctypes.sizeof(LrFwdArgs)
                or lib.dml_lr_sizeof_grad_args() != ctypes.sizeof(LrGradArgs)):
            raise RuntimeError("LR MFMA argument layout mismatch between HIP library and Python")


def hip_error(lib=None) -> str:
    lib = lib or hip_lib()
    line = c_i32(0)
    msg = lib.dml_forest_last_error(ctypes.byref(line))
    return f"{msg.decode() if msg else '?'} (forest.hip:{line.value})"


def ptr(t) -> int:
    """Device/host address of a torch tensor or numpy array (0 for None)."""
    if t is None:
        return 0
    if isinstance(t, np.ndarray):
        return int(t.ctypes.data)
    return int(t.data_ptr())


def stream_handle(device=None) -> int:
    import torch

    return int(torch.cuda.current_stream(device).cuda_stream)


def poisson_cdf_table(lam: float) -> np.ndarray:
    """Thresholds u >= T[j] => weight > j for u uniform on [0, 2^32)."""
    import math

    out = np.empty(POIS_TABLE, dtype=np.uint64)
    p = math.exp(-lam)
    cdf = 0.0
    for j in range(POIS_TABLE):
        cdf += p
        p *= lam / (j + 1)
        out[j] = min(int(cdf * 2.0**32), 0xFFFFFFFF)
    return out.astype(np.uint32)
