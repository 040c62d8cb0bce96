"""ctypes binding of the C-ABI in include/nais.h (libnais_hip.so, built for gfx950).

There is deliberately no fallback: if the shared library is missing or fails to load, every
product entry point raises. The CPU restatement under oracle/ is test infrastructure only.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_NAME = "libnais_hip.so"
LIB_PATH = os.path.join(HERE, LIB_NAME)

ABI_VERSION = 14
PRECISION_FP32, PRECISION_FP16X3, PRECISION_FP16X3_PAIRSPLIT = 0, 1, 2
PRIOR_FINITE = 1   # nais_pair_prior_gather flags (include/nais.h NAIS_PRIOR_FINITE)
PRECISION_FP16X6, PRECISION_FP16X6_PAIRSPLIT = 3, 4
VARIANT_BASIC, VARIANT_REGION, VARIANT_REGION_DISTANCE, VARIANT_DISTANCE = 0, 1, 2, 3
FLAG_SIGMOID = 1

EXPORTS = ("nais_abi_version", "nais_last_error", "nais_forward", "nais_score_topk_workspace_size",
           "nais_score_topk", "nais_score_catalog", "nais_topk_rows", "nais_powerlaw_prior",
           "nais_distance_histogram", "nais_gather_rows", "nais_train_workspace_size",
           "nais_train_forward", "nais_train_backward", "nais_dropout_mask", "nais_adagrad",
           "nais_adagrad_rows", "nais_train_step_workspace_size", "nais_train_step", "nais_train_step_ex",
           "nais_make_train_batch", "nais_new4_tables", "nais_pair_rows_workspace_size",
           "nais_pair_rows", "nais_pair_table", "nais_pair_gather", "nais_stream_create_cu_mask",
           "nais_stream_destroy", "nais_near_attention", "nais_copy_columns",
           "nais_linear_rows", "nais_dot_forward", "nais_dot_pair_table", "nais_dot_single_fixup",
           "nais_disent_forward", "nais_pair_distances", "nais_train_forward_ex",
           "nais_train_backward_ex", "nais_pair_gather_topk", "nais_topk_keys_finish",
           "nais_pair_prior_table",
           "nais_pair_prior_gather", "nais_topk_blend_rows", "nais_topk_blend_rows_f64",
           "nais_topk_merge_f64", "nais_train_ucache_size", "nais_pair_table_split",
           "nais_pair_bound_topk", "nais_pair_refine_topk")


class NaisDotTables(ctypes.Structure):
    """Mirror of `nais_dot_tables_t` (include/nais.h)."""
    _fields_ = [("embed_dim", ctypes.c_int32), ("num_pois", ctypes.c_int64), ("beta", ctypes.c_float),
                ("scale_dim", ctypes.c_float), ("xh", ctypes.c_void_p), ("xt", ctypes.c_void_p),
                ("qt", ctypes.c_void_p), ("kh", ctypes.c_void_p), ("vh", ctypes.c_void_p)]


class NaisTrainSide(ctypes.Structure):
    """Mirror of `nais_train_side_t` (include/nais.h)."""
    _fields_ = [("hist_region", ctypes.c_void_p), ("target_region", ctypes.c_void_p),
                ("target_lat_long", ctypes.c_void_p), ("latlon_ld", ctypes.c_int64),
                ("ucache", ctypes.c_void_p), ("ucache_bytes", ctypes.c_uint64)]


class NaisTrainGrads(ctypes.Structure):
    """Mirror of `nais_train_grads_t` (include/nais.h)."""
    _fields_ = [(n, ctypes.c_void_p) for n in ("embed_history", "embed_target", "embed_region", "w1",
                                               "b1", "w2", "dist_w", "dist_b")]


class NaisDisentParams(ctypes.Structure):
    """Mirror of `nais_disent_params_t` (include/nais.h)."""
    _fields_ = [("embed_dim", ctypes.c_int32), ("hidden", ctypes.c_int32), ("num_pois", ctypes.c_int64),
                ("num_regions", ctypes.c_int64), ("beta", ctypes.c_float)] + \
        [(n, ctypes.c_void_p) for n in ("embed_history", "embed_target", "embed_region", "embed_distance",
                                        "w1", "b1", "w2", "region_w1", "region_b1", "region_w2")]


class NaisParams(ctypes.Structure):
    """Mirror of `nais_params_t` (include/nais.h)."""
    _fields_ = [
        ("variant", ctypes.c_int32), ("embed_dim", ctypes.c_int32), ("item_dim", ctypes.c_int32),
        ("region_dim", ctypes.c_int32), ("hidden", ctypes.c_int32), ("din", ctypes.c_int32),
        ("num_pois", ctypes.c_int64), ("num_regions", ctypes.c_int64),
        ("beta", ctypes.c_float), ("precision", ctypes.c_int32),
        ("embed_history", ctypes.c_void_p), ("embed_target", ctypes.c_void_p),
        ("embed_region", ctypes.c_void_p), ("w1", ctypes.c_void_p), ("b1", ctypes.c_void_p),
        ("w2", ctypes.c_void_p), ("dist_w", ctypes.c_void_p), ("dist_b", ctypes.c_void_p),
    ]


class NaisPrior(ctypes.Structure):
    """Mirror of `nais_prior_t`."""
    _fields_ = [("a", ctypes.c_double), ("b", ctypes.c_double), ("alpha", ctypes.c_double),
                ("coords", ctypes.c_void_p)]


class NaisAdagradState(ctypes.Structure):
    """Mirror of `nais_adagrad_state_t`."""
    _fields_ = [("lr", ctypes.c_float), ("lr_decay", ctypes.c_float),
                ("weight_decay", ctypes.c_float), ("eps", ctypes.c_float), ("step", ctypes.c_int64)] + \
        [(n, ctypes.c_void_p) for n in ("sum_embed_history", "sum_embed_target", "sum_w1", "sum_b1",
                                        "sum_w2", "grad_embed_history", "grad_embed_target",
                                        "grad_small", "stamp_embed_history", "stamp_embed_target")]


class NaisAdagradSide(ctypes.Structure):
    """Mirror of `nais_adagrad_side_t` (the region / distance variants' extra Adagrad state)."""
    _fields_ = [(n, ctypes.c_void_p) for n in ("sum_embed_region", "grad_embed_region", "sum_dist_w",
                                               "sum_dist_b", "grad_dist")]


class NaisError(RuntimeError):
    pass


_lib = None


def load(path: str | None = None):
    """Load (once) and type the shared library; raises NaisError if it cannot be loaded."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or os.environ.get("NAIS_HIP_LIB", LIB_PATH)
    if not os.path.exists(p):
        raise NaisError(f"{p} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                        "(hipcc --offload-arch=gfx950); there is no CPU fallback for the NAIS path")
    try:
        lib = ctypes.CDLL(p)
    except OSError as e:
        raise NaisError(f"failed to load {p}: {e}") from e
    vp, i32, i64, sz = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_size_t
    lib.nais_abi_version.restype = i32
    lib.nais_abi_version.argtypes = []
    lib.nais_last_error.restype = ctypes.c_char_p
    lib.nais_last_error.argtypes = []
    lib.nais_forward.restype = i32
    lib.nais_forward.argtypes = [ctypes.POINTER(NaisParams), vp, i64, i64, i64, vp, vp, i64, vp, vp,
                                 i64, vp, vp, i32, vp]
    lib.nais_score_topk_workspace_size.restype = sz
    lib.nais_score_topk_workspace_size.argtypes = [ctypes.POINTER(NaisParams), i32, i32, i32]
    lib.nais_score_topk.restype = i32
    lib.nais_score_topk.argtypes = [ctypes.POINTER(NaisParams), vp, vp, vp, i32, i32, vp, vp, vp,
                                    ctypes.c_void_p, vp, vp, vp, vp, vp, sz, vp]
    lib.nais_score_catalog.restype = i32
    lib.nais_score_catalog.argtypes = [ctypes.POINTER(NaisParams), vp, vp, vp, i32, vp, vp, vp, vp,
                                       i64, vp, vp]
    lib.nais_topk_rows.restype = i32
    lib.nais_topk_rows.argtypes = [vp, i64, i64, i32, i32, vp, vp, vp, vp]
    f64 = ctypes.c_double
    lib.nais_powerlaw_prior.restype = i32
    lib.nais_powerlaw_prior.argtypes = [vp, i64, vp, vp, vp, i32, f64, f64, vp, i64, vp, vp]
    lib.nais_distance_histogram.restype = i32
    lib.nais_distance_histogram.argtypes = [vp, vp, vp, i64, vp, i64, vp, vp]
    lib.nais_gather_rows.restype = i32
    lib.nais_gather_rows.argtypes = [vp, i64, i32, vp, i64, vp, vp]
    f32, u64 = ctypes.c_float, ctypes.c_uint64
    lib.nais_train_workspace_size.restype = sz
    lib.nais_train_workspace_size.argtypes = [ctypes.POINTER(NaisParams), i64, i64]
    lib.nais_train_forward.restype = i32
    lib.nais_train_forward.argtypes = [ctypes.POINTER(NaisParams), vp, i64, vp, i64, f32, u64, vp, vp,
                                       vp, vp, sz, vp]
    lib.nais_train_backward.restype = i32
    lib.nais_train_backward.argtypes = [ctypes.POINTER(NaisParams), vp, i64, vp, i64, f32, u64, vp, vp,
                                        vp, vp, vp, vp, vp, vp, vp, sz, vp]
    lib.nais_dropout_mask.restype = i32
    lib.nais_dropout_mask.argtypes = [u64, i64, i64, i32, f32, vp, vp]
    lib.nais_adagrad.restype = i32
    lib.nais_adagrad.argtypes = [vp, vp, vp, i64, f32, f32, f32, vp]
    lib.nais_adagrad_rows.restype = i32
    lib.nais_adagrad_rows.argtypes = [vp, vp, vp, i32, vp, i64, f32, f32, vp]
    lib.nais_train_step_workspace_size.restype = sz
    lib.nais_train_step_workspace_size.argtypes = [ctypes.POINTER(NaisParams), i64, i64]
    lib.nais_train_step.restype = i32
    lib.nais_train_step.argtypes = [ctypes.POINTER(NaisParams), ctypes.POINTER(NaisAdagradState), vp,
                                    i64, vp, vp, i64, f32, u64, vp, vp, vp, vp, sz, vp]
    lib.nais_train_step_ex.restype = i32
    lib.nais_train_step_ex.argtypes = [ctypes.POINTER(NaisParams), ctypes.POINTER(NaisTrainSide),
                                       ctypes.POINTER(NaisAdagradState), ctypes.POINTER(NaisAdagradSide),
                                       vp, i64, vp, vp, i64, f32, u64, vp, vp, vp, vp, sz, vp]
    lib.nais_make_train_batch.restype = i32
    lib.nais_make_train_batch.argtypes = [vp, vp, i64, i64, i64, i32, u64, vp, vp, vp, vp, vp]
    lib.nais_new4_tables.restype = i32
    lib.nais_new4_tables.argtypes = [vp, vp, vp, vp, i64, i32, vp, i32, vp, vp, vp]
    lib.nais_near_attention.restype = i32
    lib.nais_near_attention.argtypes = [vp, vp, i64, i32, vp, i32, vp, vp, vp, vp, vp, vp,
                                        ctypes.c_float, vp, i64, vp]
    lib.nais_linear_rows.restype = i32
    lib.nais_linear_rows.argtypes = [vp, i64, i64, i32, vp, vp, i32, vp, i64, vp]
    lib.nais_dot_forward.restype = i32
    lib.nais_dot_forward.argtypes = [ctypes.POINTER(NaisDotTables), vp, i64, i64, i64, vp, vp, vp, i32, vp]
    lib.nais_dot_pair_table.restype = i32
    lib.nais_dot_pair_table.argtypes = [ctypes.POINTER(NaisDotTables), vp, i64, i64, i64, vp, vp, i64, vp]
    lib.nais_dot_single_fixup.restype = i32
    lib.nais_dot_single_fixup.argtypes = [ctypes.POINTER(NaisDotTables), vp, vp, vp, i64, i64, i64, vp,
                                          i64, i64, vp]
    lib.nais_train_forward_ex.restype = i32
    lib.nais_train_forward_ex.argtypes = [ctypes.POINTER(NaisParams), ctypes.POINTER(NaisTrainSide), vp, i64,
                                          vp, i64, f32, u64, vp, vp, vp, vp, ctypes.c_size_t, vp]
    lib.nais_train_backward_ex.restype = i32
    lib.nais_train_backward_ex.argtypes = [ctypes.POINTER(NaisParams), ctypes.POINTER(NaisTrainSide), vp,
                                           i64, vp, i64, f32, u64, vp, vp, vp,
                                           ctypes.POINTER(NaisTrainGrads), vp, ctypes.c_size_t, vp]
    lib.nais_disent_forward.restype = i32
    lib.nais_disent_forward.argtypes = [ctypes.POINTER(NaisDisentParams), vp, i64, i64, i64, vp, vp, i64, vp,
                                        vp, i64, vp, vp, i32, vp]
    lib.nais_pair_distances.restype = i32
    lib.nais_pair_distances.argtypes = [vp, vp, i64, vp, i64, vp, vp]
    lib.nais_copy_columns.restype = i32
    lib.nais_copy_columns.argtypes = [vp, i64, i64, i32, vp, i64, i32, vp]
    lib.nais_pair_rows_workspace_size.restype = sz
    lib.nais_pair_rows_workspace_size.argtypes = [i64]
    lib.nais_pair_rows.restype = i32
    lib.nais_pair_rows.argtypes = [vp, vp, vp, i32, i64, vp, vp, vp, vp, sz, vp]
    lib.nais_pair_table.restype = i32
    lib.nais_pair_table.argtypes = [ctypes.POINTER(NaisParams), vp, i64, i64, i64, vp, vp, vp, vp, vp,
                                    i64, vp, vp]
    lib.nais_pair_gather.restype = i32
    lib.nais_pair_gather.argtypes = [vp, vp, i64, vp, vp, vp, vp, i32, i64, i64, f32, vp, i64, i64, vp,
                                     vp]
    lib.nais_pair_gather_topk.restype = i32
    lib.nais_pair_gather_topk.argtypes = [vp, vp, i64, vp, vp, vp, vp, i32, i64, i64, f32, i32, vp, vp, vp,
                                          vp, vp]
    lib.nais_pair_prior_table.restype = i32
    lib.nais_pair_prior_table.argtypes = [vp, i64, vp, i64, i64, i64, f64, f64, vp, i64, vp]
    lib.nais_pair_prior_gather.restype = i32
    lib.nais_pair_prior_gather.argtypes = [vp, i64, vp, vp, vp, vp, i32, i64, i64, vp, i64, i64, vp, i32, vp]
    lib.nais_topk_blend_rows.restype = i32
    lib.nais_topk_blend_rows.argtypes = [vp, i64, vp, i64, vp, i64, i32, i32, f64, vp, vp, vp, vp]
    lib.nais_topk_blend_rows_f64.restype = i32
    lib.nais_topk_blend_rows_f64.argtypes = [vp, i64, vp, i64, vp, i64, i32, i32, f64, vp, vp, vp, vp, vp]
    lib.nais_train_ucache_size.restype = sz
    lib.nais_train_ucache_size.argtypes = [ctypes.POINTER(NaisParams), i64, i64]
    lib.nais_topk_merge_f64.restype = i32
    lib.nais_topk_merge_f64.argtypes = [vp, vp, i32, i32, i32, vp, vp, vp, vp]
    lib.nais_topk_keys_finish.restype = i32
    lib.nais_topk_keys_finish.argtypes = [vp, vp, i32, i32, vp, vp, vp, vp]
    lib.nais_pair_table_split.restype = i32
    lib.nais_pair_table_split.argtypes = [ctypes.POINTER(NaisParams), vp, i64, i64, i64, vp, vp, vp, vp,
                                          vp, i64, vp, vp]
    lib.nais_pair_bound_topk.restype = i32
    lib.nais_pair_bound_topk.argtypes = [vp, i64, vp, vp, vp, vp, i32, i64, i64, f32, i32, vp, vp, vp, vp,
                                         i32, vp, vp, vp, vp]
    lib.nais_pair_refine_topk.restype = i32
    lib.nais_pair_refine_topk.argtypes = [vp, i64, i64, i64, vp, vp, vp, vp, i32, i64, i64, f32, i32,
                                          vp, vp, vp, vp, i32, vp, vp, vp, vp, vp, vp, vp]
    lib.nais_stream_create_cu_mask.restype = i32
    lib.nais_stream_create_cu_mask.argtypes = [vp, ctypes.c_uint32, ctypes.POINTER(ctypes.c_void_p)]
    lib.nais_stream_destroy.restype = i32
    lib.nais_stream_destroy.argtypes = [vp]
    v = lib.nais_abi_version()
    if v != ABI_VERSION:
        raise NaisError(f"{p}: ABI version {v}, expected {ABI_VERSION}")
    if path is None:
        _lib = lib
    return lib


def check(rc: int, what: str):
    if rc != 0:
        msg = load().nais_last_error().decode(errors="replace")
        raise NaisError(f"{what} failed ({rc}): {msg}")


def ptr(t) -> int | None:
    """Device pointer of a torch tensor (None for None)."""
    return None if t is None else t.data_ptr()


def stream_handle(device) -> int:
    import torch
    return torch.cuda.current_stream(device).cuda_stream
