"""ctypes binding of libavdino.so (include/avdino.h).

There is no fallback: if the shared library is missing or was built for another
architecture, importing this module raises, so nothing can silently run a CPU path.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("AVDINO_LIB", os.path.join(_HERE, "libavdino.so"))

F32, BF16 = 0, 1

P = ctypes.c_void_p
I = ctypes.c_int
L = ctypes.c_longlong
F = ctypes.c_float
U64 = ctypes.c_ulonglong
D = ctypes.c_double

# name -> argtypes (restype is always c_int except where noted)
PROTOS = {
    "avd_version": [],
    "avd_set_options": [P],
    "avd_get_options": [P],
    "avd_bn_finalize": [P, I, I, I, L, P, P, F, F, P, P, P, P, P, P, P, I, P],
    "avd_bn_bwd_finalize": [P, I, I, I, L, P, P, P, P, P, P, P, I, P],
    "avd_gemm": [I, I, I, P, L, L, P, L, L, P, L, P, F, F, I, P, L, P],
    "avd_gemm_ws_elems": [I, I, I, I],
    "avd_linear_bwd": [I, I, I, P, L, P, L, P, P, P, L, P, I, I, P, L, P],
    "avd_linear_bwd_ws_elems": [I, I, I, I],
    "avd_linear_hwc_ws_elems": [I, I, I],
    "avd_linear_weight_hwc": [I, P, P, P, P, P, P],
    "avd_linear_fwd_hwc": [I, I, I, I, P, P, P, P, L, P, L, P],
    "avd_linear_bwd_hwc": [I, I, I, I, P, L, P, P, P, P, P, I, P, L, P],
    "avd_cl_weight_elems": [I, I, I, I],
    "avd_cl_weight_layout": [P, P, I, I, I, I, I, P],
    "avd_cl_weight_layout_batch": [I, P, P, P, P, P, P, I, P],
    "avd_cl_stat_rows": [I, I, I, I, I, I, I],
    "avd_cl_conv_fwd": [P, P, P, P, P, I, I, I, I, I, I, I, I, I, P],
    "avd_cl_stat_pivot": [I, I, I, I, I, I, I],
    "avd_cl_conv_fwd_pv": [P, P, P, P, P, P, I, I, I, I, I, I, I, I, I, P],
    "avd_cl_conv_dgrad": [P, P, P, I, I, I, I, I, I, I, I, P],
    "avd_cl_wgrad_chunks": [I, I, I, I],
    "avd_cl_conv_wgrad": [P, P, I, P, I, I, I, I, I, I, I, P],
    "avd_cl_bn_bwd_reduce_pooled": [P, I, P, P, I, P, P, P, P, P, I, I, I, I, I, P],
    "avd_cl_c1_moment_cols": [I, I],
    "avd_cl_c1_codes_rows": [I, I, I, I],
    "avd_cl_c1_codes_cols": [],
    "avd_cl_c1_apply_codes": [P, P, P, P, P, P, P, I, I, I, I, P],
    "avd_cl_c1_moments_codes": [P, P, P, P, I, I, I, I, P],
    "avd_cl_c1_codes_combine": [P, P, P, P, P, P, L, P, P, P, P, P, I, P],
    "avd_cl_c1r5_codes_rows": [I, I, I, I],
    "avd_cl_c1r5_codes_cols": [],
    "avd_cl_c1r5_apply_codes": [P, P, P, P, P, P, P, I, I, I, I, P],
    "avd_cl_c1r5_stats_rows": [I, I, I, I],
    "avd_cl_c1r5_stats": [P, P, P, P, I, I, I, I, P],
    "avd_cl_c1r5_moments_codes": [P, P, P, P, I, I, I, I, P],
    "avd_cl_c1r5_codes_combine": [P, P, P, P, P, P, L, P, P, P, P, P, I, P],
    "avd_counters_add": [P, P, P, I, P],
    "avd_mark": [P, I, P],
    "avd_mark_span": [P, I, I, P],
    "avd_cl_bn_relu_pool": [P, I, P, P, P, I, I, I, I, I, I, P],
    "avd_cl_bn_bwd_rows": [I, I, I, I, I],
    "avd_cl_bn_bwd_reduce": [P, I, P, I, P, P, P, P, P, I, I, I, I, I, P],
    "avd_cl_bn_bwd_apply": [P, I, P, I, P, P, P, P, I, I, I, I, I, P],
    "avd_cl_apply_wgrad_slabs": [I, I, I, I, I, I, I, I],
    "avd_cl_c1_recompute_rows": [I, I, I, I, I, I, I, I, I, I],
    "avd_cl_c1_recompute": [I, P, P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, I, I, I, I, P],
    "avd_cl_c1_recompute_combine": [P, P, P, P, P, I, I, I, P],
    "avd_cl_bn_bwd_apply_wgrad": [P, P, P, P, P, P, P, I, I, I, I, I, I, I, I, I, P],
    "avd_lds_poison": [P],
    "avd_xent_fused_ws": [I, I, I],
    "avd_xent_fused": [P, P, I, I, I, I, I, I, I, I, F, F, P, P, P, P, L, P],
    "avd_cl_layer_bwd_slabs": [I, I, I, I, I, I, I, I],
    "avd_cl_layer_bwd": [P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, P],
    "avd_sum_rows": [P, I, I, L, P, I, P],
    "avd_sum_rows_chunks": [I, I],
    "avd_sum_rows_split": [P, I, I, L, P, I, P, L, P],
    "avd_colstats_parts": [I],
    "avd_colstats": [P, I, I, I, P, P, P],
    "avd_act_fwd": [P, P, I, P, P, I, I, I, F, U64, P],
    "avd_act_bwd": [P, P, P, I, P, P, I, I, I, F, U64, P],
    "avd_act_fwd_dev": [P, P, I, P, P, I, I, I, F, U64, P, P],
    "avd_act_bwd_dev": [P, P, P, I, P, P, I, I, I, F, U64, P, P],
    "avd_step_begin": [P, P, P, D, D, U64, P],
    "avd_adam_dev": [P, P, P, P, L, P, F, F, F, F, P],
    "avd_adamw_dev": [P, P, P, P, L, P, F, F, F, F, P],
    "avd_bn1d_bwd_reduce": [P, P, P, P, I, I, I, P, P],
    "avd_bn1d_act_bwd_reduce": [P, P, P, P, P, P, P, I, I, I, F, U64, P, P, P],
    "avd_bn1d_bwd_apply": [P, P, P, P, I, I, I, P],
    "avd_dino_loss": [P, P, P, I, I, I, I, F, F, F, I, P, P, P, P, P],
    "avd_mse_loss": [P, P, I, I, P, P, P, P],
    "avd_l2norm_fwd": [P, P, P, I, I, P],
    "avd_l2norm_bwd": [P, P, P, P, I, I, P],
    "avd_softmax_xent": [P, L, I, I, P, I, I, I, I, F, P, P, L, I, P],
    "avd_cosine_consistency": [P, I, I, I, F, P, P, P],
    "avd_ema": [P, P, L, F, P],
    "avd_adam": [P, P, P, P, L, F, F, F, F, F, F, F, P],
    "avd_adamw": [P, P, P, P, L, F, F, F, F, F, F, F, P],
    "avd_axpy": [P, P, L, F, P],
    "avd_bn_eval_coef": [P, P, P, P, F, I, P, P, P],
    "avd_argmax_correct": [P, L, I, I, P, P, P],
    "avd_sum": [P, I, F, P, P],
    "avd_stage_views": [P, I, P, I, P, I, I, P, I, P],
    "avd_augment_views": [P, P, L, I, I, I, I, P, P, P, I, I, U64, I, P, P],
    "avd_augment_views_dt": [P, P, L, I, I, I, I, P, P, P, I, I, U64, I, P, I, P],
    "avd_augment_views_lds_check": [P, P, I, I, I, I, P, P, P, I, I, U64, I, P, P, P, P],
    "avd_augment_views_nolds": [P, P, I, I, I, I, P, P, P, I, I, U64, I, P, P],
    "avd_augment_views_seq": [P, P, L, I, I, I, I, P, P, P, I, I, U64, I, P, I, P, I, P],
    "avd_augment_records": [P, I, I, I, I, I, U64, P, P, I, P],
    "avd_row_sqnorm": [P, I, I, P, P],
    "avd_knn_select": [P, L, P, I, I, I, P, P, I, P, I, P, P, P],
    "avd_argmax_rows": [P, L, I, I, P, P],
    "avd_cl_c1_gram_cols": [],
    "avd_cl_c1_gram": [P, P, I, I, I, I, P],
    "avd_cl_c1_gram_finalize": [P, P, P, P, P, L, F, F, P, P, P, P, P, P, I, P],
    "avd_cl_c1_moments_codes_ng": [P, P, P, P, I, I, I, I, P],
    "avd_cl_c1_codes_combine_gram": [P, P, P, P, P, P, P, L, P, P, P, P, P, I, P],
    "avd_cl_c1r3_codes_rows": [I, I, I, I, I],
    "avd_cl_c1r3_codes_cols": [I],
    "avd_cl_c1r3_apply_codes": [P, P, P, P, P, P, P, I, I, I, I, I, P],
    "avd_cl_c1r3_moments_codes": [P, P, P, P, P, I, I, I, I, I, P],
    "avd_cl_c1r3_codes_combine": [P, P, P, P, P, P, L, P, P, P, P, P, I, I, P],
    "avd_mx_weight_bytes": [I, I, I, I],
    "avd_mx_scale_bytes": [I, I, I, I],
    "avd_mx_weight_layout": [P, P, P, I, I, I, I, P],
    "avd_mx_weight_layout_batch": [I, P, P, P, P, P, P, P, P],
    "avd_mx_conv_serves": [I, I, I, I, I, I, I],
    "avd_mx_conv_ns": [I, I, I, I, I, I, I],
    "avd_mx_stat_rows": [I, I, I, I, I, I, I],
    "avd_mx_conv_fwd": [P, P, P, P, P, P, P, I, I, I, I, I, I, I, I, P],
    "avd_mx_conv_dgrad": [P, P, P, P, I, I, I, I, I, I, I, P],
    "avd_mx_wgrad_chunks": [I, I, I, I, I, I],
    "avd_mx_conv_wgrad": [P, P, P, I, I, I, I, I, I, I, P],
}


class AvdError(RuntimeError):
    pass


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libavdino.so not found at {LIB_PATH}: build it with "
            f"`make -C multimodal-ssl-avmnist_amd/csrc` (or __graft_entry__.build()). "
            f"There is no CPU fallback.")
    lib = ctypes.CDLL(LIB_PATH)
    for name, args in PROTOS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = ctypes.c_int
    lib.avd_gemm_ws_elems.restype = ctypes.c_longlong
    lib.avd_linear_hwc_ws_elems.restype = ctypes.c_longlong
    lib.avd_mx_weight_bytes.restype = ctypes.c_longlong
    lib.avd_mx_scale_bytes.restype = ctypes.c_longlong
    lib.avd_last_error.argtypes = []
    lib.avd_last_error.restype = ctypes.c_char_p
    return lib


lib = _load()

STATUS = {-1: "AVD_ERR_SHAPE", -2: "AVD_ERR_DTYPE", -3: "AVD_ERR_HIP", -4: "AVD_ERR_ARG"}


def check(rc, name="avd"):
    if rc != 0:
        msg = STATUS.get(rc, str(rc))
        if rc == -3:
            msg += f" ({lib.avd_last_error().decode()})"
        raise AvdError(f"{name} failed: {msg}")
    return rc


def call(name, *args):
    return check(getattr(lib, name)(*args), name)
