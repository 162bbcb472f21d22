"""ctypes binding of libcomet_hip.so (include/comet_hip.h).

The product path has no fallback: if the library is missing or fails to load, every op raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# COMET_DEBUG=1 selects the `make DEBUG=1` library (a synchronise + device index-check read after
# every launch; comet_amd/debug.py); COMET_HIP_LIB names any other build explicitly
_DEFAULT_LIB = "libcomet_hip_debug.so" if os.environ.get("COMET_DEBUG") == "1" else "libcomet_hip.so"
LIB_PATH = os.environ.get("COMET_HIP_LIB", os.path.join(os.path.dirname(_HERE), _DEFAULT_LIB))

F32 = 0
BF16 = 1
ACT_NONE, ACT_GELU, ACT_RELU, ACT_SIGMOID = 0, 1, 2, 3
SQ_NORM_PARTIALS = 1024  # COMET_SQ_NORM_PARTIALS: scratch floats of comet_sq_norm_multi

c_i64 = ctypes.c_int64
c_i32 = ctypes.c_int32
c_vp = ctypes.c_void_p


class GemmArgs(ctypes.Structure):
    _fields_ = [
        ("dtype_ab", c_i32), ("dtype_c", c_i32), ("layout_a", c_i32), ("layout_b", c_i32),
        ("m", c_i64), ("n", c_i64), ("k", c_i64), ("batch", c_i64 * 2),
        ("a", c_vp), ("lda", c_i64), ("stride_a", c_i64 * 2),
        ("b", c_vp), ("ldb", c_i64), ("stride_b", c_i64 * 2),
        ("c", c_vp), ("ldc", c_i64), ("stride_c", c_i64 * 2),
        ("bias", c_vp), ("bias_mode", c_i32), ("stride_bias", c_i64 * 2),
        ("resid", c_vp), ("ldr", c_i64), ("stride_r", c_i64 * 2),
        ("aux", c_vp), ("ldaux", c_i64), ("stride_aux", c_i64 * 2),
        ("alpha", ctypes.c_float), ("beta", ctypes.c_float), ("act", c_i32),
        ("workspace", c_vp), ("workspace_bytes", c_i64), ("split_k", c_i32),
        ("convert_a", c_i32), ("convert_b", c_i32),
    ]


class RowLNArgs(ctypes.Structure):
    _fields_ = [
        ("y16", c_vp), ("ldy", c_i64), ("eps_y", ctypes.c_float),
        ("z16", c_vp), ("ldz", c_i64), ("zw", c_vp), ("zb", c_vp), ("eps_z", ctypes.c_float),
        ("raw_c", c_i32),
    ]


class ConvArgs(ctypes.Structure):
    _fields_ = [
        ("dtype", c_i32), ("dtype_y", c_i32),
        ("x", c_vp), ("n", c_i64), ("h", c_i64), ("w", c_i64), ("c", c_i64),
        ("weight", c_vp), ("cout", c_i64), ("ldw", c_i64),
        ("kh", c_i32), ("kw", c_i32), ("stride", c_i32), ("pad", c_i32),
        ("bias", c_vp),
        ("y", c_vp), ("ldy", c_i64),
        ("resid", c_vp), ("ldr", c_i64), ("beta", ctypes.c_float),
        ("act", c_i32),
    ]


class AttnArgs(ctypes.Structure):
    _fields_ = [
        ("dtype", c_i32), ("head_dim", c_i32),
        ("batch", c_i64), ("heads", c_i64), ("lq", c_i64), ("lk", c_i64),
        ("q", c_vp), ("sq_b", c_i64), ("sq_h", c_i64), ("sq_l", c_i64),
        ("k", c_vp), ("sk_b", c_i64), ("sk_h", c_i64), ("sk_l", c_i64),
        ("v", c_vp), ("sv_b", c_i64), ("sv_h", c_i64), ("sv_l", c_i64),
        ("o", c_vp), ("so_b", c_i64), ("so_h", c_i64), ("so_l", c_i64),
        ("lse", c_vp), ("scale", ctypes.c_float),
        ("batch_inner", c_i64), ("sq_i", c_i64), ("sk_i", c_i64), ("sv_i", c_i64), ("so_i", c_i64),
    ]


class AttnBwdArgs(ctypes.Structure):
    _fields_ = [
        ("dtype", c_i32), ("head_dim", c_i32),
        ("batch", c_i64), ("heads", c_i64), ("lq", c_i64), ("lk", c_i64),
        ("q", c_vp), ("sq_b", c_i64), ("sq_h", c_i64), ("sq_l", c_i64),
        ("k", c_vp), ("sk_b", c_i64), ("sk_h", c_i64), ("sk_l", c_i64),
        ("v", c_vp), ("sv_b", c_i64), ("sv_h", c_i64), ("sv_l", c_i64),
        ("o", c_vp), ("so_b", c_i64), ("so_h", c_i64), ("so_l", c_i64),
        ("dout", c_vp), ("sd_b", c_i64), ("sd_h", c_i64), ("sd_l", c_i64),
        ("dq", c_vp), ("sdq_b", c_i64), ("sdq_h", c_i64), ("sdq_l", c_i64),
        ("dk", c_vp), ("sdk_b", c_i64), ("sdk_h", c_i64), ("sdk_l", c_i64),
        ("dv", c_vp), ("sdv_b", c_i64), ("sdv_h", c_i64), ("sdv_l", c_i64),
        ("lse", c_vp), ("delta", c_vp), ("scale", ctypes.c_float),
    ]


# (name, restype, argtypes); every exported symbol of include/comet_hip.h
_F = ctypes.c_float
_INT = ctypes.c_int
SIGNATURES = {
    "comet_count_nonfinite": (_INT, [_INT, c_vp, c_i64, c_vp, c_vp]),
    "comet_debug_flags": (_INT, [_INT]),
    "comet_lds_probe": (_INT, [_INT, _INT, _INT, c_vp, c_vp]),
    "comet_shfl_probe": (_INT, [_INT, _INT, _INT, c_vp, c_vp]),
    "comet_version": (_INT, []),
    "comet_last_error": (ctypes.c_char_p, []),
    "comet_gemm": (_INT, [ctypes.POINTER(GemmArgs), c_vp]),
    "comet_gemm_workspace": (_INT, [ctypes.POINTER(GemmArgs), ctypes.POINTER(c_i64)]),
    "comet_gemm_plan": (_INT, [ctypes.POINTER(GemmArgs), ctypes.POINTER(c_i64), ctypes.POINTER(ctypes.c_int32)]),
    "comet_gemm_rowln_ok": (_INT, [ctypes.POINTER(GemmArgs)]),
    "comet_gemm_rowln_workspace": (_INT, [ctypes.POINTER(GemmArgs), ctypes.POINTER(ctypes.c_int64)]),
    "comet_gemm_rowln": (_INT, [ctypes.POINTER(GemmArgs), ctypes.POINTER(RowLNArgs), c_vp]),
    "comet_gemm_dact_ok": (_INT, [ctypes.POINTER(GemmArgs), _INT, c_vp, c_i64]),
    "comet_gemm_dact": (_INT, [ctypes.POINTER(GemmArgs), _INT, c_vp, c_i64, c_vp, c_vp]),
    "comet_conv2d_nhwc": (_INT, [ctypes.POINTER(ConvArgs), c_vp]),
    "comet_layernorm_fwd": (_INT, [_INT, _INT, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64,
                                   c_i64, _F, _INT, c_vp]),
    "comet_layernorm_bwd": (_INT, [_INT, _INT, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, _INT, c_vp, c_vp, c_vp, c_i64, c_i64,
                                   _INT, c_vp]),
    "comet_layernorm_bwd_res": (_INT, [_INT, _INT, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64,
                                       c_vp]),
    "comet_attention_bwd": (_INT, [ctypes.POINTER(AttnBwdArgs), c_vp]),
    "comet_attention_fwd": (_INT, [ctypes.POINTER(AttnArgs), c_vp]),
    "comet_attn_probs": (_INT, [_INT, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, _F, c_vp]),
    "comet_attn_delta": (_INT, [_INT, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp]),
    "comet_attn_dsoftmax": (_INT, [_INT, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, _F, c_vp]),
    "comet_cast": (_INT, [_INT, _INT, c_vp, c_vp, c_i64, c_vp]),
    "comet_cast_multi_f32_bf16": (_INT, [c_vp, c_vp, c_vp, _INT, c_vp]),
    "comet_act_bwd": (_INT, [_INT, _INT, _INT, c_vp, c_vp, c_vp, _INT, c_i64, c_vp]),
    "comet_axpby": (_INT, [c_vp, c_vp, _F, _F, c_i64, c_vp]),
    "comet_act_bwd_colsum": (_INT, [_INT, _INT, c_vp, _INT, c_vp, _INT, c_vp, c_vp, c_i64, c_i64, _INT, c_vp]),
    "comet_colsum": (_INT, [_INT, c_vp, c_vp, c_i64, c_i64, c_i64, _INT, c_vp]),
    "comet_sq_norm_multi": (_INT, [c_vp, c_vp, _INT, c_vp, c_vp, c_vp]),
    "comet_adamw_multi": (_INT, [c_vp, c_vp, c_vp, c_vp, c_vp, _INT, _F, _F, _F, _F, _F, _INT, c_vp, _F, c_vp]),
    "comet_im2col_nhwc": (_INT, [_INT, _INT, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, _INT, _INT, _INT, _INT, c_i64, c_i64, c_i64, c_vp]),
    "comet_instnorm_workspace": (_INT, [c_i64, c_i64, c_i64, ctypes.POINTER(c_i64)]),
    "comet_instnorm_nhwc": (_INT, [_INT, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, _F, _INT, _INT, c_vp, c_i64, c_vp]),
    "comet_resize_bilinear": (_INT, [_INT, _INT, _INT, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, _INT, c_vp]),
    "comet_resize_bilinear_pool_nhwc": (_INT, [_INT, _INT, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp]),
    "comet_conv1x1_resize_pool_nhwc": (_INT, [c_vp, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp,
                                               c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp]),
    "comet_resize_bilinear_nhwc_into": (_INT, [_INT, _INT, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64,
                                               _INT, c_vp]),
    "comet_act_fwd": (_INT, [_INT, _INT, _INT, c_vp, c_vp, c_i64, c_vp]),
    "comet_binary": (_INT, [_INT, _INT, c_vp, c_vp, c_vp, c_i64, c_vp]),
    "comet_add_rows": (_INT, [_INT, _INT, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp]),
    "comet_rowscale_fwd": (_INT, [_INT, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp]),
    "comet_rowscale_bwd": (_INT, [_INT, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp]),
    "comet_sincos_table": (_INT, [c_vp, c_vp, c_i64, _INT, c_i64, c_i64, c_vp]),
    "comet_harmonic_fwd": (_INT, [c_vp, c_vp, c_vp, c_vp, c_i64, _INT, _INT, _INT, c_vp]),
    "comet_pose_pair_errors": (_INT, [c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp]),
    "comet_pose_frame_errors": (_INT, [c_vp, c_i64, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "comet_harmonic_bwd": (_INT, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, _INT, _INT, _INT, c_vp]),
    "comet_pose_encode": (_INT, [c_vp, c_vp, c_vp, ctypes.c_double, c_vp, c_vp, c_i64, _INT, c_vp]),
    "comet_pose_decode": (_INT, [c_vp, c_vp, c_vp, ctypes.c_double, c_vp, ctypes.c_double, ctypes.c_double,
                                 ctypes.c_double, ctypes.c_double, c_vp, c_vp, c_i64, _INT, c_vp]),
    "comet_pose_encode3": (_INT, [c_vp, c_vp, c_vp, c_i64, _INT, c_vp]),
    "comet_pose_decode3": (_INT, [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, _INT, c_vp]),
    "comet_resample_coeffs": (_INT, [_INT, _F, _F, _INT, c_vp, c_vp, _INT, ctypes.POINTER(_INT)]),
    "comet_lanczos_crop_resize": (_INT, [c_vp, c_i64, _INT, _INT, c_i64, _INT, _INT, _INT, _INT, _INT, _INT, c_vp, c_vp,
                                         _INT, c_vp, c_vp, _INT, _INT, _INT, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "comet_sp_preprocess": (_INT, [_INT, c_vp, c_vp, _INT, _INT, _INT, _INT, _INT, _INT, c_vp]),
    "comet_maxpool2_nhwc": (_INT, [_INT, c_vp, c_vp, c_i64, _INT, _INT, _INT, c_vp]),
    "comet_sp_scores": (_INT, [c_vp, c_vp, _INT, _INT, _INT, c_vp]),
    "comet_maxfilt2d": (_INT, [c_vp, c_vp, c_vp, _INT, _INT, _INT, _INT, c_vp]),
    "comet_gapr_fwd": (_INT, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, _INT, _INT, _F, _F, c_vp]),
    "comet_gapr_bwd": (_INT, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, _INT, _INT,
                              _F, _F, c_vp]),
    "comet_sample_bilinear": (_INT, [_INT, c_vp, c_i64, _INT, _INT, _INT, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64,
                                     c_i64, c_i64, _INT, c_vp]),
    "comet_corr_sample": (_INT, [_INT, _INT, c_vp, c_vp, c_vp, _INT, _INT, _INT, c_vp, c_vp, c_vp, c_i64, c_i64,
                                 c_i64, c_i64, _INT, c_vp]),
    "comet_tracker_tokens": (_INT, [_INT, c_vp, c_vp, _INT, c_vp, c_i64, _INT, c_vp, _INT, c_vp, c_i64, c_i64, _INT, c_vp]),
    "comet_coords_update": (_INT, [_INT, c_vp, c_vp, c_i64, c_vp, _F, c_i64, c_i64, _INT, c_vp]),
    "comet_avgpool2_nhwc": (_INT, [_INT, c_vp, c_vp, c_i64, _INT, _INT, _INT, c_vp]),
    "comet_patch_gather": (_INT, [_INT, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, _INT, c_i64, _INT, _INT, _INT, _INT, c_vp]),
    "comet_images_nhwc": (_INT, [_INT, c_vp, c_vp, c_i64, _INT, _INT, _INT, _INT, _INT, c_vp]),
    "comet_refine_combine": (_INT, [c_vp, c_vp, c_vp, c_vp, c_i64, _INT, c_i64, c_vp]),
    "comet_track_score": (_INT, [_INT, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, _INT, c_i64, _INT, _INT, _INT, c_vp]),
    "comet_dino_prep": (_INT, [_INT, c_vp, c_vp, c_i64, _INT, _INT, _INT, _INT, c_i64, c_vp, c_vp, c_vp]),
}

_lib = None


class CometHipError(RuntimeError):
    pass


def load():
    """Load libcomet_hip.so once; raise (never fall back) if it is unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.isfile(LIB_PATH):
        raise CometHipError(
            f"libcomet_hip.so not found at {LIB_PATH}: build it with `make -C comet-pose-estimation_amd` "
            "(or __graft_entry__.build()); there is no CPU fallback")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc, what=""):
    if rc != 0:
        msg = load().comet_last_error()
        raise CometHipError(f"{what}: {msg.decode() if msg else 'error'} (code {rc})")
