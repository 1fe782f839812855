"""ctypes binding of ``librepurpose_amd.so`` (C ABI declared in ``include/rp_api.h``).

The library is built in-tree by ``make`` (or ``__graft_entry__.build()``) with
``hipcc --offload-arch=gfx950``.  There is no CPU fallback anywhere in the product path: if the
library cannot be loaded, every kernel call raises ``RuntimeError``.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("REPURPOSE_AMD_LIB", os.path.join(_HERE, "_native", "librepurpose_amd.so"))

RP_OK, RP_ERR_ARG, RP_ERR_LAUNCH = 0, 1, 2
RP_F32, RP_BF16, RP_F16, RP_F64, RP_I64 = 0, 1, 2, 3, 4

c_i64 = ctypes.c_int64
c_vp = ctypes.c_void_p
c_f = ctypes.c_float
c_i = ctypes.c_int
c_u32 = ctypes.c_uint32


class GemmEpilogue(ctypes.Structure):
    _fields_ = [("bias", c_vp), ("relu", c_i), ("dropout_p", c_f), ("dropout_seed", c_u32),
                ("residual", c_vp), ("ldr", c_i64), ("gate", c_vp), ("gate_dtype", c_i),
                ("ldg", c_i64), ("gate_scale", c_f), ("accumulate", c_i), ("col_scale_n", c_i64),
                ("col_scale", c_f), ("seed_base", c_vp)]


class LnFwdArgs(ctypes.Structure):
    _fields_ = [("x", c_vp), ("x_dtype", c_i), ("ldx", c_i64), ("gamma", c_vp), ("beta", c_vp),
                ("eps", c_f), ("pe", c_vp), ("pe_period", c_i64), ("relu", c_i), ("dropout_p", c_f),
                ("dropout_seed", c_u32), ("out_f32", c_vp), ("ld_out_f32", c_i64), ("out_lp", c_vp),
                ("out_lp_dtype", c_i), ("ld_out_lp", c_i64), ("mean", c_vp), ("rstd", c_vp), ("seed_base", c_vp)]


class LnBwdArgs(ctypes.Structure):
    _fields_ = [("dy", c_vp), ("dy_dtype", c_i), ("lddy", c_i64), ("x", c_vp), ("x_dtype", c_i),
                ("ldx", c_i64), ("mean", c_vp), ("rstd", c_vp), ("gamma", c_vp), ("y", c_vp),
                ("y_dtype", c_i), ("ldy", c_i64), ("dropout_p", c_f), ("dropout_seed", c_u32),
                ("dres", c_vp), ("lddres", c_i64), ("dx_f32", c_vp), ("lddx", c_i64), ("dx_lp", c_vp),
                ("dx_lp_dtype", c_i), ("lddx_lp", c_i64), ("dx_lp_dropout_p", c_f),
                ("dx_lp_seed", c_u32), ("dgamma_part", c_vp), ("dbeta_part", c_vp),
                ("ld_part", c_i64), ("seed_base", c_vp)]


class MhaGeneralArgs(ctypes.Structure):
    _fields_ = [("q", c_vp), ("ldq", c_i64), ("k", c_vp), ("ldk", c_i64), ("v", c_vp), ("ldv", c_i64), ("B", c_i),
                ("Tq", c_i), ("Tk", c_i), ("H", c_i), ("head_dim", c_i), ("scale", c_f), ("mask", c_vp),
                ("mask_sb", c_i64), ("mask_sh", c_i64), ("mask_sq", c_i64), ("mask_sk", c_i64), ("probs", c_vp),
                ("out", c_vp), ("ldo", c_i64), ("dout", c_vp), ("lddo", c_i64), ("dscores", c_vp), ("dq", c_vp),
                ("lddq", c_i64), ("dk", c_vp), ("lddk", c_i64), ("dv", c_vp), ("lddv", c_i64)]


class GemmLnArgs(ctypes.Structure):
    _fields_ = [("A", c_vp), ("lda", c_i64), ("W", c_vp), ("ldw", c_i64), ("bias", c_vp), ("dropout_p", c_f),
                ("dropout_seed", c_u32), ("seed_base", c_vp), ("residual", c_vp), ("ldr", c_i64), ("x_out", c_vp),
                ("ldx_out", c_i64), ("gamma", c_vp), ("beta", c_vp), ("eps", c_f), ("h_out", c_vp), ("ldh", c_i64),
                ("mean", c_vp), ("rstd", c_vp), ("x", c_vp), ("ldx", c_i64), ("dres", c_vp), ("lddres", c_i64),
                ("dx", c_vp), ("lddx", c_i64), ("dx_lp", c_vp), ("lddx_lp", c_i64), ("lp_dropout_p", c_f),
                ("lp_seed", c_u32), ("dgamma_part", c_vp), ("dbeta_part", c_vp), ("ld_part", c_i64),
                ("xchg", c_vp)]


class WgradItem(ctypes.Structure):
    _fields_ = [("dY", c_vp), ("X", c_vp), ("dW", c_vp), ("db", c_vp), ("M", c_i64), ("N", c_i64), ("ldy", c_i64),
                ("ldx", c_i64)]


class SumsqItem(ctypes.Structure):
    _fields_ = [("x", c_vp), ("n", c_i64), ("out", c_vp)]


class ColsumItem(ctypes.Structure):
    _fields_ = [("X", c_vp), ("out", c_vp), ("rows", c_i64), ("cols", c_i64), ("ldx", c_i64), ("accumulate", c_i)]


class MhaArgs(ctypes.Structure):
    _fields_ = [("q", c_vp), ("ldq", c_i64), ("k", c_vp), ("ldk", c_i64), ("v", c_vp), ("ldv", c_i64),
                ("key_valid", c_vp), ("B", c_i), ("Tq", c_i), ("Tk", c_i), ("H", c_i), ("head_dim", c_i),
                ("scale", c_f), ("dropout_p", c_f), ("seed", c_u32), ("out", c_vp), ("ldo", c_i64), ("lse", c_vp),
                ("dropmask", c_vp), ("dout", c_vp), ("lddo", c_i64), ("dq", c_vp), ("lddq", c_i64), ("dk", c_vp),
                ("lddk", c_i64), ("dv", c_vp), ("lddv", c_i64), ("delta_ws", c_vp), ("out_lo", c_vp),
                ("empty_rows_uniform", c_i), ("seed_base", c_vp)]


# name -> (restype, argtypes); mirrors include/rp_api.h one to one
_SIGNATURES = {
    "rp_version": (c_i, []),
    "rp_last_error": (c_i, [ctypes.c_char_p, ctypes.c_size_t]),
    "rp_concat_rows": (c_i, [c_vp, c_i, c_vp, c_i, c_vp, c_i, c_i64, c_vp, c_i, c_vp]),
    "rp_cast_f32_to_bf16": (c_i, [c_vp, c_vp, c_i64, c_vp]),
    "rp_gemm": (c_i, [c_i, c_i64, c_i64, c_i64, c_vp, c_i64, c_i, c_vp, c_i64, c_i, c_vp, c_i64, c_i,
                      c_f, ctypes.POINTER(GemmEpilogue), c_vp]),
    "rp_gemm_wgrad_workspace": (c_i64, [c_i64, c_i64, c_i64]),
    "rp_gemm_wgrad": (c_i, [c_i, c_i64, c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_i, c_vp, c_i64, c_vp]),
    "rp_gemm_wgrad_grouped": (c_i, [c_i64, c_vp, c_i, c_i, c_vp]),
    "rp_gemm_ln_fwd": (c_i, [c_i64, c_i64, ctypes.POINTER(GemmLnArgs), c_vp]),
    "rp_gemm_ln_bwd": (c_i, [c_i64, c_i64, ctypes.POINTER(GemmLnArgs), c_vp]),
    "rp_gemm_ln_xchg_bytes": (c_i64, [c_i64]),
    "rp_gemm_ln_status": (c_i, []),
    "rp_gemm_ln_reset": (c_i, [c_vp, c_i64, c_vp]),
    "rp_debug_gemm_ln_partial": (c_i, [c_i, c_i64, c_i64, ctypes.POINTER(GemmLnArgs), c_i64, ctypes.c_double, c_vp]),
    "rp_debug_occupy": (c_i, [c_i, c_i, c_vp]),
    "rp_debug_set_lnx_rows": (c_i, [c_i]),
    "rp_layernorm_fwd": (c_i, [c_i64, c_i64, ctypes.POINTER(LnFwdArgs), c_vp]),
    "rp_layernorm_bwd_blocks": (c_i64, [c_i64]),
    "rp_layernorm_bwd": (c_i, [c_i64, c_i64, ctypes.POINTER(LnBwdArgs), c_vp]),
    "rp_colsum_workspace": (c_i64, [c_i64, c_i64]),
    "rp_colsum_batched": (c_i, [c_vp, c_i, c_vp]),
    "rp_sumsq_batched": (c_i, [c_vp, c_i, c_vp]),
    "rp_colsum": (c_i, [c_vp, c_i, c_i64, c_i64, c_i64, c_vp, c_vp, c_i, c_vp, c_vp]),
    "rp_attn_dropmask_elems": (c_i64, [c_i, c_i, c_i]),
    "rp_attn_fwd": (c_i, [c_i, c_vp, c_vp, c_i, c_i, c_i, c_i, c_f, c_f, c_u32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "rp_attn_bwd_uses_roles": (c_i, [c_i, c_i, c_i, c_i, c_i]),
    "rp_attn_bwd_given_delta": (c_i, [c_i, c_vp, c_vp, c_vp, c_vp, c_vp, c_i, c_i, c_i, c_i, c_f, c_f, c_vp, c_vp,
                                      c_vp]),
    "rp_gemm_attn_dout_delta": (c_i, [c_vp, c_i64, c_vp, c_i64, c_i64, c_i64, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp,
                                      c_i, c_i, c_i, c_f, c_vp, c_vp]),
    "rp_attn_bwd": (c_i, [c_i, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i, c_i, c_i, c_i, c_f, c_f, c_vp,
                          c_vp, c_vp, c_vp]),
    "rp_attn_bwd_delta": (c_i, [c_i, c_vp, c_vp, c_vp, c_vp, c_i, c_i, c_i, c_i, c_f, c_vp, c_vp]),
    "rp_attn_bwd_dkdv": (c_i, [c_i, c_vp, c_vp, c_vp, c_vp, c_vp, c_i, c_i, c_i, c_i, c_f, c_f, c_vp, c_vp, c_vp]),
    "rp_attn_bwd_dq_delta": (c_i, [c_i, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i, c_i, c_i, c_i, c_f, c_f, c_vp,
                                   c_vp, c_vp]),
    "rp_attn_bwd_dq": (c_i, [c_i, c_vp, c_vp, c_vp, c_vp, c_vp, c_i, c_i, c_i, c_i, c_f, c_f, c_vp, c_vp, c_vp]),
    "rp_mha_dropmask_elems": (c_i64, [c_i, c_i, c_i, c_i]),
    "rp_mha_fwd": (c_i, [c_i, ctypes.POINTER(MhaArgs), c_vp]),
    "rp_mha_general_fwd": (c_i, [ctypes.POINTER(MhaGeneralArgs), c_vp]),
    "rp_mha_general_bwd": (c_i, [ctypes.POINTER(MhaGeneralArgs), c_vp]),
    "rp_mha_bwd": (c_i, [c_i, ctypes.POINTER(MhaArgs), c_i, c_vp]),
    "rp_pad_rows": (c_i, [c_vp, c_i, c_vp, c_i, c_i, c_i, c_f, c_vp, c_vp]),
    "rp_tiou_hits": (c_i, [c_vp, c_vp, c_i, c_vp, c_vp, c_i, c_vp, c_i, c_i, c_vp, c_vp]),
    "rp_diou_fwd": (c_i, [c_vp, c_vp, c_i64, c_f, c_i, c_vp, c_vp]),
    "rp_diou_bwd": (c_i, [c_vp, c_vp, c_i64, c_f, c_vp, c_i, c_f, c_vp, c_vp, c_vp]),
    "rp_focal_fwd_sum": (c_i, [c_vp, c_vp, c_vp, c_i64, c_f, c_f, c_vp, c_vp]),
    "rp_focal_ws_elems": (c_i64, [c_i64]),
    "rp_focal_fwd_sum_ws": (c_i, [c_vp, c_vp, c_vp, c_i64, c_f, c_f, c_vp, c_i64, c_vp, c_vp]),
    "rp_focal_elementwise": (c_i, [c_vp, c_vp, c_i64, c_f, c_f, c_vp, c_vp]),
    "rp_focal_bwd": (c_i, [c_vp, c_vp, c_vp, c_i64, c_f, c_f, c_vp, c_i, c_vp, c_vp]),
    "rp_rowdot_fwd": (c_i, [c_i, c_vp, c_i64, c_i64, c_i, c_vp, c_vp, c_i, c_i, c_vp, c_i64, c_vp]),
    "rp_rowdot_bwd_dx": (c_i, [c_vp, c_i64, c_i64, c_i, c_vp, c_i, c_vp, c_i, c_i64, c_f, c_vp, c_i,
                               c_i64, c_vp]),
    "rp_adam_step": (c_i, [c_vp, c_vp, c_vp, c_vp, c_i64, c_f, c_f, c_f, c_f, c_f, c_i, c_vp, c_vp]),
    "rp_adam_coefficients": (c_i, [c_f, c_f, c_f, c_f, c_f, c_i, c_vp]),
    "rp_adam_step_dev": (c_i, [c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp]),
    "rp_infer_select": (c_i, [c_vp, c_vp, c_vp, c_i, c_i, c_f, c_i, c_f, c_f, c_vp, c_vp, c_vp, c_vp,
                              c_vp]),
    "rp_softnms_workspace": (c_i64, [c_i, c_i]),
    "rp_softnms": (c_i, [c_vp, c_vp, c_vp, c_i, c_i, c_f, c_f, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp]),
}

EXPORTED = tuple(_SIGNATURES)

_lib = None
_load_error = None


def load(path=None):
    """Load (once) and return the native library; raises RuntimeError if it is missing."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    p = path or os.environ.get("RP_LIB_PATH") or LIB_PATH  # RP_LIB_PATH: A/B builds for tuning
    try:
        lib = ctypes.CDLL(p)
    except OSError as e:  # no silent fallback: the HIP library is the product
        _load_error = e
        raise RuntimeError(f"repurpose_amd: cannot load HIP library {p!r} ({e}); build it with "
                           f"`make -C {os.path.dirname(_HERE)}` or __graft_entry__.build()") from e
    for name, (res, args) in _SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def last_error():
    buf = ctypes.create_string_buffer(1024)
    load().rp_last_error(buf, len(buf))
    return buf.value.decode(errors="replace")


def call(name, *args):
    """Call an rp_* entry point and raise RuntimeError(rp_last_error) on a non-zero status."""
    rc = getattr(load(), name)(*args)
    if rc != RP_OK:
        raise RuntimeError(f"{name} failed ({rc}): {last_error()}")
    return rc
