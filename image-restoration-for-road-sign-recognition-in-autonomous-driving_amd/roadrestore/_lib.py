"""ctypes binding of the gfx950 C-ABI library (include/roadrestore.h).

The library is built in-tree by ``__graft_entry__.build()`` (csrc/Makefile) and
loaded from this directory.  There is no fallback: if the library is missing
or a GPU is absent, every op raises.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# RR_LIB_PATH: load another build of the same ABI (A/B of two builds on one box)
LIB_PATH = os.environ.get("RR_LIB_PATH") or os.path.join(_HERE, "libroadrestore.so")



def path_flag(key: str, default: int) -> int:
    """The stack's one A/B and test knob, shared with the library
    (csrc/common.h rr_path): RR_PATH="key=value[,key=value...]".  Every
    default is the measured-best path; the Python schedule reads its fusion
    keys (fused_pool=0, split_dgrad=0, ...) once at import."""
    for item in os.environ.get("RR_PATH", "").split(","):
        k, sep, v = item.partition("=")
        if sep and k.strip() == key:
            return int(v)
    return default


RR_F32, RR_BF16 = 0, 1
RR_CONV3X3, RR_CONV1X1, RR_CONVT_UP, RR_CONVT_DOWN = 0, 1, 2, 3
RR_ACT_NONE, RR_ACT_RELU, RR_ACT_PRELU, RR_ACT_RES, RR_ACT_POOL, RR_ACT_NOFULL = 0, 1, 2, 4, 8, 16

_STATUS = {0: "ok", -1: "EINVAL", -2: "EUNSUPPORTED", -3: "ELAUNCH", -4: "EWORKSPACE"}
RR_EUNSUPPORTED = -2


class IgemmDesc(C.Structure):
    _fields_ = [(n, C.c_int32) for n in (
        "dtype", "mode", "n", "h", "w", "c_in1", "c_in2", "c_out", "out_split", "act",
        "accumulate", "has_bias", "has_mask", "want_stats", "out_nchw")]


class WgradDesc(C.Structure):
    _fields_ = [(n, C.c_int32) for n in (
        "dtype", "mode", "n", "h", "w", "c_in1", "c_in2", "c_out", "accumulate")]


class BnBwdDesc(C.Structure):
    _fields_ = [("dtype", C.c_int32), ("P", C.c_int64), ("C", C.c_int32),
                ("mask_kind", C.c_int32), ("nbn", C.c_int32), ("h", C.c_int32), ("w", C.c_int32),
                ("pool_dy", C.c_void_p), ("pool_idx", C.c_void_p), ("eval", C.c_int32),
                ("dbias0", C.c_void_p), ("dbias1", C.c_void_p)]


class DistortParam(C.Structure):
    _fields_ = [("sigma", C.c_double), ("fog_mul", C.c_float), ("fog_add", C.c_float),
                ("flags", C.c_int32), ("ksize", C.c_int32)]


class BnFinalizeDesc(C.Structure):          # mirrors rr_bn_finalize_desc
    _fields_ = [("C", C.c_int32), ("blocks", C.c_int32), ("count", C.c_int64),
                ("part", C.c_void_p), ("bias", C.c_void_p), ("gamma", C.c_void_p),
                ("beta", C.c_void_p), ("running_mean", C.c_void_p), ("running_var", C.c_void_p),
                ("momentum", C.c_float), ("eps", C.c_float), ("scale", C.c_void_p),
                ("shift", C.c_void_p), ("save_mean", C.c_void_p), ("save_invstd", C.c_void_p),
                ("num_batches_tracked", C.c_void_p)]


class PackJob(C.Structure):
    _fields_ = [("w", C.c_void_p), ("w_fwd", C.c_void_p), ("w_dgrad", C.c_void_p),
                ("c_out", C.c_int32), ("c_in", C.c_int32), ("k", C.c_int32), ("pad_", C.c_int32),
                ("begin", C.c_int64)]


RR_DISTORT_FOG, RR_DISTORT_NOISE, RR_DISTORT_BLUR = 1, 2, 4
RR_DISTORT_KMAX = 15

P_ = C.c_void_p
I_ = C.c_int
L_ = C.c_longlong
F_ = C.c_float
S_ = C.c_size_t

# name -> (restype, argtypes)
_SIGS = {
    "rr_igemm": (I_, [C.POINTER(IgemmDesc), P_, P_, P_, P_, P_, P_, P_, P_, P_]),
    "rr_igemm_ex": (I_, [C.POINTER(IgemmDesc), P_, P_, P_, P_, P_, P_, P_, P_, P_, P_, P_]),
    "rr_igemm_stat_blocks": (I_, [C.POINTER(IgemmDesc)]),
    "rr_igemm_kernel_name": (C.c_char_p, [C.POINTER(IgemmDesc), I_]),
    "rr_igemm_pool": (I_, [C.POINTER(IgemmDesc), P_, P_, P_, P_, P_, P_, P_]),
    "rr_igemm_pool_kernel_name": (C.c_char_p, [C.POINTER(IgemmDesc)]),
    "rr_igemm_dgrad_sc": (I_, [C.POINTER(IgemmDesc), P_, P_, P_, P_, I_, P_, P_]),
    "rr_igemm_dgrad_sc_kernel_name": (C.c_char_p, [C.POINTER(IgemmDesc), I_]),
    "rr_igemm_pre_ok": (I_, [C.POINTER(IgemmDesc)]),
    "rr_igemm_pre": (I_, [C.POINTER(IgemmDesc), P_, P_, P_, P_, P_, P_, P_, P_, P_]),
    "rr_wgrad_pre_ok": (I_, [C.POINTER(WgradDesc)]),
    "rr_wgrad_pre": (I_, [C.POINTER(WgradDesc), P_, P_, P_, P_, P_, P_, P_, S_, P_]),
    "rr_wgrad_kernel_name": (C.c_char_p, [C.POINTER(WgradDesc)]),
    "rr_igemm_bnbwd_workspace": (S_, [C.POINTER(IgemmDesc)]),
    "rr_igemm_bnbwd": (I_, [C.POINTER(IgemmDesc), P_, P_, P_, P_, P_, P_, P_, P_, P_, P_, P_]),
    "rr_wgrad_workspace": (S_, [C.POINTER(WgradDesc)]),
    "rr_wgrad": (I_, [C.POINTER(WgradDesc), P_, P_, P_, P_, P_, S_, P_]),
    "rr_wgrad_partial": (I_, [C.POINTER(WgradDesc), P_, P_, P_, P_, S_, P_]),
    "rr_wgrad_reduce": (I_, [C.POINTER(WgradDesc), P_, S_, P_, P_]),
    "rr_pack_conv": (I_, [I_, I_, I_, I_, P_, P_, P_, P_]),
    "rr_pack_conv_elems": (L_, [I_, I_, I_, I_]),
    "rr_pack_conv_batch": (I_, [I_, I_, P_, L_, P_]),
    "rr_pack_convT": (I_, [I_, I_, I_, P_, P_, P_, P_]),
    "rr_bias_tile4": (I_, [I_, P_, P_, P_]),
    "rr_bn_finalize": (I_, [I_, I_, L_, P_, P_, P_, P_, P_, P_, F_, F_, P_, P_, P_, P_, P_, P_,
                            S_, P_]),
    "rr_bn_finalize_workspace": (S_, [I_, I_]),
    "rr_bn_finalize_pair": (I_, [C.POINTER(BnFinalizeDesc), C.POINTER(BnFinalizeDesc), P_]),
    "rr_bn_eval_affine": (I_, [I_, P_, P_, P_, P_, F_, P_, P_, P_]),
    "rr_affine_act": (I_, [I_, L_, I_, P_, P_, P_, P_, P_, P_, P_, I_, P_, P_]),
    "rr_affine_act_pool": (I_, [I_, I_, I_, I_, I_, P_, P_, P_, P_, P_, P_, I_, P_, P_, P_, P_]),
    "rr_bn_bwd_blocks": (I_, [C.POINTER(BnBwdDesc)]),
    "rr_bn_bwd_reduce": (I_, [C.POINTER(BnBwdDesc), P_, P_, P_, P_, P_, P_, P_, P_, P_, P_, P_,
                              P_, P_]),
    "rr_bn_bwd_reduce_gm": (I_, [C.POINTER(BnBwdDesc), P_, P_, P_, P_, P_, P_, P_, P_]),
    "rr_bn_bwd_finalize": (I_, [C.POINTER(BnBwdDesc), P_, P_, P_, P_, P_, P_, P_, P_, P_, P_,
                                P_, P_]),
    "rr_bn_bwd_finalize_rows_workspace": (S_, [I_, I_]),
    "rr_bn_bwd_finalize_rows": (I_, [C.POINTER(BnBwdDesc), I_, P_, I_, P_, P_, P_, P_, P_, P_, P_,
                                     P_, S_, P_]),
    "rr_bn_bwd_apply": (I_, [C.POINTER(BnBwdDesc), P_, P_, P_, P_, P_, P_, P_, P_, P_, P_, P_,
                             P_, P_, P_, P_, P_]),
    "rr_channel_sum": (I_, [I_, L_, I_, P_, P_, I_, P_, S_, P_]),
    "rr_channel_sum_workspace": (S_, [L_, I_]),
    "rr_bn_stats_blocks": (I_, [L_]),
    "rr_bn_stats": (I_, [I_, L_, I_, P_, P_, P_]),
    "rr_maxpool2_fwd": (I_, [I_, I_, I_, I_, I_, P_, P_, P_, P_]),
    "rr_nearest_resize": (I_, [I_, I_, I_, I_, I_, I_, I_, P_, P_, P_]),
    "rr_png_encode": (L_, [I_, I_, I_, P_, I_, P_, L_]),
    "rr_fold_conv_bn": (I_, [I_, I_, P_, P_, P_, P_, P_, P_, P_]),
    "rr_png_write_batch": (I_, [I_, I_, I_, I_, P_, P_, I_, I_]),
    "rr_nearest_resize_bwd": (I_, [I_, I_, I_, I_, I_, I_, I_, P_, P_, P_]),
    "rr_maxpool2_bwd": (I_, [I_, I_, I_, I_, I_, P_, P_, P_, I_, P_, P_]),
    "rr_maxpool2_bwd_pooled": (I_, [I_, I_, I_, I_, I_, P_, P_, P_, P_, P_]),
    "rr_conv_in_mfma": (I_, [I_, I_, I_, P_, P_, I_, P_, P_, P_, P_]),
    "rr_im2col3": (I_, [I_, I_, I_, I_, I_, I_, P_, P_, P_]),
    "rr_pack_conv_in": (I_, [I_, I_, I_, I_, P_, P_, P_, P_]),
    "rr_unpack_conv_in_grad": (I_, [I_, I_, I_, P_, P_, P_, P_]),
    "rr_conv_in_fwd": (I_, [I_, I_, I_, I_, I_, I_, P_, P_, P_, I_, P_, P_, P_]),
    "rr_conv_in_wgrad": (I_, [I_, I_, I_, I_, I_, I_, P_, P_, P_, P_, P_, S_, P_]),
    "rr_conv_in_wgrad_workspace": (S_, [I_, I_, I_, I_, I_]),
    "rr_conv_in_wgrad_act_workspace": (S_, [I_, I_, I_]),
    "rr_conv_in_wgrad_act": (I_, [I_, I_, I_, P_, P_, P_, I_, P_, P_, P_, P_, P_, S_, P_]),
    "rr_conv_in_dgrad": (I_, [I_, I_, I_, I_, I_, I_, P_, P_, P_, I_, P_]),
    "rr_prelu_bwd": (I_, [I_, L_, P_, P_, P_, P_, P_, I_, P_, P_]),
    "rr_conv_out_fwd": (I_, [I_, I_, I_, I_, I_, I_, P_, P_, P_, P_, P_]),
    "rr_conv_out_bwd": (I_, [I_, I_, I_, I_, I_, I_, P_, P_, P_, P_, I_, P_, P_, P_, S_, P_]),
    "rr_conv_out_bwd_workspace": (S_, [I_, I_, I_, I_, I_]),
    "rr_conv_out_bwd_bnred_workspace": (S_, [L_, I_, I_]),
    "rr_conv_out_bwd_bnred": (I_, [C.POINTER(BnBwdDesc), I_, I_, I_, I_, P_, P_, P_, P_, P_, P_, P_, P_,
                                   P_, P_, P_, P_, P_, S_, P_]),
    "rr_bn_bwd_apply_convout": (I_, [C.POINTER(BnBwdDesc), I_, I_, P_, P_, I_, P_, P_, P_, P_, P_, P_, P_,
                                     P_, P_, P_, P_, P_]),
    "rr_nchw_to_nhwc": (I_, [I_, I_, I_, I_, I_, P_, P_, P_]),
    "rr_nhwc_to_nchw": (I_, [I_, I_, I_, I_, I_, P_, P_, P_]),
    "rr_loss_fwd": (I_, [I_, I_, L_, P_, P_, P_, F_, I_, P_, S_, P_]),
    "rr_loss_workspace": (S_, [L_]),
    "rr_loss_bwd": (I_, [I_, I_, L_, P_, P_, P_, F_, P_, P_, I_, I_, P_]),
    "rr_adamw_dev": (I_, [L_, P_, P_, P_, P_, P_, F_, F_, F_, F_, I_, P_, P_]),
    "rr_adamw": (I_, [L_, P_, P_, P_, P_, F_, F_, F_, F_, F_, I_, I_, P_]),
    "rr_to_uint8_hwc": (I_, [I_, I_, I_, I_, P_, P_, I_, P_]),
    "rr_psnr_u8": (I_, [I_, L_, P_, P_, P_, P_]),
    "rr_argmax_rows": (I_, [I_, I_, P_, P_, P_]),
    "rr_adaptive_avgpool_flatten": (I_, [I_, I_, I_, I_, I_, I_, I_, P_, P_, P_]),
    "rr_resize_workspace": (S_, [I_, I_, I_, I_, I_, I_]),
    "rr_cv_resize_linear_u8": (I_, [I_, I_, I_, I_, I_, I_, P_, P_, I_, P_]),
    "rr_resize_bilinear_u8": (I_, [I_, I_, I_, I_, I_, I_, P_, I_, P_, P_, P_, P_, S_, P_]),
    "rr_ssim_workspace": (S_, [I_, I_]),
    "rr_ssim_u8": (I_, [I_, I_, I_, I_, P_, P_, P_, P_, S_, P_]),
    "rr_distort_workspace": (S_, [I_, I_, I_, I_]),
    "rr_distort_u8": (I_, [I_, I_, I_, I_, I_, P_, P_, P_, P_, P_, C.c_ulonglong, P_, S_, P_]),
    "rr_motion_blur_kernel": (I_, [I_, I_, P_]),
    "rr_motion_blur_table_floats": (S_, []),
    "rr_motion_blur_table": (I_, [P_]),
    "rr_distort_random_workspace": (S_, [I_, I_, I_, I_]),
    "rr_distort_random_u8": (I_, [I_, I_, I_, I_, P_, P_, C.c_ulonglong, P_, P_, P_, S_, P_]),
    "rr_distort_random_draws": (I_, [I_, I_, I_, I_, P_, C.POINTER(S_), C.POINTER(S_),
                                     C.POINTER(S_)]),
    "rr_scalar_accumulate": (I_, [P_, P_, P_, P_]),
    "rr_zero": (I_, [P_, S_, P_]),
    "rr_version": (C.c_char_p, []),
}

EXPORTED = tuple(_SIGS)


class Lib:
    """Loaded library with typed entry points; ``check`` turns status codes
    into RuntimeError (the reference's ATen ops raise RuntimeError too)."""

    def __init__(self, path=LIB_PATH):
        if not os.path.exists(path):
            raise RuntimeError(
                f"roadrestore HIP library not built: {path} is missing "
                "(run __graft_entry__.build())")
        self.path = path
        self.dll = C.CDLL(path)
        # another build loaded for an A/B (RR_LIB_PATH) may predate entry
        # points this binding knows: those stay unbound (calling one raises)
        # instead of refusing the library; the in-tree library must export all
        other = os.path.abspath(path) != os.path.abspath(os.path.join(_HERE, "libroadrestore.so"))
        for name, (res, args) in _SIGS.items():
            try:
                fn = getattr(self.dll, name)
            except AttributeError:
                if not other:
                    raise
                continue
            fn.restype = res
            fn.argtypes = args
            setattr(self, name, fn)

    @staticmethod
    def check(rc, what):
        if rc != 0:
            raise RuntimeError(f"{what} failed: {_STATUS.get(rc, rc)} ({rc})")
        return rc


_LIB = None


def lib() -> Lib:
    global _LIB
    if _LIB is None:
        _LIB = Lib()
    return _LIB
