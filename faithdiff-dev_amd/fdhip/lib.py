"""ctypes binding of libfaithdiff_hip.so (C ABI: include/faithdiff_hip.h).

This is the only door into the device path.  There is no fallback: if the library is missing or the
device is not gfx950, every op raises.  PyTorch is used only for device memory and the current HIP
stream (``torch.cuda.current_stream().cuda_stream``), so launches are ordered with (and capturable by)
torch's stream / graph machinery.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# FD_LIB_PATH (benchmarks only): an alternative build of the same library for in-session A/B timing
LIB_PATH = os.environ.get("FD_LIB_PATH") or os.path.join(_HERE, "libfaithdiff_hip.so")

FD_BF16, FD_F16, FD_F32 = 0, 1, 2
ACT = {"none": 0, "silu": 1, "gelu": 2, "quickgelu": 3, "geglu": 4, "lrelu": 5, "softmax": 6}
_ERR = {-1: "FD_ERR_SHAPE", -2: "FD_ERR_DTYPE", -3: "FD_ERR_ARCH", -4: "FD_ERR_HIP", -5: "FD_ERR_ARG"}

c_vp, c_int, c_ll, c_f, c_char_p = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong, ctypes.c_float, ctypes.c_char_p


class GemmParams(ctypes.Structure):
    _fields_ = [
        ("A", c_vp), ("B", c_vp), ("C", c_vp),
        ("lda", c_ll), ("ldb", c_ll), ("ldc", c_ll),
        ("strideA", c_ll), ("strideB", c_ll), ("strideC", c_ll),
        ("M", c_int), ("N", c_int), ("K", c_int), ("batch", c_int),
        ("bias", c_vp), ("residual", c_vp), ("ldr", c_ll), ("strideR", c_ll),
        ("rowbias", c_vp), ("rowbias_ld", c_ll), ("rows_per_group", c_int),
        ("alpha", c_f), ("act", c_int), ("dtype", c_int), ("out_dtype", c_int),
        ("conv", c_int), ("nimg", c_int), ("Hin", c_int), ("Win", c_int), ("Cin", c_int),
        ("Hout", c_int), ("Wout", c_int), ("stride", c_int), ("pad", c_int), ("upsample", c_int),
        ("A2", c_vp), ("C1", c_int),
        ("m_ref", c_int), ("ws", c_vp), ("ws_bytes", c_ll),
        ("ln_out", c_vp), ("ln_in", c_vp), ("ln_c", c_vp), ("ln_eps", c_f),
        ("gn_part", c_vp), ("gn_groups", c_int), ("gn_hw", c_int), ("gn_done", c_int),
        ("gi_affine", c_vp), ("gi_silu", c_int),
        ("batch_inner", c_int), ("strideA_o", c_ll), ("strideB_o", c_ll), ("strideC_o", c_ll),
        ("bsel_rows", c_int), ("bsel_mod", c_int), ("bsel_strideB", c_ll), ("bsel_strideN", c_ll),
        ("sm_group", c_int), ("sm_len", c_int),
        ("up_phase", c_int),
        ("rowbias_rows", c_ll), ("residual_rows", c_ll),
    ]


# name -> (restype, argtypes)
_SIGS = {
    "fd_gemm": (c_int, [ctypes.POINTER(GemmParams), c_vp]),
    "fd_gemm_ws_bytes": (c_ll, [ctypes.POINTER(GemmParams)]),
    "fd_conv_halo_plan": (c_int, [ctypes.POINTER(GemmParams)]),
    "fd_conv_halo_pt": (c_int, [ctypes.POINTER(GemmParams)]),
    "fd_group_norm_affine": (c_int, [c_vp, c_vp, c_int, c_vp, c_vp, c_int, c_int, c_int, c_int, c_f, c_vp, c_vp, c_int,
                                     c_vp]),
    "fd_conv2d_direct": (c_int, [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_f,
                                 c_int, c_int, c_vp]),
    "fd_group_norm_ws_bytes": (c_ll, [c_int, c_int, c_int, c_int]),
    "fd_group_norm": (c_int, [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_f, c_int, c_int, c_vp, c_vp]),
    "fd_group_norm_partials": (c_int, [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_f, c_int, c_vp, c_int,
                                       c_vp, c_int, c_vp]),
    "fd_gemm_e4m3": (c_int, [c_vp, c_ll, c_vp, c_vp, c_ll, c_f, c_vp, c_ll, c_int, c_int, c_int, c_vp, c_vp, c_ll,
                             c_int, c_int, c_vp]),
    "fd_layer_norm_e4m3": (c_int, [c_vp, c_ll, c_vp, c_ll, c_vp, c_vp, c_vp, c_int, c_int, c_f, c_int, c_vp]),
    "fd_quant_rows_e4m3": (c_int, [c_vp, c_ll, c_vp, c_ll, c_vp, c_int, c_int, c_int, c_vp]),
    "fd_gemm_mxe4m3": (c_int, [c_vp, c_ll, c_vp, c_ll, c_vp, c_ll, c_f, c_vp, c_ll, c_vp, c_ll, c_int, c_int, c_int,
                               c_vp, c_vp, c_ll, c_int, c_int, c_vp]),
    "fd_quant_rows_mx": (c_int, [c_vp, c_ll, c_vp, c_ll, c_vp, c_ll, c_int, c_int, c_int, c_vp]),
    "fd_layer_norm_mx": (c_int, [c_vp, c_ll, c_vp, c_ll, c_vp, c_ll, c_vp, c_vp, c_int, c_int, c_f, c_int, c_vp]),
    "fd_flash_attn_mx": (c_int, [c_vp, c_ll, c_ll, c_vp, c_ll, c_ll, c_vp, c_ll, c_ll, c_vp, c_ll, c_ll, c_vp, c_ll,
                                 c_ll, c_int, c_int, c_int, c_int, c_int, c_int, c_f, c_int, c_vp]),
    "fd_layer_norm": (c_int, [c_vp, c_ll, c_vp, c_ll, c_vp, c_vp, c_int, c_int, c_f, c_int, c_vp]),
    "fd_flash_attn": (c_int, [c_vp, c_ll, c_ll, c_vp, c_ll, c_ll, c_vp, c_ll, c_ll, c_vp, c_ll, c_ll, c_int, c_int,
                              c_int, c_int, c_int, c_int, c_f, c_int, c_vp]),
    "fd_embed_tokens": (c_int, [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_vp]),
    "fd_conv3x3_narrow": (c_int, [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_vp]),
    "fd_conv3x3_narrow_gn": (c_int, [c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_int, c_int, c_int, c_int, c_int, c_int,
                                     c_int, c_vp]),
    "fd_flash_attn_d512": (c_int, [c_vp, c_vp, c_vp, c_ll, c_ll, c_vp, c_ll, c_ll, c_int, c_int, c_f, c_int, c_vp]),
    "fd_flash_attn_d512_ksplit": (c_int, [c_int, c_int]),
    "fd_flash_attn_d512_split": (c_int, [c_vp, c_vp, c_vp, c_ll, c_ll, c_vp, c_ll, c_ll, c_int, c_int, c_f, c_int, c_vp,
                                         c_ll, c_int, c_vp]),
    "fd_mha_seq_axis": (c_int, [c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp]),
    "fd_softmax_rows": (c_int, [c_vp, c_vp, c_int, c_int, c_ll, c_f, c_int, c_vp]),
    "fd_xattn_consts": (c_int, [c_vp, c_ll, c_int, c_int, c_vp, c_ll, c_ll, c_vp, c_int, c_int, c_int, c_f, c_vp, c_vp,
                                c_int, c_vp]),
    "fd_concat_channels": (c_int, [c_vp, c_int, c_vp, c_int, c_vp, c_ll, c_int, c_vp]),
    "fd_group_norm_chunk_rows": (c_int, [c_int, c_int]),
    "fd_concat_channels_gn": (c_int, [c_vp, c_int, c_vp, c_int, c_vp, c_int, c_int, c_int, c_vp, c_int, c_vp]),
    "fd_unary": (c_int, [c_vp, c_vp, c_ll, c_int, c_int, c_int, c_vp]),
    "fd_add_strided": (c_int, [c_vp, c_ll, c_vp, c_ll, c_vp, c_ll, c_int, c_int, c_int, c_int, c_vp]),
    "fd_axpby": (c_int, [c_vp, c_ll, c_vp, c_ll, c_vp, c_ll, c_int, c_int, c_f, c_f, c_int, c_vp]),
    "fd_nchw_to_nhwc": (c_int, [c_vp, c_vp, c_int, c_int, c_int, c_f, c_int, c_int, c_vp]),
    "fd_nhwc_to_nchw": (c_int, [c_vp, c_vp, c_int, c_int, c_int, c_f, c_int, c_int, c_vp]),
    "fd_transpose": (c_int, [c_vp, c_ll, c_vp, c_ll, c_int, c_int, c_int, c_ll, c_ll, c_int, c_vp]),
    "fd_time_features": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_vp]),
    "fd_tlc_scale_input": (c_int, [c_vp, c_vp, c_int, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                   c_f, c_vp, c_int, c_vp]),
    "fd_tlc_scale_input_t": (c_int, [c_vp, c_vp, c_int, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                     c_f, c_vp, c_int, c_vp, c_int, c_f, c_vp]),
    "fd_tlc_cfg_euler_step": (c_int, [c_vp, c_vp, c_vp, c_int, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                      c_int, c_f, c_f, c_f, c_f, c_vp, c_int, c_vp]),
    "fd_tlc_blend": (c_int, [c_vp, c_vp, c_vp, c_int, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp, c_vp]),
    "fd_tlc_grids_nhwc": (c_int, [c_vp, c_vp, c_int, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                  c_int, c_vp, c_int, c_vp]),
    "fd_vae_sample_add_noise": (c_int, [c_vp, c_vp, c_vp, c_vp, c_int, c_f, c_f, c_f, c_f, c_int, c_int, c_vp]),
    "fd_postprocess_u8": (c_int, [c_vp, c_vp, c_ll, c_int, c_vp]),
    "fd_blend_edge": (c_int, [c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_vp]),
    "fd_set_knob": (c_int, [c_char_p, c_int, ctypes.POINTER(c_int)]),
    "fd_get_knob": (c_int, [c_char_p, ctypes.POINTER(c_int), ctypes.POINTER(c_int)]),
    "fd_knob_name": (c_char_p, [c_int]),
    "fd_reset_knobs": (None, []),
    "fd_splitk_health": (c_int, [ctypes.POINTER(ctypes.c_uint), c_int]),
    "fd_splitk_test_drop": (c_int, [c_int]),
    "fd_device_check": (c_int, []),
    "fd_version": (c_char_p, []),
}

_lib = None


def load():
    """Load the shared library (no device access).  Raises if it was not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"libfaithdiff_hip.so not built ({LIB_PATH}); run `make -C faithdiff-dev_amd/csrc` "
                               "or __graft_entry__.build() -- there is no CPU fallback")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(lib, name)
            f.restype = res
            f.argtypes = args
        _lib = lib
    return _lib


def exported_symbols():
    return list(_SIGS)


_checked = False


def require_device():
    """Fail loudly unless a gfx950 device is current."""
    global _checked
    if _checked:
        return
    if not torch.cuda.is_available():
        raise RuntimeError("faithdiff HIP path needs an MI355X (gfx950) GPU; none is visible")
    rc = load().fd_device_check()
    if rc != 0:
        raise RuntimeError(f"fd_device_check failed: {_ERR.get(rc, rc)} (device is not gfx950?)")
    _checked = True


def check(rc, name):
    if rc != 0:
        raise RuntimeError(f"{name} failed: {_ERR.get(rc, rc)}")


def dtype_code(dt):
    if dt == torch.bfloat16:
        return FD_BF16
    if dt == torch.float16:
        return FD_F16
    if dt == torch.float32:
        return FD_F32
    raise TypeError(f"unsupported dtype {dt}")


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
