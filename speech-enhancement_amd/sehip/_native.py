"""ctypes binding of libsehip.so (the C ABI declared in include/sehip.h).

The product path has no fallback: if the HIP library is missing or a call
returns an error, a RuntimeError is raised. torch is imported first so that
the process-wide HIP runtime (torch's bundled libamdhip64.so.7) is the one
libsehip.so binds to — device pointers and hipStream_t handles taken from
torch are then valid inside the library.
"""
from __future__ import annotations

import ctypes
import os
import re

import torch  # noqa: F401  (must precede the CDLL load, see module doc)

_HERE = os.path.dirname(os.path.abspath(__file__))
# SEHIP_LIB may point at another in-tree build of the same library (A/B
# measurement of kernel variants); the default is the package's own build.
LIB_PATH = os.environ.get("SEHIP_LIB") or os.path.join(_HERE, "libsehip.so")
HEADER_PATH = os.path.abspath(os.path.join(_HERE, "..", "..", "include", "sehip.h"))

c_int = ctypes.c_int
c_float = ctypes.c_float
c_size_t = ctypes.c_size_t
c_void_p = ctypes.c_void_p
c_char_p = ctypes.c_char_p


class ConvDesc(ctypes.Structure):
    """Mirror of se_conv2d_desc (include/sehip.h)."""

    _fields_ = [(n, c_int) for n in (
        "batch", "in_channels", "in_h", "in_w", "out_channels",
        "kernel_h", "kernel_w", "stride_h", "stride_w", "pad_h", "pad_w",
        "dil_h", "dil_w", "out_pad_h", "out_pad_w", "transposed",
        "complex_weights", "pad_h_end", "pad_w_end", "math")] + [
        ("x_amax", c_void_p), ("dy_amax", c_void_p),   # SE_MATH_F16X3 scale sources (or NULL)
        ("w_amax", c_void_p),   # SE_MATH_F16X3 bound of max |w| (or NULL)
        ("dtype", c_int),           # SE_DTYPE_* storage of the conv's tensors (ABI 4)
        ("data_weights", c_void_p),   # prepared data-grad weight image (or NULL, ABI 5)
        ("join_cat", c_int)]          # joined forms: 0 complex_concat, 1 torch.cat order (ABI 8)


class FirstConvDesc(ctypes.Structure):
    """Mirror of se_first_conv (include/sehip.h)."""

    _fields_ = [("x0", c_void_p)] + [(n, c_int) for n in (
        "cin", "in_h", "in_w", "kernel_h", "kernel_w", "stride_h", "stride_w", "pad_h", "pad_w",
        "dil_h", "dil_w")] + [("dwr", c_void_p), ("dwi", c_void_p)]


class GemmDesc(ctypes.Structure):
    """Mirror of se_gemm_desc (include/sehip.h, ABI 6; dtype / bias_rows ABI 10)."""

    _fields_ = [(n, c_int) for n in ("M", "N", "K", "batches", "sum_batches", "a_mcontig", "b_ncontig",
                                     "lda", "ldb", "ldc")] + [
        (n, ctypes.c_longlong) for n in ("stride_a", "stride_b", "stride_c", "stride_bias")] + [
        (n, c_int) for n in ("kmask_period", "kmask_phase", "splits", "dtype", "bias_rows")]


_P = c_void_p
ABI_VERSION = 11   # SEHIP_ABI_VERSION (include/sehip.h)
CBN_SAVE_FLOATS = 20   # SE_CBN_SAVE_FLOATS (include/sehip.h)
_PP = ctypes.POINTER(c_void_p)   # host array of device pointers
_SIGNATURES = {
    "se_abi_version": (c_int, []),
    "se_strerror": (c_char_p, [c_int]),
    "se_probe": (c_int, [_P, c_int, _P]),
    "se_stft_num_frames": (c_int, [c_int] * 5),
    "se_stft_fwd": (c_int, [_P, _P, _P] + [c_int] * 7 + [_P, _P, c_int, _P]),
    "se_istft_fwd": (c_int, [_P, _P] + [c_int] * 7 + [_P, _P, c_int, _P]),
    "se_istft_bwd": (c_int, [_P, _P] + [c_int] * 7 + [_P, _P, c_int, _P]),
    "se_conv2d_out_shape": (c_int, [_P, _P, _P]),
    "se_amax": (c_int, [_P, ctypes.c_longlong, _P, _P]),
    "se_amax_init": (c_int, [_P, ctypes.c_longlong, _P, _P]),
    "se_amax_weights": (c_int, [_P, ctypes.c_longlong, _P, _P, _P]),
    "se_mix_snr": (c_int, [_P, _P, c_int, c_int, c_int, _P, _P, _P, _P, c_int, _P, _P, _P, _P]),
    "se_crop_pad": (c_int, [_P, _P, _P, _P, c_int, c_int, _P, _P]),
    "se_pcm16_to_float": (c_int, [_P, ctypes.c_longlong, _P, _P]),
    "se_float_to_pcm16": (c_int, [_P, ctypes.c_longlong, _P, _P]),
    "se_resample": (c_int, [_P, c_int, c_int, c_int, c_int, _P, c_int, c_int, _P, c_int, _P]),
    "se_conv2d_workspace_size": (c_size_t, [_P]),
    "se_conv2d_data_weights_size": (c_size_t, [_P]),
    "se_conv2d_prep_data_weights": (c_int, [_P] * 4 + [c_size_t, _P]),
    "se_conv2d_fwd": (c_int, [_P] * 7 + [_P, c_size_t, _P]),
    "se_conv2d_bwd_data": (c_int, [_P] * 5 + [_P, c_size_t, _P]),
    "se_conv2d_bwd_weight": (c_int, [_P] * 7 + [_P, c_size_t, _P]),
    "se_conv2d_fwd_joined": (c_int, [_P, _P, c_int, c_int] + [_P] * 6 + [_P, c_size_t, _P]),
    "se_conv2d_bwd_data_joined": (c_int, [_P] * 5 + [c_int, c_int, _P, _P, c_size_t, _P]),
    "se_conv2d_bwd_weight_joined": (c_int, [_P, _P, c_int, c_int] + [_P] * 6 + [_P, c_size_t, _P]),
    "se_cbn_workspace_size": (c_size_t, [c_int, c_int, c_int]),
    "se_cbn_fwd": (c_int, [_P, _P, c_int, c_int, c_int, _PP, _PP, _P, _P, c_int, c_float, c_float, c_int,
                           c_float, _P, _P, c_int, _P, c_size_t, _P]),
    "se_cbn_bwd": (c_int, [_P, _P, _P, _P, c_int, c_int, c_int, _PP, _P, _PP, c_int, c_int, c_float, _P, _P, _P,
                           c_int, _P, c_size_t, _P]),
    "se_cbn_bwd2": (c_int, [_P, _P, _P, _P, c_int, c_int, c_int, _PP, _P, _PP, c_int, c_int, c_float, _P, _P, _P,
                            c_int, _P, c_size_t, _P]),
    "se_cbn_bwd_ccbam": (c_int, [_P] * 10 + [c_int, c_int, c_int, _PP, _P, _PP, c_int, c_int, c_float, _P, _P,
                                               c_size_t, _P]),
    "se_cbn_head_workspace_size": (c_size_t, [c_int, c_int, c_int]),
    "se_cbn_first_conv_workspace_size": (c_size_t, [c_int] * 6),
    "se_cbn_bwd_first_conv": (c_int, [_P, _P, _P] + [c_int] * 4 + [_PP, _P, _PP, c_int, c_int, c_float, _P, _P,
                                                                  c_size_t, _P]),
    "se_cbn_head_fwd": (c_int, [_P, _P] + [c_int] * 4 + [_PP, _PP, _P, _P, c_int, c_float, c_float, c_int,
                                c_float, _P, c_int, c_int, _P, c_size_t, _P]),
    "se_cbn_head_bwd": (c_int, [_P, _P, _P] + [c_int] * 4 + [_PP, _P, _PP, _P, _P, c_int, c_int, c_int, c_int,
                                c_float, _P, _P, c_size_t, _P]),
    "se_gemm_workspace_size": (c_size_t, [_P]),
    "se_gemm": (c_int, [_P] * 8 + [_P, c_size_t, _P]),
    "se_colsum_workspace_size": (c_size_t, [c_int, ctypes.c_longlong, c_int]),
    "se_colsum": (c_int, [_P, c_int, ctypes.c_longlong, c_int, _P, _P, _P, c_size_t, _P]),
    "se_lstm_supported": (c_int, [c_int]),
    "se_lstm_fwd": (c_int, [_P, ctypes.c_longlong, c_int, _P, _P, _P, _P, _P] + [c_int] * 4
                    + [ctypes.c_uint, _P]),
    "se_lstm_bwd": (c_int, [_P] * 5 + [c_int] * 4 + [ctypes.c_uint, _P]),
    "se_bn_workspace_size": (c_size_t, [c_int, c_int]),
    "se_bn_fwd": (c_int, [_P, ctypes.c_longlong, c_int, c_int, c_int, _P, _P, _P, _P, c_int, c_float, c_float,
                          c_int, _P, c_int, c_float, _P, _P, c_int, _P, c_size_t, _P]),
    "se_bn_bwd": (c_int, [_P, _P, ctypes.c_longlong, c_int, c_int, c_int, _P, _P, _P, c_int, c_int, _P, c_int,
                          c_float, _P, _P, _P, _P, c_int, _P, c_size_t, _P]),
    "se_sisnr_save_bytes": (c_size_t, [c_int]),
    "se_mask_fwd": (c_int, [_P, _P, c_int, c_int, c_int, _P, _P]),
    "se_polar_mask_fwd": (c_int, [_P, _P, ctypes.c_longlong, ctypes.c_longlong, _P, _P, ctypes.c_longlong,
                                  ctypes.c_longlong, c_int, c_int,
                                  c_int, c_int, c_int, c_int, _P, _P]),
    "se_mask_bwd": (c_int, [_P, _P, _P, c_int, c_int, c_int, _P, _P]),
    "se_polar_mask_bwd": (c_int, [_P, _P, _P, ctypes.c_longlong, ctypes.c_longlong, _P, _P, ctypes.c_longlong,
                                  ctypes.c_longlong, c_int, c_int, c_int, c_int, c_int, c_int, c_int, _P, _P]),
    "se_sisnr_fwd": (c_int, [_P, c_int, ctypes.c_longlong, _P, c_int, c_int, c_int, c_float, _P, _P, c_int, _P]),
    "se_sisnr_bwd": (c_int, [_P, c_int, ctypes.c_longlong, _P, c_int, c_int, c_int, c_float, _P, _P, _P,
                             ctypes.c_longlong, c_int, _P]),
    "se_grad_sumsq": (c_int, [_P, c_int, ctypes.c_longlong, _P, c_int, _P]),
    "se_clip_grads": (c_int, [_P, c_int, ctypes.c_longlong, _P, c_float, _P, c_int, _P]),
    "se_adamw_step": (c_int, [_P, c_int, ctypes.c_longlong] + [ctypes.c_double] * 5 + [ctypes.c_longlong, c_int,
                                                                                          _P]),
    "se_lstm_wide_supported": (c_int, [c_int]),
    "se_lstm_wide_sync_ints": (c_int, []),
    "se_lstm_wide_fwd": (c_int, [_P, ctypes.c_longlong, c_int, _P, _P, _P, _P] + [c_int] * 4
                         + [ctypes.c_uint, _P, _P, _P]),
    "se_lstm_wide_bwd": (c_int, [_P] * 5 + [c_int] * 4 + [ctypes.c_uint, _P, _P, _P]),
    "se_ccbam_workspace_size": (c_size_t, [c_int] * 3),
    "se_ccbam_channel_pool": (c_int, [_P] * 4 + [c_int] * 3 + [_P]),
    "se_ccbam_spatial_pool": (c_int, [_P] * 4 + [c_int] * 3 + [_P]),
    "se_ccbam_apply": (c_int, [_P] * 4 + [c_int] * 3 + [_P, _P]),
    "se_ccbam_bwd_sa": (c_int, [_P] * 2 + [c_int] * 3 + [_P]),
    "se_ccbam_bwd_sa_sigmoid": (c_int, [_P] * 3 + [c_int] * 3 + [_P]),
    "se_ccbam_bwd_dca": (c_int, [_P] * 5 + [c_int] * 3 + [_P, c_size_t, _P]),
    "se_ccbam_bwd_dx": (c_int, [_P] * 8 + [c_int] * 3 + [_P]),
    "se_ccbam_mlp_fwd": (c_int, [_P] * 6 + [c_int] * 3 + [_P] * 3),
    "se_ccbam_mlp_bwd": (c_int, [_P] * 9 + [c_int] * 3 + [_P] * 7),
    # ABI 10: Linear bias gradient, strided copy / cast, ComplexLSTM combine, CARN glue, chunking
    "se_bias_grad_workspace_size": (c_size_t, [c_int, ctypes.c_longlong, c_int]),
    "se_bias_grad": (c_int, [_P, c_int, ctypes.c_longlong, c_int] + [ctypes.c_longlong] * 3 + [c_int, _P, _P,
                                                                                              c_size_t, _P]),
    "se_copy_strided": (c_int, [_P, c_int, _P, c_int, c_int, _P, _P, _P, _P]),
    "se_complex_lstm_combine_fwd": (c_int, [_P, ctypes.c_longlong, c_int, c_int, c_int, _P] + [ctypes.c_longlong] * 3
                                    + [c_int, _P]),
    "se_complex_lstm_combine_bwd": (c_int, [_P] + [ctypes.c_longlong] * 3 + [c_int, c_int, c_int, c_int, _P,
                                                                            ctypes.c_longlong, _P]),
    "se_carn_mask_fwd": (c_int, [_P, ctypes.c_longlong, _P, c_int, c_int, c_int, c_int, _P, _P]),
    "se_carn_mask_bwd": (c_int, [_P, _P, ctypes.c_longlong, _P, c_int, c_int, c_int, c_int, _P, _P, _P]),
    "se_add_sigmoid_fwd": (c_int, [_P, _P, _P, ctypes.c_longlong, c_int, _P]),
    "se_sigmoid_bwd": (c_int, [_P, _P, _P, ctypes.c_longlong, c_int, _P]),
    "se_sigmoid_fwd": (c_int, [_P, _P, ctypes.c_longlong, c_int, _P]),
    "se_gate_cat_fwd": (c_int, [_P, _P, _P, c_int, c_int, ctypes.c_longlong, c_int, _P]),
    "se_gate_cat_bwd": (c_int, [_P, _P, _P, _P, _P, c_int, c_int, ctypes.c_longlong, c_int, _P]),
    "se_glu_fwd": (c_int, [_P, _P, _P, ctypes.c_longlong, c_int, _P]),
    "se_glu_bwd": (c_int, [_P, _P, _P, _P, _P, ctypes.c_longlong, c_int, _P]),
    "se_clamp_fwd": (c_int, [_P, _P, ctypes.c_longlong, c_float, c_float, c_int, _P]),
    "se_clamp_bwd": (c_int, [_P, _P, _P, ctypes.c_longlong, c_float, c_float, c_int, _P]),
    "se_chunk_split": (c_int, [_P, ctypes.c_longlong, c_int, c_int, c_int, c_int, _P, _P]),
    "se_chunk_overlap_add": (c_int, [_P, c_int, c_int, c_int, c_int, ctypes.c_longlong, c_int, _P, _P]),
    "se_complex_join": (c_int, [_P, c_int, c_int, c_int, _P, c_int, c_int, c_int, _P, c_int, c_int, _P]),
    "se_complex_join_bwd": (c_int, [_P, _P, c_int, c_int, c_int, _P, c_int, c_int, c_int, c_int, c_int, _P]),
}


def header_symbols(path: str = HEADER_PATH) -> list[str]:
    """Every function name declared in include/sehip.h."""
    with open(path) as f:
        text = f.read()
    return sorted(set(re.findall(r"\b(se_[a-z0-9_]+)\s*\(", text)))


_lib = None
MISSING: list[str] = []


def lib() -> ctypes.CDLL:
    """Load libsehip.so once; raise loudly if it is missing."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"sehip: native library not built ({LIB_PATH}); run "
                "`python -c 'import __graft_entry__ as g; g.build()'`")
        handle = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in _SIGNATURES.items():
            try:
                f = getattr(handle, name)
            except AttributeError:
                MISSING.append(name)   # tests/test_abi.py requires this to stay empty
                continue
            f.restype = res
            f.argtypes = args
        if "se_abi_version" not in MISSING and handle.se_abi_version() != ABI_VERSION:
            # a stale build: the struct mirrors above would not match its layout
            raise RuntimeError(f"sehip: {LIB_PATH} has ABI {handle.se_abi_version()}, this package "
                               f"needs {ABI_VERSION}; rebuild it")
        _lib = handle
    return _lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().se_strerror(rc).decode()
        raise RuntimeError(f"sehip: {what} failed: {msg} (code {rc})")


def stream_of(t: torch.Tensor) -> int:
    """The caller's current HIP stream for tensor t's device."""
    return torch.cuda.current_stream(t.device).cuda_stream


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()


def require_device(*ts: torch.Tensor, dtype=torch.float32) -> None:
    for t in ts:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError("sehip ops run on the GPU only (got a CPU tensor); "
                               "there is no CPU fallback in the product path")
        if t.dtype != dtype:
            raise RuntimeError(f"sehip ops take {dtype} tensors (got {t.dtype})")


# SE_DTYPE_* (include/sehip.h): storage types of the dtype-aware entry points
DTYPES = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}


def dtype_code(t: torch.Tensor) -> int:
    try:
        return DTYPES[t.dtype]
    except KeyError:
        raise RuntimeError(f"sehip: unsupported storage type {t.dtype} (fp32, bf16, fp16)") from None


def ptr_array(ts):
    """Host array of device pointers (for the se_cbn_* pointer-array args)."""
    if ts is None:
        return None
    return (c_void_p * len(ts))(*[t.data_ptr() for t in ts])


def probe(n: int = 1000, device: str = "cuda") -> torch.Tensor:
    out = torch.empty(n, dtype=torch.int32, device=device)
    check(lib().se_probe(out.data_ptr(), n, stream_of(out)), "se_probe")
    return out
