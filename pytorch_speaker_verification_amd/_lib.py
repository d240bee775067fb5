"""Loader for the in-tree gfx950 HIP library (libsv_ge2e.so) behind include/sv_ge2e.h.

There is no fallback: if the library is missing or fails to load, every op raises.
The library binds to the HIP runtime torch already loaded (same soname,
libamdhip64.so.7), so torch must be imported first -- this module does that.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (loads the HIP runtime the library binds to)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libsv_ge2e.so")

_c_void_p = ctypes.c_void_p
_c_int = ctypes.c_int
_c_long = ctypes.c_long
_c_float = ctypes.c_float
_c_size_t = ctypes.c_size_t

# name -> (restype, argtypes); mirrors include/sv_ge2e.h
_P = _c_void_p
SIGNATURES = {
    "sv_abi_version": (_c_int, []),
    "sv_gemm_f32_workspace": (_c_size_t, [_c_int, _c_int, _c_int]),
    "sv_gemm_f32": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _P, _c_long, _P, _c_long, _P, _c_long, _P, _P,
                             _c_float, _P, _P]),
    "sv_colsum_workspace": (_c_size_t, [_c_int, _c_int]),
    "sv_colsum": (_c_int, [_P, _c_int, _c_int, _P, _P, _P]),
    "sv_frames_to_time_major": (_c_int, [_P, _P, _c_int, _c_int, _c_int, _P]),
    "sv_transpose": (_c_int, [_P, _c_long, _c_int, _c_int, _P, _c_long, _P]),
    "sv_lstm_layer_fwd": (_c_int, [_P, _c_int, _c_int, _c_int, _c_int, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "sv_lstm_step_fwd": (_c_int, [_P, _P, _P, _P, _P, _P, _c_int, _c_int, _P]),
    "sv_lstm_step_bwd": (_c_int, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _c_int, _c_int, _P]),
    "sv_lstm_stack_fwd": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                   _c_int, _P, _P, _P]),
    "sv_lstm_stack_bwd_workspace": (_c_size_t, [_c_int, _c_int, _c_int, _c_int, _c_int]),
    "sv_lstm_stack_bwd": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int] + [_P] * 16 + [_c_int, _P, _P, _P]),
    "sv_lstm_layer_bwd_workspace": (_c_size_t, [_c_int, _c_int, _c_int, _c_int]),
    "sv_lstm_layer_bwd": (_c_int, [_c_int, _c_int, _c_int, _c_int, _P, _c_long, _P, _P, _P, _P, _P, _P, _c_int, _P,
                                   _P, _P, _P, _P, _P, _P, _P, _P]),
    "sv_proj_norm_workspace": (_c_size_t, [_c_int, _c_int, _c_int]),
    "sv_proj_norm_fwd": (_c_int, [_P, _c_int, _c_int, _c_int, _P, _P, _P, _P, _P, _P, _P]),
    "sv_proj_norm_bwd": (_c_int, [_P, _P, _P, _P, _c_int, _c_int, _c_int, _P, _P, _P, _P, _P, _P]),
    "sv_ge2e_workspace_size": (_c_size_t, [_c_int, _c_int, _c_int, _c_int]),
    "sv_ge2e_speaker_sums": (_c_int, [_P, _c_int, _c_int, _c_int, _P, _P]),
    "sv_ge2e_fwd_rows": (_c_int, [_P, _c_int, _c_int, _c_int, _c_int, _c_int, _P, _P, _P, _P, _P, _P, _P]),
    "sv_ge2e_fwd": (_c_int, [_P, _c_int, _c_int, _c_int, _P, _P, _P, _P, _P, _P, _P]),
    "sv_ge2e_bwd_rows": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _P, _P, _P, _P, _P, _P, _P, _P]),
    "sv_ge2e_bwd_finalize": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _P, _P, _P, _P, _P]),
    "sv_ge2e_bwd": (_c_int, [_c_int, _c_int, _c_int, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "sv_ge2e_centroids": (_c_int, [_P, _c_int, _c_int, _c_int, _P, _P]),
    "sv_ge2e_cossim_workspace": (_c_size_t, [_c_int, _c_int, _c_int, _c_int]),
    "sv_ge2e_cossim": (_c_int, [_P, _c_int, _c_int, _c_int, _P, _c_int, _P, _P, _P]),
    "sv_ge2e_calc_loss": (_c_int, [_P, _c_int, _c_int, _c_int, _P, _P, _P]),
    "sv_gemm_bf16_workspace": (_c_size_t, [_c_int, _c_int, _c_int]),
    "sv_gemm_bf16": (_c_int, [_c_int, _c_int, _c_int, _P, _c_long, _P, _c_long, _P, _c_long, _P, _P, _c_float, _P,
                              _P]),
    "sv_cast_bf16": (_c_int, [_P, _P, _c_long, _P]),
    "sv_transpose_cast_bf16": (_c_int, [_P, _c_long, _c_int, _c_int, _P, _c_long, _P]),
    "sv_lstm_layer_fwd_bf16": (_c_int, [_P, _c_int, _c_int, _c_int, _c_int, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "sv_lstm_stack_fwd_bf16": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                        _P, _c_int, _P, _P, _P]),
    "sv_lstm_layer_bwd_bf16_workspace": (_c_size_t, [_c_int, _c_int, _c_int, _c_int]),
    "sv_lstm_layer_bwd_bf16": (_c_int, [_c_int, _c_int, _c_int, _c_int, _P, _c_long, _P, _P, _P, _P, _P, _P, _c_int,
                                        _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "sv_eer_counts": (_c_int, [_P, _c_int, _c_int, _c_int, _P, _c_int, _P, _P, _P]),
    "sv_lstm_stack_bwd_bf16_workspace": (_c_size_t, [_c_int, _c_int, _c_int, _c_int, _c_int]),
    "sv_lstm_stack_bwd_bf16": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int] + [_P] * 16 + [_c_int, _P, _P, _P]),
    "sv_set_f32_products": (_c_int, [_c_int]),
    "sv_persist_fwd_ok": (_c_int, [_c_int, _c_int]),
    "sv_persist_bwd_ok": (_c_int, [_c_int, _c_int]),
    "sv_persist_bwd_scratch": (_c_size_t, [_c_int, _c_int, _c_int]),
    "sv_persist_status": (_c_int, []),
    "sv_persist_stamps": (_c_int, [_P, _c_int]),
    "sv_clip_sgd_workspace": (_c_size_t, []),
    "sv_clip_sgd_step": (_c_int, [_P, _P, _c_long, _c_float, _c_float, _c_int, _P, _P, _P]),
}

ERRORS = {-1: "invalid argument (SV_EARG)", -2: "misaligned pointer/leading dim (SV_EALIGN)",
          -3: "unsupported shape (SV_ESHAPE)"}

_lib = None


class NativeLibraryError(RuntimeError):
    pass


def lib():
    """The loaded library (loaded once).  Raises NativeLibraryError if absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeLibraryError(
                f"{LIB_PATH} not found: build it with `make` (or __graft_entry__.build()); "
                "there is no non-native fallback")
        try:
            h = ctypes.CDLL(LIB_PATH)
        except OSError as e:
            raise NativeLibraryError(f"failed to load {LIB_PATH}: {e}") from e
        for name, (res, args) in SIGNATURES.items():
            f = getattr(h, name)
            f.restype = res
            f.argtypes = args
        _lib = h
    return _lib


def call(name, *args):
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        msg = ERRORS.get(rc, f"HIP error {rc}")
        raise RuntimeError(f"{name} failed: {msg}")


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_of(t):
    """hipStream_t of the current stream on the tensor's device."""
    return torch.cuda.current_stream(t.device).cuda_stream


def require_device(*tensors):
    for t in tensors:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError("pytorch_speaker_verification_amd ops run on the GPU only "
                               f"(got a {t.device} tensor); move the module/tensors with .to('cuda')")
        if t.dtype != torch.float32:
            raise RuntimeError(f"expected float32 tensors, got {t.dtype}")
        if not t.is_contiguous():
            raise RuntimeError("expected contiguous tensors")
