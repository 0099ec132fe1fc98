"""ctypes binding of libvrq.so (include/vrq.h).

The product path has no CPU fallback: if the HIP library is missing or cannot
be loaded, every call raises ``VrqNativeError`` -- tests on a GPU box therefore
fail loudly instead of silently running something else.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

from . import _build

VRQ_OK = 0
VRQ_EINVAL = -1
VRQ_EHIP = -2
VRQ_EUNSUPPORTED = -3
VRQ_EWORKSPACE = -4

VRQ_SEARCH_PHASE1_ONLY = 1
VRQ_SEARCH_SHARD = 2
VRQ_SEARCH_SCAN_VALU = 4
VRQ_SEARCH_SCAN_MFMA = 8
VRQ_SCAN_STAGE_PREFIX = 16
VRQ_SCAN_STAGE_MATRIX = 32
VRQ_SCAN_STAGE_SUFFIX = 64
VRQ_SCAN_STAGE_RECHECK = 128
VRQ_GEMM_BINARY = 2
VRQ_GEMM_INT8_COSINE = 3
VRQ_GEMM_FLOAT_IP = 4
VRQ_GEMM_STAGE_SAMPLE = 16
VRQ_GEMM_STAGE_MAIN = 32
VRQ_GEMM_STAGE_FINISH = 64
VRQ_GEMM_NO_FALLBACK = 128
VRQ_RESCORE_F32 = 16  # vrq_rescore_dequant: compare_float32 rows
VRQ_SCAN_KIND_VALU = 0
VRQ_SCAN_KIND_MFMA = 1

ENC_MODES = {
    "int8g": 0,   # VectorDBInt8Global
    "int16g": 1,  # VectorDBInt16Global
    "int4g": 2,   # VectorDBInt4Global (limit ignored, reference bug)
    "int8": 3,    # VectorDBInt8
    "int4": 4,    # VectorDBInt4
    "bin16": 5,   # VectorDBInt16._to_binary
    "cohere": 6,  # synthetic Cohere provider (int8 global + sign bits)
}

# name -> (restype, argtypes); mirrors include/vrq.h
_P, _I32, _I64, _SZ, _D = C.c_void_p, C.c_int32, C.c_int64, C.c_size_t, C.c_double
SIGNATURES = {
    "vrq_abi_version": (C.c_int, []),
    "vrq_strerror": (C.c_char_p, [C.c_int]),
    "vrq_hamming_topk_workspace_size": (_SZ, [_I64, _I32, _I32, _I32]),
    "vrq_hamming_topk": (C.c_int, [_P, _I64, _I32, _I64, _P, _I32, _I32, _P, _P, _P, _SZ, _P]),
    "vrq_search3_workspace_size": (_SZ, [_I64, _I32, _I32, _I32]),
    "vrq_search3": (C.c_int, [_P, _P, _P, _P, _I64, _I32, _I64, _P, _P, _I32, _I32, _I32, _I32, _I32,
                              _P, _P, _P, _P, _P, _P, _SZ, _P]),
    "vrq_search3_scan": (C.c_int, [_P, _I64, _I32, _P, _I32, _I32, _I32, _P, _SZ, _P]),
    "vrq_search3_finish": (C.c_int, [_P, _P, _P, _P, _I64, _I32, _I64, _P, _I32, _I32, _I32, _I32, _I32,
                                     _P, _P, _P, _P, _P, _P, _SZ, _P]),
    "vrq_scan_kind": (C.c_int, [_I64, _I32, _I32, _I32, _I32, _P]),
    "vrq_scan_plan": (C.c_int, [_I64, _I32, _I32, _I32, _I32, _P]),
    "vrq_scan_sample_plan": (C.c_int, [_I64, _I32, _I32, _I32, _I32, _P]),
    "vrq_merge_shards": (C.c_int, [_I32, _I32, _I32, _P, _P, _P, _P, _P, _I32, _I32, _P, _P, _P, _P, _P, _P, _P]),
    "vrq_rescore_binary": (C.c_int, [_P, _I32, _I32, _P, _I64, _P, _I32, _P, _P]),
    "vrq_rescore_int8_cosine": (C.c_int, [_P, _I32, _I32, _P, _P, _I64, _P, _I32, _P, _P]),
    "vrq_encode": (C.c_int, [_I32, _P, _I64, _I32, _D, _P, _P, _P, _P]),
    "vrq_int8_row_norms": (C.c_int, [_P, _I64, _I32, _P, _P]),
    "vrq_dequantize": (C.c_int, [_I32, _P, _P, _I64, _I32, _D, _P, _P]),
    "vrq_rescore_dequant": (C.c_int, [_I32, _P, _I32, _I32, _P, _P, _D, _I64, _P, _I32, _P, _P]),
    "vrq_gemm_topk_workspace_size": (_SZ, [_I32, _I64, _I32, _I32, _I32]),
    "vrq_gemm_topk_pieces": (C.c_int, []),
    "vrq_gemm_topk_plan": (C.c_int, [_I32, _I64, _I32, _I32, _I32, _P]),
    "vrq_gemm_topk_layout": (C.c_int, [_I32, _I64, _I32, _I32, _I32, _P]),
    "vrq_gemm_topk": (C.c_int, [_I32, _P, _P, _P, _I64, _I32, _I64, _P, _I32, _I32, _I32, _P, _P, _P, _P, _SZ,
                                _P]),
    "vrq_flat_ip_prepare": (C.c_int, [_P, _I64, _I32, _P, _P, _P, _P]),
    "vrq_flat_ip_topk": (C.c_int, [_P, _P, _P, _P, _I64, _I32, _I64, _P, _I32, _I32, _I32, _P, _P, _P, _P, _SZ,
                                   _P]),
}


class VrqNativeError(RuntimeError):
    pass


_lib = None
_lock = threading.Lock()


_override = None


def use_library(path: str) -> None:
    """Load ``path`` instead of the in-tree libvrq.so in this process (tools/ sweeps of probe variants
    and tests only; call before the first load()).  The product never reads the environment for it."""
    global _override, _lib
    if _lib is not None:
        raise VrqNativeError("use_library() after the library was loaded")
    _override = path


def lib_path() -> str:
    return _override or _build.LIB


def _open(path: str, default: str, probe: bool = False):
    if not os.path.exists(path) or (path == default and not _build.up_to_date(default)):
        try:
            _build.build(probe=probe)
        except Exception as e:  # no hipcc on this host and no prebuilt library
            if not os.path.exists(path):
                raise VrqNativeError(f"{os.path.basename(path)} missing and cannot be built: {e}") from e
    try:
        lib = C.CDLL(path)
    except OSError as e:
        raise VrqNativeError(f"cannot load {path}: {e}") from e
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.vrq_abi_version() != 1:
        raise VrqNativeError("libvrq ABI version mismatch")
    return lib


def load():
    """Load (building first if needed and possible) libvrq.so; raise on failure."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            _lib = _open(lib_path(), _build.LIB)
        return _lib


_probe = None


def load_probe():
    """The probe build libvrq_probe.so: the same kernels, but its planners read the VRQ_* tuning
    overrides (VRQ_SAMPLE_DIV, VRQ_MFMA_MB, VRQ_MFMA_ROWS, VRQ_GEMM_SAMPLE_DIV, VRQ_GEMM_CHUNK_MULT)
    from the environment.  For sweeps and tests only; the product path always uses load()."""
    global _probe
    with _lock:
        if _probe is None:
            _probe = _open(_build.PROBE_LIB, _build.PROBE_LIB, probe=True)
        return _probe


def check(rc: int, what: str) -> None:
    if rc != VRQ_OK:
        msg = load().vrq_strerror(rc).decode()
        raise VrqNativeError(f"{what} failed: {msg} ({rc})")


def ptr(t) -> int:
    """Raw device pointer of a torch tensor (None -> NULL)."""
    return 0 if t is None else int(t.data_ptr())


def stream_handle(device=None) -> int:
    import torch
    return int(torch.cuda.current_stream(device).cuda_stream)
