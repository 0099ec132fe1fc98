"""Scalar-quantise + packbits encode path of the ``VectorDBInt{4,8,16}{,Global}`` classes on MI355X.

``encode(mode, X, limit)`` runs one gfx950 kernel launch (``vrq_encode``, one
wave per vector) over a whole batch of embeddings resident in HBM and returns
device tensors.  The classes below mirror the reference's static encoder
methods (same names, same argument meaning, same return types: NumPy arrays,
plus ``(q, min, max)`` tuples for the local quantizers) so reference call sites
keep working; they accept one vector (1-D) or a batch (2-D):

=====================  ==========================================  ==================
reference              method                                       mode
=====================  ==========================================  ==================
VectorDBInt8Global     ``_quantize_to_int8`` (``:130-142``)          ``int8g``
VectorDBInt16Global    ``_quantize_to_int16`` (``:130-142``)         ``int16g``
VectorDBInt4Global     ``_quantize_to_int4`` (``:129-164``, bug)     ``int4g``
VectorDBInt8           ``_quantize_to_int8`` (``:114-126``)          ``int8``
VectorDBInt4           ``_quantize_to_int4`` (``:116-154``)          ``int4``
VectorDBInt16          ``_to_binary`` on int16 (``:148-157``)        ``bin16``
all of them            ``_to_binary`` (e.g. ``VectorDBInt8Global.py:154-160``)
=====================  ==========================================  ==================
"""
from __future__ import annotations

import numpy as np
import torch

from . import _native as N
from .index import _device, as_device_tensor


def encode(mode: str, X, limit: float = 0.3, device=None) -> dict:
    """Batch encode on device.  X: f32[n, d] (i16[n, d] for ``bin16``).

    Returns ``{"codes": u8[n, d/8], "q": int8[n,d] | int16[n,d] | int8[n,d/2] | None,
    "minmax": f64[n,2] | None}`` as device tensors.
    """
    if mode not in N.ENC_MODES:
        raise ValueError(f"unknown encode mode {mode!r}")
    dev = _device(device)
    in_dtype = torch.int16 if mode == "bin16" else torch.float32
    X = as_device_tensor(X, in_dtype, dev)
    if X.dim() == 1:
        X = X.reshape(1, -1)
    n, d = X.shape
    codes = torch.empty((n, d // 8), dtype=torch.uint8, device=dev)
    q = None
    if mode in ("int8g", "int8", "cohere"):
        q = torch.empty((n, d), dtype=torch.int8, device=dev)
    elif mode == "int16g":
        q = torch.empty((n, d), dtype=torch.int16, device=dev)
    elif mode in ("int4g", "int4"):
        q = torch.empty((n, (d + 1) // 2), dtype=torch.int8, device=dev)
    mm = torch.empty((n, 2), dtype=torch.float64, device=dev) if mode in ("int8", "int4") else None
    lib = N.load()
    with torch.cuda.device(dev):
        rc = lib.vrq_encode(N.ENC_MODES[mode], N.ptr(X), n, d, float(limit), N.ptr(codes), N.ptr(q), N.ptr(mm),
                            N.stream_handle(dev))
    N.check(rc, f"vrq_encode({mode})")
    return {"codes": codes, "q": q, "minmax": mm}


def int8_row_norms(x8: torch.Tensor) -> torch.Tensor:
    """float64 ``np.linalg.norm`` of every int8 row (``CohereEnhancedVectorDB.py:308``)."""
    x8 = x8.contiguous()
    n, d = x8.shape
    out = torch.empty((n,), dtype=torch.float64, device=x8.device)
    lib = N.load()
    with torch.cuda.device(x8.device):
        rc = lib.vrq_int8_row_norms(N.ptr(x8), n, d, N.ptr(out), N.stream_handle(x8.device))
    N.check(rc, "vrq_int8_row_norms")
    return out


def _host(x: torch.Tensor, one: bool):
    a = x.cpu().numpy()
    return a[0] if one else a


def _to_binary(embedding, mode="int8g"):
    one = np.ndim(embedding) == 1
    return _host(encode(mode, embedding, 1.0)["codes"], one)


class _Binary:
    @staticmethod
    def _to_binary(embedding):
        """packbits(embedding > np.mean(embedding)) (MSB-first)."""
        return _to_binary(embedding, "int8g")


class VectorDBInt8Global(_Binary):
    @staticmethod
    def _quantize_to_int8(embedding, limit: float):
        one = np.ndim(embedding) == 1
        return _host(encode("int8g", embedding, limit)["q"], one)

    @staticmethod
    def _dequantize_int8(emb_int8, limit: float):
        """``VectorDBInt8Global.py:144-152``: int8 * float32(limit/127)."""
        return np.asarray(emb_int8).astype(np.float32) * (limit / 127.0)


class VectorDBInt16Global(_Binary):
    @staticmethod
    def _quantize_to_int16(embedding, limit: float):
        one = np.ndim(embedding) == 1
        return _host(encode("int16g", embedding, limit)["q"], one)

    @staticmethod
    def _dequantize_int16(emb_int16, limit: float):
        """``VectorDBInt16Global.py:144-152``."""
        return np.asarray(emb_int16).astype(np.float32) * (limit / 32767.0)


class VectorDBInt4Global(_Binary):
    @staticmethod
    def _quantize_to_int4(embedding, limit: float):
        """Reproduces the reference: ``limit`` is ignored (per-vector 7/max|x| scale)."""
        one = np.ndim(embedding) == 1
        return _host(encode("int4g", embedding, 1.0)["q"], one)


class VectorDBInt8(_Binary):
    @staticmethod
    def _quantize_to_int8(embedding):
        one = np.ndim(embedding) == 1
        r = encode("int8", embedding)
        q, mm = _host(r["q"], one), r["minmax"].cpu().numpy()
        if one:
            return q, np.float32(mm[0, 0]), np.float32(mm[0, 1])
        return q, mm.astype(np.float32)[:, 0], mm.astype(np.float32)[:, 1]


class VectorDBInt4(_Binary):
    @staticmethod
    def _quantize_to_int4(embedding):
        one = np.ndim(embedding) == 1
        r = encode("int4", embedding)
        q, mm = _host(r["q"], one), r["minmax"].cpu().numpy()
        if one:
            return q, float(mm[0, 0]), float(mm[0, 1])
        return q, mm[:, 0], mm[:, 1]


class VectorDBInt16:
    @staticmethod
    def _to_binary(embedding):
        """``VectorDBInt16.py:148-157``: packbits(int16 > float64 mean)."""
        return _to_binary(embedding, "bin16")
