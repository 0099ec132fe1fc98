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


_DEQ_MODES = {"int8g": 0, "int16g": 1, "int4g": 2, "int8": 3, "int4": 4}


def dequantize(mode: str, q, minmax=None, limit: float = 0.0, dim: int = None, device=None) -> torch.Tensor:
    """Device ``_dequantize_*`` of the VectorDB* classes for a batch of rows (``vrq_dequantize``):
    ``int8g``/``int16g``/``int4g`` take the global ``limit``, ``int8``/``int4`` the per-row
    (min, max) f64[n, 2].  Returns f32[n, dim] on the device, bit-identical to the reference."""
    dev = _device(device)
    dt = {"int8g": torch.int8, "int8": torch.int8, "int16g": torch.int16, "int4g": torch.int8, "int4": torch.int8}[mode]
    q = as_device_tensor(q, dt, dev)
    if q.dim() == 1:
        q = q.reshape(1, -1)
    n = q.shape[0]
    d = dim if dim is not None else (2 * q.shape[1] if mode in ("int4g", "int4") else q.shape[1])
    mm = as_device_tensor(np.asarray(minmax, np.float64).reshape(n, 2), torch.float64, dev) if minmax is not None else None
    out = torch.empty((n, d), dtype=torch.float32, device=dev)
    lib = N.load()
    with torch.cuda.device(dev):
        rc = lib.vrq_dequantize(_DEQ_MODES[mode], N.ptr(q), N.ptr(mm), n, d, float(limit), N.ptr(out),
                                N.stream_handle(dev))
    N.check(rc, f"vrq_dequantize({mode})")
    return out


def vectordb_search(mode: str, codes: torch.Tensor, q: torch.Tensor, qf: torch.Tensor, qb: torch.Tensor, k: int = 10,
                    binary_oversample: int = 10, minmax: torch.Tensor = None, limit: float = 0.0,
                    rescore_row: torch.Tensor = None):
    """``VectorDBInt{4,8,16}{,Global}.search`` for a query batch (e.g. VectorDBInt8Global.py:205-252):
    Phase I Hamming top-``k * binary_oversample`` over the ubinary codes (``vrq_hamming_topk``, FAISS
    order), Phase II ``float(np.dot(query_float, doc_emb))`` (``vrq_rescore_dequant``), Python's stable
    sort by score descending, first k.  ``doc_emb`` is the dequantised row of ``mode`` or, for
    ``mode="f32"`` (the ``compare_float32`` branch, ``:239-240``), the f32 float row ``q``.
    ``mode="bin16"`` (VectorDBInt16.search) stops after Phase I and ranks by Hamming distance.
    ``rescore_row`` (i64[n], optional) maps an index row to the row whose stored vector the
    reference's ``doc_db[str(id)]`` lookup returns (the last add of a duplicated id).
    Returns (rows i64[nq, k], hamming i32[nq, k], score f64[nq, k]) on the device; rows past the
    corpus are -1 (score NaN)."""
    dev = codes.device
    n, cb = codes.shape
    nq = qb.shape[0]
    K = min(k * binary_oversample, n)
    lib = N.load()
    dist = torch.empty((nq, K), dtype=torch.int32, device=dev)
    rows = torch.empty((nq, K), dtype=torch.int64, device=dev)
    ws = torch.empty((max(8, lib.vrq_hamming_topk_workspace_size(n, cb, nq, K)),), dtype=torch.uint8, device=dev)
    with torch.cuda.device(dev):
        N.check(lib.vrq_hamming_topk(N.ptr(codes), n, cb, 0, N.ptr(qb), nq, K, N.ptr(dist), N.ptr(rows), N.ptr(ws),
                                     ws.numel(), N.stream_handle(dev)), "vrq_hamming_topk")
    if mode == "bin16":
        kk = min(k, K)
        return rows[:, :kk], dist[:, :kk], dist[:, :kk].to(torch.float64)
    if q is None or q.shape[0] != n or (minmax is not None and minmax.shape[0] != n):
        # the ABI indexes q / minmax by candidate row and cannot see their lengths
        raise N.VrqNativeError(f"vectordb_search: {n} code rows but {None if q is None else q.shape[0]} stored rows")
    cand = rows
    if rescore_row is not None:
        cand = torch.where(rows >= 0, rescore_row[rows.clamp_min(0)], rows).contiguous()
    score = torch.empty((nq, K), dtype=torch.float64, device=dev)
    d = qf.shape[1]
    m = N.VRQ_RESCORE_F32 if mode == "f32" else _DEQ_MODES[mode]
    with torch.cuda.device(dev):
        N.check(lib.vrq_rescore_dequant(m, N.ptr(qf), nq, d, N.ptr(q), N.ptr(minmax), float(limit), n,
                                        N.ptr(cand), K, N.ptr(score), N.stream_handle(dev)), "vrq_rescore_dequant")
    # Python's stable sort by score desc over the Phase-I order (VectorDBInt8Global.py:251);
    # missing candidates (-1) sort last, -0.0 ties +0.0
    key = torch.where(rows >= 0, score + 0.0, torch.full_like(score, float("-inf")))
    o = torch.sort(-key, dim=1, stable=True).indices[:, :k]
    return torch.gather(rows, 1, o), torch.gather(dist, 1, o), torch.gather(score, 1, o)


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
        """``VectorDBInt8Global.py:144-152``: int8 * float32(limit/127) (on the device)."""
        one = np.ndim(emb_int8) == 1
        return _host(dequantize("int8g", emb_int8, limit=limit), one)


class VectorDBInt16Global(_Binary):
    @staticmethod
    def _quantize_to_int16(embedding, limit: float):
        one = np.ndim(embedding) == 1
        return _host(encode("int16g", embedding, limit)["q"], one)

    @staticmethod
    def _dequantize_int16(emb_int16, limit: float):
        """``VectorDBInt16Global.py:144-152`` (on the device)."""
        one = np.ndim(emb_int16) == 1
        return _host(dequantize("int16g", emb_int16, limit=limit), one)


class VectorDBInt4Global(_Binary):
    @staticmethod
    def _quantize_to_int4(embedding, limit: float):
        """Reproduces the reference: ``limit`` is ignored (per-vector 7/max|x| scale)."""
        one = np.ndim(embedding) == 1
        return _host(encode("int4g", embedding, 1.0)["q"], one)

    @staticmethod
    def _dequantize_int4(q_packed, length: int, limit: float):
        """``VectorDBInt4Global.py:166-188`` (on the device)."""
        one = np.ndim(q_packed) == 1
        return _host(dequantize("int4g", np.asarray(q_packed).astype(np.int8), limit=limit, dim=length), one)


class VectorDBInt8(_Binary):
    @staticmethod
    def _quantize_to_int8(embedding):
        one = np.ndim(embedding) == 1
        r = encode("int8", embedding)
        q, mm = _host(r["q"], one), r["minmax"].cpu().numpy()
        if one:
            return q, np.float32(mm[0, 0]), np.float32(mm[0, 1])
        return q, mm.astype(np.float32)[:, 0], mm.astype(np.float32)[:, 1]

    @staticmethod
    def _dequantize_int8(emb_int8, min_max):
        """``VectorDBInt8.py:129-138`` (on the device); min_max = (min, max) or an [n, 2] array."""
        one = np.ndim(emb_int8) == 1
        return _host(dequantize("int8", emb_int8, minmax=np.asarray(min_max, np.float64)), one)


class VectorDBInt4(_Binary):
    @staticmethod
    def _quantize_to_int4(embedding):
        one = np.ndim(embedding) == 1
        r = encode("int4", embedding)
        q, mm = _host(r["q"], one), r["minmax"].cpu().numpy()
        if one:
            return q, float(mm[0, 0]), float(mm[0, 1])
        return q, mm[:, 0], mm[:, 1]

    @staticmethod
    def _dequantize_int4(q_packed, length: int, min_max):
        """``VectorDBInt4.py:157-184`` (on the device)."""
        one = np.ndim(q_packed) == 1
        return _host(dequantize("int4", np.asarray(q_packed).astype(np.int8), minmax=np.asarray(min_max, np.float64),
                                dim=length), one)


class VectorDBInt16:
    @staticmethod
    def _to_binary(embedding):
        """``VectorDBInt16.py:148-157``: packbits(int16 > float64 mean)."""
        return _to_binary(embedding, "bin16")
