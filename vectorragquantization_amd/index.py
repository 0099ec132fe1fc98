"""Device-resident binary index with FAISS ``IndexBinaryIDMap2`` semantics.

Replaces ``faiss.IndexBinaryIDMap2(faiss.IndexBinaryFlat(d))`` as the
reference creates it (``CohereEnhancedVectorDB.py:126``; also
``VectorDBInt8Global.py:84`` and the other ``VectorDBInt*`` classes).  The
protocol the reference exercises is kept: ``add_with_ids`` (``:217``),
``search`` (``:268``), ``reconstruct`` (``:286``), ``remove_ids`` (``:334``),
``ntotal`` (``:247,267,350``), plus FAISS's on-disk ``IBM2`` format
(``faiss.write_index_binary`` / ``read_index_binary``, ``:123,346``).

Layout in HBM: codes ``u8[capacity, d/8]`` row-major (row = internal index =
insertion order after compaction), ``id_map i64[capacity]``; capacity grows
geometrically so appends are amortised O(1).  Search runs the hand-written
gfx950 Phase-I kernels through ``libvrq.so`` (``vrq_hamming_topk``); there is no
CPU fallback.
"""
from __future__ import annotations

import struct

import numpy as np
import torch

from . import _native as N

INT32_MAX = np.iinfo(np.int32).max


def _device(device=None) -> torch.device:
    if device is not None:
        return torch.device(device)
    if not torch.cuda.is_available():
        raise N.VrqNativeError("vectorragquantization_amd needs a ROCm GPU (torch.cuda.is_available() is False)")
    return torch.device("cuda", torch.cuda.current_device())


def as_device_tensor(x, dtype, device) -> torch.Tensor:
    if isinstance(x, torch.Tensor):
        return x.to(device=device, dtype=dtype).contiguous()
    a = np.ascontiguousarray(np.asarray(x), dtype=torch_to_np(dtype))
    if not a.flags.writeable:      # read-only (e.g. np.load) arrays: torch.from_numpy needs a writable buffer
        a = a.copy()
    return torch.from_numpy(a).to(device)


def torch_to_np(dtype):
    return {torch.uint8: np.uint8, torch.int8: np.int8, torch.int16: np.int16, torch.int32: np.int32,
            torch.int64: np.int64, torch.float32: np.float32, torch.float64: np.float64}[dtype]


def ibm2_pack(d: int, codes: np.ndarray, ids: np.ndarray) -> bytes:
    """FAISS ``write_index_binary`` image of ``IndexBinaryIDMap2(IndexBinaryFlat(d))``:
    "IBM2" + header(d, code_size, ntotal, is_trained, metric) + "IBxF" + header + xb + id_map."""
    n = int(codes.shape[0])
    hdr = struct.pack("<iiqbi", d, d // 8, n, 1, 1)
    xb = np.ascontiguousarray(codes, dtype=np.uint8).tobytes()
    return (b"IBM2" + hdr + b"IBxF" + hdr + struct.pack("<q", len(xb)) + xb + struct.pack("<q", n)
            + np.ascontiguousarray(ids, dtype="<i8").tobytes())


def ibm2_unpack(b: bytes):
    """Inverse of ``ibm2_pack`` -> (d, codes u8[n, d/8], ids i64[n])."""
    if b[:4] != b"IBM2" or b[25:29] != b"IBxF":
        raise ValueError("not a FAISS IndexBinaryIDMap2(IndexBinaryFlat) file")
    d, cs, nt, _, _ = struct.unpack("<iiqbi", b[4:25])
    off = 50
    nb, = struct.unpack("<q", b[off:off + 8]); off += 8
    xb = np.frombuffer(b, np.uint8, nb, off).reshape(nt, cs); off += nb
    ni, = struct.unpack("<q", b[off:off + 8]); off += 8
    ids = np.frombuffer(b, "<i8", ni, off)
    return d, xb, ids


class _GrowBuffer:
    """Row-major device buffer with geometric capacity growth."""

    def __init__(self, row_shape, dtype, device):
        self.row_shape = tuple(row_shape)
        self.dtype = dtype
        self.device = device
        self.buf = torch.empty((0, *self.row_shape), dtype=dtype, device=device)
        self.n = 0

    def view(self) -> torch.Tensor:
        return self.buf[: self.n]

    def append(self, x: torch.Tensor) -> None:
        m = x.shape[0]
        need = self.n + m
        if need > self.buf.shape[0]:
            cap = max(need, int(self.buf.shape[0] * 1.5) + 1024)
            nb = torch.empty((cap, *self.row_shape), dtype=self.dtype, device=self.device)
            if self.n:
                nb[: self.n].copy_(self.buf[: self.n])
            self.buf = nb
        self.buf[self.n:need].copy_(x)
        self.n = need

    def keep(self, mask: torch.Tensor) -> None:
        kept = self.view()[mask]
        self.buf = torch.empty((max(kept.shape[0], 1), *self.row_shape), dtype=self.dtype, device=self.device)
        self.buf[: kept.shape[0]].copy_(kept)
        self.n = kept.shape[0]


class BinaryIndexIDMap2:
    """``faiss.IndexBinaryIDMap2(IndexBinaryFlat(d))`` on one MI355X (HBM-resident)."""

    def __init__(self, d: int = 1024, device=None):
        if d % 8:
            raise ValueError("d must be a multiple of 8")
        self.d = d
        self.code_size = d // 8
        self.device = _device(device)
        self._codes = _GrowBuffer((self.code_size,), torch.uint8, self.device)
        self._ids = _GrowBuffer((), torch.int64, self.device)
        self._rev = {}        # external id -> row (last add wins, like FAISS rev_map)
        self._dup = False     # some external id occupies more than one row
        self.is_trained = True

    # -- FAISS protocol ------------------------------------------------------
    @property
    def ntotal(self) -> int:
        return self._codes.n

    @property
    def codes(self) -> torch.Tensor:
        return self._codes.view()

    @property
    def id_map(self) -> torch.Tensor:
        return self._ids.view()

    def add_with_ids(self, x, ids) -> None:
        x = as_device_tensor(x, torch.uint8, self.device).reshape(-1, self.code_size)
        # a private, writable copy (torch.from_numpy warns on read-only arrays, e.g. a mmap'd index.bin)
        ids_np = np.array(ids.cpu() if isinstance(ids, torch.Tensor) else ids, dtype=np.int64, copy=True).reshape(-1)
        if ids_np.shape[0] != x.shape[0]:
            raise ValueError("add_with_ids: codes and ids differ in length")
        base = self.ntotal
        self._codes.append(x)
        self._ids.append(torch.from_numpy(ids_np).to(self.device))
        for j, e in enumerate(ids_np.tolist()):
            if e in self._rev:
                self._dup = True
            self._rev[e] = base + j

    def search(self, q, k: int):
        """(D i32[nq,k], L i64[nq,k]) on the host, like ``faiss.Index.search``."""
        D, R = self.search_device(q, k)
        L = torch.where(R >= 0, self.id_map[R.clamp_min(0)] if self.ntotal else R, R)
        return D.cpu().numpy(), L.cpu().numpy()

    def search_device(self, q, k: int):
        """Phase I on device -> (dist i32[nq,k], internal row i64[nq,k]) device tensors."""
        q = as_device_tensor(q, torch.uint8, self.device).reshape(-1, self.code_size)
        nq = q.shape[0]
        D = torch.empty((nq, k), dtype=torch.int32, device=self.device)
        R = torch.empty((nq, k), dtype=torch.int64, device=self.device)
        lib = N.load()
        n = self.ntotal
        ws_bytes = lib.vrq_hamming_topk_workspace_size(n, self.code_size, nq, k) if n and nq and k else 0
        ws = torch.empty(max(ws_bytes, 8), dtype=torch.uint8, device=self.device)
        with torch.cuda.device(self.device):
            rc = lib.vrq_hamming_topk(N.ptr(self.codes) if n else 0, n, self.code_size, 0, N.ptr(q), nq, k,
                                      N.ptr(D), N.ptr(R), N.ptr(ws), ws.numel(), N.stream_handle(self.device))
        N.check(rc, "vrq_hamming_topk")
        return D, R

    def reconstruct(self, key) -> np.ndarray:
        row = self._rev[int(key)]
        return self.codes[row].cpu().numpy()

    def remove_ids(self, ids) -> int:
        rm = torch.as_tensor(np.asarray(ids, dtype=np.int64).reshape(-1), device=self.device)
        keep = ~torch.isin(self.id_map, rm)
        nrm = int((~keep).sum().item())
        if nrm:
            self._compact(keep)
        return nrm

    def reset(self) -> None:
        self._codes = _GrowBuffer((self.code_size,), torch.uint8, self.device)
        self._ids = _GrowBuffer((), torch.int64, self.device)
        self._rev = {}
        self._dup = False

    # -- helpers ---------------------------------------------------------------
    def _compact(self, keep: torch.Tensor) -> None:
        self._codes.keep(keep)
        self._ids.keep(keep)
        self._rebuild_rev()

    def _rebuild_rev(self) -> None:
        ids = self.id_map.cpu().numpy().tolist()
        self._rev = {}
        self._dup = False
        for j, e in enumerate(ids):
            if e in self._rev:
                self._dup = True
            self._rev[e] = j

    def rescore_rows(self):
        """Per-row row used by Phases II/III (``rev_map[id_map[r]]``) or None when ids are unique."""
        if not self._dup:
            return None
        ids = self.id_map.cpu().numpy()
        return torch.from_numpy(np.array([self._rev[int(e)] for e in ids], dtype=np.int64)).to(self.device)

    # -- FAISS IBM2 on-disk format (faiss.write_index_binary / read_index_binary) ----
    def to_bytes(self) -> bytes:
        return ibm2_pack(self.d, self.codes.cpu().numpy(), self.id_map.cpu().numpy())

    def write(self, path: str) -> None:
        with open(path, "wb") as f:
            f.write(self.to_bytes())

    @classmethod
    def from_bytes(cls, b: bytes, device=None) -> "BinaryIndexIDMap2":
        d, xb, ids = ibm2_unpack(b)
        idx = cls(d, device)
        if xb.shape[0]:
            idx.add_with_ids(xb, ids)
        return idx

    @classmethod
    def read(cls, path: str, device=None) -> "BinaryIndexIDMap2":
        with open(path, "rb") as f:
            return cls.from_bytes(f.read(), device)
