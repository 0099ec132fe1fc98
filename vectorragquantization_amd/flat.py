"""``CohereVectorDBFloat`` on MI355X: exact float32 inner-product search (FAISS
``IndexIDMap(IndexFlatIP(d))``) on the matrix cores, behind the reference's surface.

Reference: ``CohereVectorDBFloat.py`` (aitrailblazer/VectorRAGQuantization).  Same constructor
(``:19-36``), config handling (``:38-53``), ``add_documents`` (``:103-140``: dedupe, 64-doc batches),
``search`` (``:142-172``: ``{"doc_id", "score", "doc"}`` dicts, stable re-sort by score desc),
``remove_document`` (``:174-180``), ``save`` (``:182-185``: ``index.faiss`` in FAISS's ``IxMp``/``IxFI``
format, byte-compatible with the reference's file), ``__len__`` (``:187``).  Batch additions that
bypass HTTP: ``add_vectors`` / ``search_vectors``.

Device layout (rows = FAISS internal order): the float32 rows xf[n, 1024] (the exact scores read
them), the matrix pass's per-row-scaled int8 copy x8[n, 1024] and 1/scale f64[n], and the corpus
error bounds f64[2] -- all from ``vrq_flat_ip_prepare`` at add time.  A search is one
``vrq_flat_ip_topk`` call for the whole query batch.
"""
from __future__ import annotations

import json
import logging
import os
import struct
from typing import Dict, List

import numpy as np
import torch

from . import _native as N
from .docstore import DocStoreError, RocksDictReader, is_rocksdict_dir
from .index import _GrowBuffer, _device, as_device_tensor

logger = logging.getLogger(__name__)


def flat_ip_prepare(xf: torch.Tensor, bounds: torch.Tensor):
    """``vrq_flat_ip_prepare``: (x8 int8[n, d], inv_scale f64[n]) of float32 rows; max-accumulates
    the corpus bounds into ``bounds`` (f64[2], zero before the first batch)."""
    n, d = xf.shape
    x8 = torch.empty((n, d), dtype=torch.int8, device=xf.device)
    inv = torch.empty((n,), dtype=torch.float64, device=xf.device)
    N.check(N.load().vrq_flat_ip_prepare(N.ptr(xf), n, d, N.ptr(x8), N.ptr(inv), N.ptr(bounds),
                                         N.stream_handle(xf.device)), "vrq_flat_ip_prepare")
    return x8, inv


def flat_ip_topk(xf: torch.Tensor, x8: torch.Tensor, inv_scale: torch.Tensor, bounds: torch.Tensor,
                 qf: torch.Tensor, k: int, row_offset: int = 0, flags: int = 0,
                 workspace: torch.Tensor | None = None):
    """Exact IndexFlatIP top-k of a query batch (``vrq_flat_ip_topk``).  Returns device tensors
    (count i32[nq], rows i64[nq, k] (+ row_offset, -1 padded), scores f64[nq, k] holding float32
    values), ordered (score desc, row asc)."""
    dev = qf.device
    nq, n = qf.shape[0], xf.shape[0]
    cnt = torch.full((nq,), -2, dtype=torch.int32, device=dev)  # -2: never written
    rows = torch.full((nq, k), -2, dtype=torch.int64, device=dev)
    scores = torch.empty((nq, k), dtype=torch.float64, device=dev)
    lib = N.load()
    need = lib.vrq_gemm_topk_workspace_size(N.VRQ_GEMM_FLOAT_IP, n, qf.shape[1], nq, k)
    if need == 0:
        raise N.VrqNativeError(f"vrq_flat_ip_topk: unsupported shape n={n} dim={qf.shape[1]} nq={nq} k={k}")
    if workspace is None or workspace.numel() < need:
        workspace = torch.empty((need,), dtype=torch.uint8, device=dev)
    N.check(lib.vrq_flat_ip_topk(N.ptr(xf), N.ptr(x8), N.ptr(inv_scale), N.ptr(bounds), n, qf.shape[1], row_offset,
                                 N.ptr(qf), nq, k, flags, N.ptr(cnt), N.ptr(rows), N.ptr(scores),
                                 N.ptr(workspace), workspace.numel(), N.stream_handle(dev)), "vrq_flat_ip_topk")
    stages = flags & (N.VRQ_GEMM_STAGE_SAMPLE | N.VRQ_GEMM_STAGE_MAIN | N.VRQ_GEMM_STAGE_FINISH)
    if (not stages or stages & N.VRQ_GEMM_STAGE_FINISH) and bool((cnt < 0).any()):
        # only with VRQ_GEMM_NO_FALLBACK in flags: the library left queries it could not serve on the
        # matrix path unwritten (count -1) instead of running the exact scan
        raise N.VrqNativeError("vrq_flat_ip_topk: queries needed the exact fallback, which VRQ_GEMM_NO_FALLBACK disabled")
    return cnt, rows, scores


# -- FAISS write_index / read_index image of IndexIDMap(IndexFlatIP(d)) -------------------------
def _hdr(d: int, n: int) -> bytes:
    # write_index_header: d, ntotal, two dummy idx_t (1 << 20), is_trained, metric (0 = inner product)
    return struct.pack("<iqqqbi", d, n, 1 << 20, 1 << 20, 1, 0)


def ixmp_pack(d: int, xf: np.ndarray, ids: np.ndarray) -> bytes:
    n = int(xf.shape[0])
    return b"".join([b"IxMp", _hdr(d, n), b"IxFI", _hdr(d, n), struct.pack("<q", n * d),
                     np.ascontiguousarray(xf, dtype="<f4").tobytes(), struct.pack("<q", n),
                     np.ascontiguousarray(ids, dtype="<i8").tobytes()])


def ixmp_unpack(b: bytes):
    if b[:4] != b"IxMp" or b[37:41] != b"IxFI":
        raise ValueError("not a FAISS IndexIDMap(IndexFlat) image")
    d, n = struct.unpack("<iq", b[4:16])
    metric, = struct.unpack("<i", b[33:37])
    if metric != 0:
        raise ValueError("index.faiss is not an inner-product index")
    off = 74
    nx, = struct.unpack("<q", b[off:off + 8])
    off += 8
    xf = np.frombuffer(b, "<f4", nx, off).reshape(n, d).copy()
    off += 4 * nx
    ni, = struct.unpack("<q", b[off:off + 8])
    off += 8
    ids = np.frombuffer(b, "<i8", ni, off).copy()
    return d, xf, ids


class FloatIndexIDMap:
    """``faiss.IndexIDMap(faiss.IndexFlatIP(d))`` on one MI355X (HBM-resident): ``add_with_ids``,
    ``search``, ``reconstruct``, ``remove_ids``, ``ntotal`` and the ``index.faiss`` format."""

    def __init__(self, d: int = 1024, device=None):
        self.d = d
        self.device = _device(device)
        self._xf = _GrowBuffer((d,), torch.float32, self.device)
        self._x8 = _GrowBuffer((d,), torch.int8, self.device)
        self._inv = _GrowBuffer((), torch.float64, self.device)
        self._ids = _GrowBuffer((), torch.int64, self.device)
        self.bounds = torch.zeros((2,), dtype=torch.float64, device=self.device)
        self._ws = None

    @property
    def ntotal(self) -> int:
        return self._xf.n

    @property
    def xf(self) -> torch.Tensor:
        return self._xf.view()

    @property
    def id_map(self) -> torch.Tensor:
        return self._ids.view()

    def add_with_ids(self, x, ids) -> None:
        ids_t = as_device_tensor(ids, torch.int64, self.device).reshape(-1)
        xf = as_device_tensor(x, torch.float32, self.device).reshape(ids_t.shape[0], self.d)
        if ids_t.shape[0] == 0:
            return
        with torch.cuda.device(self.device):
            x8, inv = flat_ip_prepare(xf, self.bounds)
        self._xf.append(xf)
        self._x8.append(x8)
        self._inv.append(inv)
        self._ids.append(ids_t)

    def search_rows(self, qf, k: int, flags: int = 0):
        """Device (count, rows, scores) of the exact top-k (internal rows); ``flags`` as
        ``vrq_flat_ip_topk`` (e.g. VRQ_GEMM_NO_FALLBACK)."""
        qf = as_device_tensor(qf, torch.float32, self.device).reshape(-1, self.d)
        lib = N.load()
        need = lib.vrq_gemm_topk_workspace_size(N.VRQ_GEMM_FLOAT_IP, self.ntotal, self.d, qf.shape[0], k)
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty((max(need, 8),), dtype=torch.uint8, device=self.device)
        with torch.cuda.device(self.device):
            return flat_ip_topk(self._xf.view(), self._x8.view(), self._inv.view(), self.bounds, qf, k,
                                flags=flags, workspace=self._ws)

    def search(self, q, k: int):
        """FAISS ``search``: numpy (distances f32[nq, k], labels i64[nq, k]); unused slots -FLT_MAX / -1."""
        q = np.asarray(q.cpu() if isinstance(q, torch.Tensor) else q, dtype=np.float32).reshape(-1, self.d)
        nq = q.shape[0]
        D = np.full((nq, k), -np.finfo(np.float32).max, dtype=np.float32)  # FAISS CMin neutral
        L = np.full((nq, k), -1, dtype=np.int64)
        if self.ntotal == 0 or k <= 0 or nq == 0:
            return D, L
        cnt, rows, scores = self.search_rows(q, k)
        cnt = cnt.cpu().numpy()
        r = rows.cpu().numpy()
        s = scores.cpu().numpy()
        ids = self.id_map.cpu().numpy()
        for j in range(nq):
            c = int(cnt[j])
            D[j, :c] = s[j, :c].astype(np.float32)
            L[j, :c] = ids[r[j, :c]]
        return D, L

    def reconstruct(self, key) -> np.ndarray:
        hit = (self.id_map == int(key)).nonzero()
        if hit.numel() == 0:
            raise RuntimeError(f"key {key} not found")
        return self.xf[int(hit[-1])].cpu().numpy()

    def remove_ids(self, ids) -> int:
        ids_t = as_device_tensor(ids, torch.int64, self.device).reshape(-1)
        keep = ~torch.isin(self.id_map, ids_t)
        removed = int(self.ntotal - int(keep.sum()))
        if removed:
            for b in (self._xf, self._x8, self._inv, self._ids):
                b.keep(keep)
        return removed  # the bounds stay valid upper bounds over the survivors

    def to_bytes(self) -> bytes:
        return ixmp_pack(self.d, self.xf.cpu().numpy(), self.id_map.cpu().numpy())

    def write(self, path: str) -> None:
        with open(path, "wb") as f:
            f.write(self.to_bytes())

    @classmethod
    def from_bytes(cls, b: bytes, device=None) -> "FloatIndexIDMap":
        d, xf, ids = ixmp_unpack(b)
        idx = cls(d, device)
        if xf.shape[0]:
            idx.add_with_ids(xf, ids)
        return idx

    @classmethod
    def read(cls, path: str, device=None) -> "FloatIndexIDMap":
        with open(path, "rb") as f:
            return cls.from_bytes(f.read(), device)


class CohereVectorDBFloat:
    """Drop-in for the reference class (``CohereVectorDBFloat.py:13``)."""

    def __init__(self, folder: str, model: str = "embed-english-v3.0", embedding_dim: int = 1024, *,
                 provider=None, device=None):
        if provider is None:  # the reference reads COHERE_EMBED_ENDPOINT / _KEY (:22-32)
            from .embed import CohereHTTPProvider
            provider = CohereHTTPProvider(model=model)
        self.provider = provider
        self.folder = folder
        self.model = model
        self.embedding_dim = embedding_dim
        self._setup_config(folder, model, embedding_dim)
        path = os.path.join(folder, "index.faiss")
        if os.path.exists(path):                                            # :55-64
            self.index = FloatIndexIDMap.read(path, device)
            logger.info("Existing float FAISS index loaded.")
        else:
            self.index = FloatIndexIDMap(embedding_dim, device)
        self.device = self.index.device
        self.texts: Dict[int, str] = {}
        self._load_texts()

    def _load_texts(self):
        """Document texts from this build's ``vrq_docs/texts.json`` (or a round-1 ``docs/texts.json``),
        else from the reference's RocksDict ``docs/`` (``{"doc": text}`` per id, :136; read by
        ``docstore.RocksDictReader``).  An index without a store is refused: the dedupe of
        ``add_documents`` (:108-111) and ``remove_document`` (:175) key on the store."""
        for p in (os.path.join(self.folder, "vrq_docs", "texts.json"), os.path.join(self.folder, "docs", "texts.json")):
            if os.path.exists(p):
                with open(p) as f:
                    self.texts = {int(a): b for a, b in json.load(f).items()}
                return
        docs = os.path.join(self.folder, "docs")
        if is_rocksdict_dir(docs):
            for key, val in RocksDictReader(docs).items():
                try:
                    did = int(key)
                except (TypeError, ValueError):
                    continue
                self.texts[did] = val.get("doc", "N/A") if isinstance(val, dict) else "N/A"
            return
        if self.index.ntotal:
            raise DocStoreError(f"{self.folder}: index.faiss holds {self.index.ntotal} rows but there is no document "
                                "store (docs/ RocksDict or vrq_docs/texts.json)")

    def _setup_config(self, folder: str, model: str, embedding_dim: int):
        config_path = os.path.join(folder, "config.json")
        if not os.path.exists(config_path):
            if os.path.exists(folder) and os.listdir(folder):
                raise Exception(f"Folder {folder} not empty but no config.json found. "
                                "To create new DB, folder must be empty or have config.json.")
            os.makedirs(folder, exist_ok=True)
            self.config = {"model": model, "embedding_dim": embedding_dim}
            with open(config_path, "w") as f:
                json.dump(self.config, f)
        else:
            with open(config_path) as f:
                self.config = json.load(f)

    def save(self):
        self.index.write(os.path.join(self.folder, "index.faiss"))
        p = os.path.join(self.folder, "vrq_docs")  # never inside the reference's RocksDB directory
        os.makedirs(p, exist_ok=True)
        with open(os.path.join(p, "texts.json"), "w") as f:
            json.dump({str(a): b for a, b in self.texts.items()}, f)
        logger.info("Float FAISS index saved to disk.")

    def __len__(self):
        return self.index.ntotal

    def add_vectors(self, doc_ids, xf, docs=None, save: bool = False) -> None:
        """Append pre-computed float32 embeddings -- ``:131-133`` without HTTP."""
        ids = np.asarray(doc_ids.cpu() if isinstance(doc_ids, torch.Tensor) else doc_ids, dtype=np.int64).reshape(-1)
        self.index.add_with_ids(xf, ids)
        if docs is None:
            docs = [""] * ids.shape[0]
        for i, d in zip(ids.tolist(), docs):
            self.texts[i] = d
        if save:
            self.save()

    def add_documents(self, doc_ids: List[int], docs: List[str], batch_size: int = 64, save: bool = True):
        if len(doc_ids) != len(docs):
            raise ValueError("doc_ids and docs must match length.")
        for doc_id in doc_ids:                                              # :108-111
            if int(doc_id) in self.texts:
                self.remove_document(doc_id, save=False)
        for start in range(0, len(docs), batch_size):                      # :114-137
            bi, bd = doc_ids[start:start + batch_size], docs[start:start + batch_size]
            emb = self.provider.embed(bd, "search_document", ["float"])
            if not emb:
                continue
            self.add_vectors(bi, np.asarray(emb["float"], dtype=np.float32), bd, save=False)
        if save:
            self.save()

    def remove_document(self, doc_id: int, save: bool = True):
        if int(doc_id) in self.texts:                                       # :175-178
            self.index.remove_ids(np.array([doc_id], dtype=np.int64))
            del self.texts[int(doc_id)]
        if save:
            self.save()

    def search_vectors(self, qf, k: int = 10):
        """Batched search of float32 [nq, d] queries: device (count, doc_id, score) tensors."""
        if k < 0:
            raise ValueError("k must be non-negative")
        cnt, rows, scores = self.index.search_rows(qf, k)
        ids = torch.where(rows >= 0, self.index.id_map[rows.clamp_min(0)], rows)
        return cnt, ids, scores

    def search(self, query: str, k: int = 10) -> List[Dict]:
        if self.index.ntotal == 0:                                           # :146-148
            logger.warning("No docs in index, add documents first.")
            return []
        emb = self.provider.embed([query], "search_query", ["float"])
        if not emb:
            logger.error("Query embedding generation failed.")
            return []
        D, L = self.index.search(np.asarray(emb["float"], dtype=np.float32).reshape(1, -1), k)
        results = []
        for dist, did in zip(D[0], L[0]):                                    # :158-171
            if did == -1:
                continue
            results.append({"doc_id": int(did), "score": float(dist), "doc": self.texts.get(int(did), "N/A")})
        results.sort(key=lambda x: x["score"], reverse=True)
        return results
