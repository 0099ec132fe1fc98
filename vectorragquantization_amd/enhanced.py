"""``CohereEnhancedVectorDB`` on MI355X: the reference's three-phase search as
gfx950 HIP kernels behind the same Python surface.

Reference: ``CohereEnhancedVectorDB.py`` (aitrailblazer/VectorRAGQuantization).
Same constructor (``:45-51``), ``add_documents`` (``:171-225``), ``search``
(``:227-322``: same result dict keys and order), ``remove_document``
(``:324-340``), ``save`` (``:342-347``), ``__len__`` (``:349``).  Additions for
batch / benchmark use that bypass HTTP: ``add_vectors`` and ``search_vectors``.

Storage (all HBM-resident, rows = FAISS internal indices): ubinary codes in a
``BinaryIndexIDMap2`` (u8[n,128]), int8 vectors (int8[n,1024]; the RocksDict
``"int8"`` values) and their float64 norms (computed once at add time by
``vrq_int8_row_norms``); document texts stay on the host.  ``search_vectors``
is ONE ``vrq_search3`` call for a whole query batch: Phase-I scan kernel + a
merge/rescore kernel, no host round trip between phases.
"""
from __future__ import annotations

import json
import logging
import os
from dataclasses import dataclass
from typing import Dict, List

import numpy as np
import torch

from . import _native as N
from .docstore import DocStoreError, RocksDictReader, is_rocksdict_dir
from .index import BinaryIndexIDMap2, _GrowBuffer, as_device_tensor
from .quant import int8_row_norms

logger = logging.getLogger(__name__)


@dataclass
class SearchBatch:
    """Device-tensor result of ``search_vectors`` ([nq, k], rows padded with -1)."""
    count: torch.Tensor      # i32[nq]
    doc_id: torch.Tensor     # i64[nq, k] external ids
    row: torch.Tensor        # i64[nq, k] internal rows
    hamming: torch.Tensor    # i32[nq, k]
    binary: torch.Tensor     # f64[nq, k]
    cosine: torch.Tensor     # f64[nq, k]

    def to_dicts(self, texts: dict | None = None) -> List[List[Dict]]:
        cnt = self.count.cpu().numpy()
        ids, ham = self.doc_id.cpu().numpy(), self.hamming.cpu().numpy()
        b2, c3 = self.binary.cpu().numpy(), self.cosine.cpu().numpy()
        out = []
        for q in range(cnt.shape[0]):
            res = []
            for j in range(int(cnt[q])):
                h = {"doc_id": int(ids[q, j]), "score_hamming": int(ham[q, j]),
                     "score_binary": float(b2[q, j]), "score_cosine": float(c3[q, j])}
                if texts is not None:
                    h["doc"] = texts.get(int(ids[q, j]), "N/A")
                res.append(h)
            out.append(res)
        return out


def gemm_topk(mode: str, qf: torch.Tensor, k: int, codes: torch.Tensor | None = None,
              x8: torch.Tensor | None = None, norms: torch.Tensor | None = None, row_offset: int = 0,
              flags: int = 0, workspace: torch.Tensor | None = None, lib=None):
    """Exhaustive Phase-II (``mode="binary"``) or Phase-III (``mode="int8_cosine"``) top-k of a query
    batch over EVERY row on the matrix cores (``vrq_gemm_topk``, BASELINE config 5): the scores of
    ``CohereEnhancedVectorDB.py:283-293`` / ``:302-318`` ordered like the reference's stable
    ``sorted(..., reverse=True)`` over rows in index order.  Returns (count i32[nq], rows i64[nq, k],
    scores f64[nq, k]) device tensors.  ``flags``: VRQ_GEMM_STAGE_* / VRQ_GEMM_NO_FALLBACK; ``lib``:
    another build of the library (the probe build, for sweeps), default libvrq.so."""
    m = {"binary": N.VRQ_GEMM_BINARY, "int8_cosine": N.VRQ_GEMM_INT8_COSINE}[mode]
    src = codes if m == N.VRQ_GEMM_BINARY else x8
    dev = qf.device
    nq, n = qf.shape[0], src.shape[0]
    cnt = torch.full((nq,), -2, dtype=torch.int32, device=dev)  # -2: never written
    rows = torch.full((nq, k), -2, dtype=torch.int64, device=dev)
    scores = torch.empty((nq, k), dtype=torch.float64, device=dev)
    lib = lib or N.load()
    need = lib.vrq_gemm_topk_workspace_size(m, n, qf.shape[1], nq, k)
    if need == 0:
        raise N.VrqNativeError(f"vrq_gemm_topk: unsupported shape n={n} dim={qf.shape[1]} nq={nq} k={k}")
    if workspace is None or workspace.numel() < need:
        workspace = torch.empty((need,), dtype=torch.uint8, device=dev)
    N.check(lib.vrq_gemm_topk(m, N.ptr(codes), N.ptr(x8), N.ptr(norms), n, qf.shape[1], row_offset, N.ptr(qf), nq,
                              k, flags, N.ptr(cnt), N.ptr(rows), N.ptr(scores), N.ptr(workspace),
                              workspace.numel(), N.stream_handle(dev)), "vrq_gemm_topk")
    stages = flags & (N.VRQ_GEMM_STAGE_SAMPLE | N.VRQ_GEMM_STAGE_MAIN | N.VRQ_GEMM_STAGE_FINISH)
    if (not stages or stages & N.VRQ_GEMM_STAGE_FINISH) and bool((cnt < 0).any()):
        # only with VRQ_GEMM_NO_FALLBACK in flags: the library left queries it could not serve on the
        # matrix path unwritten (count -1) instead of running the exact scan
        raise N.VrqNativeError("vrq_gemm_topk: queries needed the exact fallback, which VRQ_GEMM_NO_FALLBACK disabled")
    return cnt, rows, scores


def search3(codes: torch.Tensor, x8: torch.Tensor, norms: torch.Tensor, qf: torch.Tensor, qb: torch.Tensor,
            k: int, K: int, K3: int, flags: int = 0, row_offset: int = 0, rescore_row: torch.Tensor | None = None,
            workspace: torch.Tensor | None = None):
    """Thin wrapper of ``vrq_search3``; returns (count, rows, dist, s2, s3) device tensors."""
    dev = qf.device
    nq = qf.shape[0]
    n = codes.shape[0]
    dim = qf.shape[1]
    kout = K if flags & (N.VRQ_SEARCH_SHARD | N.VRQ_SEARCH_PHASE1_ONLY) else k
    cnt = torch.empty((nq,), dtype=torch.int32, device=dev)
    rows = torch.empty((nq, kout), dtype=torch.int64, device=dev)
    dist = torch.empty((nq, kout), dtype=torch.int32, device=dev)
    s2 = torch.empty((nq, kout), dtype=torch.float64, device=dev)
    s3 = torch.empty((nq, kout), dtype=torch.float64, device=dev)
    if not flags & N.VRQ_SEARCH_PHASE1_ONLY and n and (x8.shape[0] != n or norms.shape[0] != n):
        # the ABI indexes x8 / norms by code row and cannot see their lengths
        raise N.VrqNativeError(f"vrq_search3: {n} code rows but {x8.shape[0]} int8 rows and {norms.shape[0]} norms")
    if rescore_row is not None and rescore_row.shape[0] != n:
        raise N.VrqNativeError(f"vrq_search3: rescore_row has {rescore_row.shape[0]} entries for {n} rows")
    lib = N.load()
    need = lib.vrq_search3_workspace_size(n, dim, nq, K) if n and nq and K else 0
    if workspace is None or workspace.numel() < need:
        workspace = torch.empty((max(need, 8),), dtype=torch.uint8, device=dev)
    rc = lib.vrq_search3(N.ptr(codes) if n else 0, N.ptr(x8) if n else 0, N.ptr(norms) if n else 0,
                         N.ptr(rescore_row), n, dim, row_offset, N.ptr(qf), N.ptr(qb), nq, k, K, K3, flags,
                         N.ptr(cnt), N.ptr(rows), N.ptr(dist), N.ptr(s2), N.ptr(s3), N.ptr(workspace),
                         workspace.numel(), N.stream_handle(dev))
    N.check(rc, "vrq_search3")
    return cnt, rows, dist, s2, s3


class CohereEnhancedVectorDB:
    """Drop-in for the reference class (``CohereEnhancedVectorDB.py:30``)."""

    def __init__(self, folder: str, model: str = "embed-english-v3.0", embedding_dim: int = 1024,
                 index_type=None, index_args: List = None, rdict_options=None, *, provider=None,
                 device=None):
        if index_args is None:
            index_args = [embedding_dim]
        if provider is None:   # the reference reads COHERE_EMBED_ENDPOINT / _KEY and raises if unset (:67-75)
            from .embed import CohereHTTPProvider
            provider = CohereHTTPProvider(model=model)
        self.provider = provider
        self.embedding_dim = embedding_dim
        self.model = model
        self.folder = folder
        self._setup_config(folder, model, embedding_dim)
        path = os.path.join(folder, "index.bin")
        if os.path.exists(path):
            self.index = BinaryIndexIDMap2.read(path, device)
            logger.info("Existing binary index loaded.")
        else:
            self.index = BinaryIndexIDMap2(index_args[0], device)
        self.device = self.index.device
        self._x8 = _GrowBuffer((embedding_dim,), torch.int8, self.device)
        self._norms = _GrowBuffer((), torch.float64, self.device)
        self.texts: Dict[int, str] = {}
        self._load_docs()
        self._ws = None

    # -- config / persistence (reference :90-115, :342-347) -----------------------
    def _setup_config(self, folder: str, model: str, embedding_dim: int):
        config_path = os.path.join(folder, "config.json")
        if not os.path.exists(config_path):
            if os.path.exists(folder) and os.listdir(folder):
                raise Exception(f"Folder {folder} contains files, but no config.json. "
                                "To create a new database, the folder must be empty.")
            os.makedirs(folder, exist_ok=True)
            config = {"version": "1.0", "model": model, "embedding_dim": embedding_dim}
            with open(config_path, "w") as f:
                json.dump(config, f)
        else:
            with open(config_path) as f:
                config = json.load(f)
            if config.get("model") != model or config.get("embedding_dim") != embedding_dim:
                logger.warning("Config model or embedding_dim mismatch. Overwriting config.")
                config = {"version": "1.0", "model": model, "embedding_dim": embedding_dim}
                with open(config_path, "w") as f:
                    json.dump(config, f)
        self.config = config

    def _docs_path(self):
        """This build's document store (int8 rows + texts).  It lives beside the reference's RocksDict
        directory ``docs/`` so that saving never writes into a RocksDB database."""
        return os.path.join(self.folder, "vrq_docs")

    def _load_docs(self):
        """Rows of the device int8 store in index-row order, from (in this order of preference) this
        build's ``vrq_docs/`` when it matches ``index.bin``, the reference's RocksDict ``docs/``
        (``CohereEnhancedVectorDB.py:88``; read by ``docstore.RocksDictReader``, no rocksdict needed), or
        a round-1 ``docs/int8.npy``.  An index without a matching store is refused: Phases II/III index
        the int8 rows and norms by index row, so a short store would be read out of bounds."""
        n = self.index.ntotal
        own = self._docs_path()
        legacy = os.path.join(self.folder, "docs")
        for p in (own, legacy):
            f = os.path.join(p, "int8.npy")
            if os.path.exists(f):
                x8 = np.load(f)
                if x8.shape[0] == n:
                    with open(os.path.join(p, "texts.json")) as fh:
                        self.texts = {int(a): b for a, b in json.load(fh).items()}
                    self._set_rows(x8)
                    return
        if is_rocksdict_dir(legacy):
            self._load_rocksdict(legacy)
            return
        if n:
            raise DocStoreError(f"{self.folder}: index.bin holds {n} rows but there is no document store "
                                "(docs/ RocksDict or vrq_docs/) to read their int8 vectors from")

    def _load_rocksdict(self, path):
        db = RocksDictReader(path)
        ids = self.index.id_map.cpu().numpy() if isinstance(self.index.id_map, torch.Tensor) else \
            np.asarray(self.index.id_map)
        recs = {}
        for key, val in db.items():
            try:
                did = int(key)
            except (TypeError, ValueError):
                continue
            recs[did] = val
            self.texts[did] = val.get("doc", "N/A") if isinstance(val, dict) else "N/A"
        x8 = np.zeros((ids.shape[0], self.embedding_dim), np.int8)
        missing = []
        for r, did in enumerate(ids.tolist()):
            v = recs.get(int(did))
            if not isinstance(v, dict) or "int8" not in v:
                missing.append(int(did))
                continue
            x8[r] = np.asarray(v["int8"], dtype=np.int8).reshape(self.embedding_dim)
        if missing:
            # the reference skips such hits in Phase III (:303-305); this build keeps one int8 row per
            # index row and refuses the inconsistent folder instead
            raise DocStoreError(f"{path}: no int8 record for index ids {missing[:8]}"
                                f"{' ...' if len(missing) > 8 else ''}")
        self._set_rows(x8)
        logger.info("Loaded %d documents from the RocksDict store %s.", len(recs), path)

    def _set_rows(self, x8: np.ndarray):
        t = torch.from_numpy(np.ascontiguousarray(x8)).to(self.device)
        self._x8 = _GrowBuffer((self.embedding_dim,), torch.int8, self.device)
        self._norms = _GrowBuffer((), torch.float64, self.device)
        if t.shape[0]:
            self._x8.append(t)
            self._norms.append(int8_row_norms(t))

    def save(self):
        """index.bin in FAISS's IBM2 format (:346) + this build's doc store (int8 rows, texts) in vrq_docs/."""
        self.index.write(os.path.join(self.folder, "index.bin"))
        p = self._docs_path()
        os.makedirs(p, exist_ok=True)
        np.save(os.path.join(p, "int8.npy"), self._x8.view().cpu().numpy())
        with open(os.path.join(p, "texts.json"), "w") as f:
            json.dump({str(a): b for a, b in self.texts.items()}, f)
        logger.info("Binary index saved.")

    def __len__(self):
        return self.index.ntotal

    # -- document management ---------------------------------------------------------
    def __contains__(self, doc_id) -> bool:
        return int(doc_id) in self.texts

    def add_vectors(self, doc_ids, int8, ubinary, docs=None, save: bool = False) -> None:
        """Append pre-computed (int8, ubinary) embeddings -- ``:217-221`` without HTTP."""
        ids = np.asarray(doc_ids.cpu() if isinstance(doc_ids, torch.Tensor) else doc_ids, dtype=np.int64).reshape(-1)
        x8 = as_device_tensor(int8, torch.int8, self.device).reshape(ids.shape[0], self.embedding_dim)
        ub = as_device_tensor(ubinary, torch.uint8, self.device).reshape(ids.shape[0], self.embedding_dim // 8)
        self.index.add_with_ids(ub, ids)
        self._x8.append(x8)
        self._norms.append(int8_row_norms(x8))
        if docs is None:
            docs = [""] * ids.shape[0]
        for i, d in zip(ids.tolist(), docs):
            self.texts[i] = d
        if save:
            self.save()

    def add_documents(self, doc_ids: List[int], docs: List[str], batch_size: int = 64, save: bool = True):
        if len(doc_ids) != len(docs):
            raise ValueError("doc_ids and docs must have the same length.")
        for doc_id in doc_ids:                                              # :190-192
            if int(doc_id) in self.texts:
                self.remove_document(doc_id, save=False)
        for start in range(0, len(docs), batch_size):                      # :195-222
            bi, bd = doc_ids[start:start + batch_size], docs[start:start + batch_size]
            emb = self.provider.embed(bd, "search_document", ["int8", "ubinary"])
            if not emb:
                logger.error("Failed to retrieve embeddings for a batch.")
                continue
            try:
                x8, ub = emb["int8"], emb["ubinary"]
                if not isinstance(x8, torch.Tensor):
                    x8 = np.array(x8, dtype=np.int8)
                    ub = np.array(ub, dtype=np.uint8)
            except Exception as e:
                logger.error("Error processing embeddings: %s", str(e))
                continue
            self.add_vectors(bi, x8, ub, bd, save=False)
        if save:
            self.save()

    def remove_document(self, doc_id: int, save: bool = True):
        if int(doc_id) in self.texts:                                       # :333-336
            keep = self.index.id_map != int(doc_id)
            self.index._compact(keep)
            self._x8.keep(keep)
            self._norms.keep(keep)
            del self.texts[int(doc_id)]
            logger.info(f"Document {doc_id} removed.")
        else:
            logger.warning(f"Document {doc_id} not found in the database.")
        if save:
            self.save()

    # -- search ------------------------------------------------------------------------
    def search_vectors(self, qf, qb, k: int = 10, binary_oversample: int = 10,
                       int8_oversample: int = 3) -> SearchBatch:
        """Batched three-phase search of float32 [nq, d] / ubinary [nq, d/8] query embeddings."""
        qf = as_device_tensor(qf, torch.float32, self.device).reshape(-1, self.embedding_dim)
        qb = as_device_tensor(qb, torch.uint8, self.device).reshape(-1, self.embedding_dim // 8)
        n = self.index.ntotal
        if k < 0 or binary_oversample < 0 or int8_oversample < 0:
            raise ValueError("k and oversample factors must be non-negative")
        K = min(k * binary_oversample, n)                                   # :267
        K3 = k * int8_oversample                                            # :297
        if self._ws is None or self._ws.device != self.device:
            self._ws = torch.empty((8,), dtype=torch.uint8, device=self.device)
        lib = N.load()
        need = lib.vrq_search3_workspace_size(n, self.embedding_dim, qf.shape[0], K) if n and K else 0
        if self._ws.numel() < need:
            self._ws = torch.empty((need,), dtype=torch.uint8, device=self.device)
        with torch.cuda.device(self.device):
            cnt, rows, dist, s2, s3 = search3(self.index.codes, self._x8.view(), self._norms.view(), qf, qb,
                                              k, K, K3, 0, 0, self.index.rescore_rows(), self._ws)
        ids = torch.where(rows >= 0, self.index.id_map[rows.clamp_min(0)] if n else rows, rows)
        return SearchBatch(cnt, ids, rows, dist, s2, s3)

    def search(self, query: str, k: int = 10, binary_oversample: int = 10, int8_oversample: int = 3) -> List[Dict]:
        if self.index.ntotal == 0:                                           # :247-249
            logger.error("No documents indexed. Please add documents before searching.")
            return []
        emb = self.provider.embed([query], "search_query", ["float", "ubinary"])
        if not emb:
            logger.error("Query embedding generation failed.")
            return []
        try:
            qf, qb = emb["float"], emb["ubinary"]
        except Exception as e:
            logger.error("Error processing query embeddings: %s", str(e))
            return []
        res = self.search_vectors(qf, qb, k, binary_oversample, int8_oversample)
        return res.to_dicts(self.texts)[0]


def find_closest_document(db: CohereEnhancedVectorDB, query: str) -> Dict:
    """``CohereEnhancedVectorDB.py:355-360``."""
    results = db.search(query, k=1)
    return results[0] if results else {}


def print_top_results(db: CohereEnhancedVectorDB, query: str, k: int = 10):
    """``CohereEnhancedVectorDB.py:363-375``."""
    results = db.search(query, k=k)
    if results:
        print(f"Top {k} Results:")
        for res in results:
            print(f"Doc ID: {res['doc_id']}, Cosine Score: {res['score_cosine']:.4f}")
            print(f"Document: {res['doc']}")
            print("-" * 40)
    else:
        print("No matching documents found.")
