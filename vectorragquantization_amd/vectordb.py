"""The ``VectorDBInt{4,8,16}{,Global}`` classes on MI355X.

Drop-ins for the reference's six scalar-quantised stores.  Constructor, ``add_documents``,
``search(query, k, binary_oversample, compare_float32)``, ``remove_document``, ``save`` and
``__len__`` keep the reference's names, argument meaning, result dicts and error behaviour:

=====================  ===========================  ==========  ====================  ========
class                  reference                     encode      stored row            scale
=====================  ===========================  ==========  ====================  ========
VectorDBInt8Global     ``VectorDBInt8Global.py``     ``int8g``   ``emb_int8``          global
VectorDBInt16Global    ``VectorDBInt16Global.py``    ``int16g``  ``emb_int16``         global
VectorDBInt4Global     ``VectorDBInt4Global.py``     ``int4g``   ``emb_int4``          global
VectorDBInt8           ``VectorDBInt8.py``           ``int8``    ``emb_int8`` + min_max  per row
VectorDBInt4           ``VectorDBInt4.py``           ``int4``    ``emb_int4`` + min_max  per row
VectorDBInt16          ``VectorDBInt16.py``          ``bin16``   (Hamming only)        --
=====================  ===========================  ==========  ====================  ========

The search of every class is the reference's two-stage loop (e.g. ``VectorDBInt8Global.py:205-252``):
1. Phase I: FAISS ``IndexBinaryFlat`` top-``min(k * binary_oversample, ntotal)`` over the ubinary
   codes -- ``vrq_hamming_topk`` (the gfx950 scan kernels shared with CohereEnhancedVectorDB);
2. Phase II: ``float(np.dot(query_float, doc_emb))`` per candidate, ``doc_emb`` the dequantised row
   (``_dequantize_*``, bit-exact) or, with ``compare_float32=True``, the float32 row kept from
   ``add_documents`` (``float_embeddings``) -- ``vrq_rescore_dequant`` on the device;
3. Python's stable ``sort(key=score, reverse=True)`` and the first k.
``VectorDBInt16.search`` (``VectorDBInt16.py:221-263``) stops after Phase I and ranks by Hamming
distance (``score`` = the distance).

Storage, all HBM-resident and indexed by index row: codes (``BinaryIndexIDMap2``), the quantised
rows (int8 / int16 / packed int4), per-row (min, max) for the local quantisers (f64 holding the
reference's float32 or Python-float values), and the float32 rows for ``compare_float32``.  Texts
stay on the host.  ``add_documents`` quantises a whole batch in ONE ``vrq_encode`` launch.

Folders: ``index.bin`` is FAISS's IBM2 file (read / written byte-compatibly); documents come from
this build's ``vrq_docs/`` or from the reference's RocksDict ``docs/`` (``docstore.RocksDictReader``,
no rocksdict needed), so ``VectorDBInt8Global("<reference db_int8_global>")`` opens with its 1000
documents.  Like the reference, float32 rows live only in memory (``float_embeddings``): after
reopening a folder ``search(..., compare_float32=True)`` raises ``KeyError`` for a hit without one,
as ``self.float_embeddings[doc_id_str]`` does.  Deliberate difference: ``remove_document`` of such
a document does not raise (the reference's ``del self.float_embeddings[...]`` would).
"""
from __future__ import annotations

import json
import logging
import os
from typing import Dict, List

import numpy as np
import torch

from . import _native as N
from . import quant as Q
from .docstore import DocStoreError, RocksDictReader, is_rocksdict_dir
from .index import BinaryIndexIDMap2, _GrowBuffer, as_device_tensor, torch_to_np

logger = logging.getLogger(__name__)

DEFAULT_EMBED_URL = "http://localhost:11434/api/embed"


class _QuantizedVectorDB:
    MODE = "int8g"          # vrq_encode / vrq_dequantize mode
    QKEY = "emb_int8"       # RocksDict value key of the quantised row
    QDTYPE = torch.int8
    LOCAL = False           # per-row (min, max)
    GLOBAL = False          # config.json carries global_limit
    HAMMING_ONLY = False    # VectorDBInt16, CohereVectorDBInt8
    VEC_DTYPE = torch.float32   # embeddings as the provider returns them
    EMPTY_MSG = "If you want to create a new database, the folder must be empty."

    def __init__(self, folder: str, model: str, embedding_dim: int, global_limit, rdict_options, embed_url: str,
                 provider, device):
        self.embedding_dim = embedding_dim
        self.model = model
        self.embed_url = embed_url
        self.rdict_options = rdict_options   # accepted for signature compatibility (no RocksDB here)
        if self.GLOBAL:
            self.global_limit = float(global_limit)
        self.folder = folder
        self._setup_config(folder, model, embedding_dim)
        if provider is None:   # the reference posts self.config["model"] to embed_url
            from .embed import Int16HTTPProvider, OllamaHTTPProvider
            cls = Int16HTTPProvider if self.HAMMING_ONLY else OllamaHTTPProvider
            provider = cls(embed_url, self.config.get("model", model) if not self.HAMMING_ONLY else model,
                           embedding_dim)
        self.provider = provider
        path = os.path.join(folder, "index.bin")
        if os.path.exists(path):
            self.index = BinaryIndexIDMap2.read(path, device)
            logger.info("Existing FAISS index loaded.")
        else:
            self.index = BinaryIndexIDMap2(embedding_dim, device)
            logger.info(f"New FAISS index created with embedding dimension {embedding_dim}.")
        self.device = self.index.device
        self._reset_rows()
        self.texts: Dict[int, str] = {}
        self._float_ids = set()     # doc ids whose float32 row is held (the reference's float_embeddings keys)
        self._load_docs()

    # -- layout ---------------------------------------------------------------------
    def _qshape(self):
        return ((self.embedding_dim + 1) // 2,) if self.MODE in ("int4g", "int4") else (self.embedding_dim,)

    def _reset_rows(self):
        self._q = _GrowBuffer(self._qshape(), self.QDTYPE, self.device)
        self._mm = _GrowBuffer((2,), torch.float64, self.device)
        self._f = _GrowBuffer((self.embedding_dim,), torch.float32, self.device)

    @property
    def limit(self) -> float:
        """The dequantisation limit the reference's search passes (``self.global_limit``; for
        VectorDBInt4Global ``self.config.get("global_limit", 0.18)``, ``VectorDBInt4Global.py:263``)."""
        return self.global_limit if self.GLOBAL else 0.0

    @property
    def float_embeddings(self) -> Dict[str, np.ndarray]:
        """The reference's ``float_embeddings`` dict (``str(doc_id) -> float32 row``), materialised
        from the device rows (for inspection; the search reads the device rows directly)."""
        ids = self.index.id_map.cpu().numpy()
        out = {}
        if self._f.n:
            F = self._f.view().cpu().numpy()
            for r, e in enumerate(ids.tolist()):
                if e in self._float_ids:
                    out[str(e)] = F[r]
        return out

    # -- config / persistence ------------------------------------------------------------
    def _setup_config(self, folder: str, model: str, embedding_dim: int):
        config_path = os.path.join(folder, "config.json")
        if not os.path.exists(config_path):
            if os.path.exists(folder) and len(os.listdir(folder)) > 0:
                raise Exception(f"Folder {folder} contains files, but no config.json. {self.EMPTY_MSG}")
            os.makedirs(folder, exist_ok=True)
            config = {"version": "1.0", "model": model, "embedding_dim": embedding_dim}
            if self.GLOBAL:
                config["global_limit"] = self.global_limit
            with open(config_path, "w") as f:
                json.dump(config, f)
        with open(config_path) as f:
            self.config = json.load(f)
        if self.GLOBAL:   # the config's limit wins (e.g. VectorDBInt8Global.py:72-73)
            self.global_limit = float(self.config.get("global_limit", self.global_limit))

    def _docs_path(self):
        return os.path.join(self.folder, "vrq_docs")

    def _load_docs(self):
        n = self.index.ntotal
        own = self._docs_path()
        tj = os.path.join(own, "texts.json")
        if os.path.exists(tj):
            q = np.load(os.path.join(own, "q.npy")) if not self.HAMMING_ONLY else None
            if self.HAMMING_ONLY or q.shape[0] == n:
                with open(tj) as fh:
                    self.texts = {int(a): b for a, b in json.load(fh).items()}
                mm = np.load(os.path.join(own, "minmax.npy")) if self.LOCAL else None
                self._set_rows(q, mm)
                return
        legacy = os.path.join(self.folder, "docs")
        if is_rocksdict_dir(legacy):
            self._load_rocksdict(legacy)
            return
        if n:
            raise DocStoreError(f"{self.folder}: index.bin holds {n} rows but there is no document store "
                                "(docs/ RocksDict or vrq_docs/) to read their vectors from")

    def _load_rocksdict(self, path):
        db = RocksDictReader(path)
        recs = {}
        for key, val in db.items():
            try:
                did = int(key)
            except (TypeError, ValueError):
                continue
            recs[did] = val
            self.texts[did] = val.get("doc", "N/A") if isinstance(val, dict) else "N/A"
        if self.HAMMING_ONLY:
            logger.info("Loaded %d documents from the RocksDict store %s.", len(recs), path)
            return
        ids = self.index.id_map.cpu().numpy()
        q = np.zeros((ids.shape[0], *self._qshape()), dtype=torch_to_np(self.QDTYPE))
        mm = np.zeros((ids.shape[0], 2), np.float64)
        missing = []
        for r, did in enumerate(ids.tolist()):
            v = recs.get(int(did))
            if not isinstance(v, dict) or self.QKEY not in v or (self.LOCAL and "min_max" not in v):
                missing.append(int(did))
                continue
            q[r] = np.asarray(v[self.QKEY]).astype(q.dtype).reshape(q.shape[1:])
            if self.LOCAL:
                mm[r] = [float(v["min_max"][0]), float(v["min_max"][1])]
        if missing:
            # the reference skips such hits (`if doc_data is None: continue`); this build keeps one
            # stored row per index row and refuses the inconsistent folder instead
            raise DocStoreError(f"{path}: no {self.QKEY} record for index ids {missing[:8]}"
                                f"{' ...' if len(missing) > 8 else ''}")
        self._set_rows(q, mm if self.LOCAL else None)
        logger.info("Loaded %d documents from the RocksDict store %s.", len(recs), path)

    def _set_rows(self, q, mm):
        self._reset_rows()
        if self.HAMMING_ONLY or q is None or not q.shape[0]:
            return
        self._q.append(torch.from_numpy(np.ascontiguousarray(q)).to(self.device))
        if self.LOCAL:
            self._mm.append(torch.from_numpy(np.ascontiguousarray(mm, np.float64)).to(self.device))
        self._f.append(torch.zeros((q.shape[0], self.embedding_dim), dtype=torch.float32, device=self.device))

    def save(self):
        """index.bin in FAISS's IBM2 format + this build's doc store (quantised rows, min/max, texts)
        in vrq_docs/ (the reference's RocksDict persists on each write; float rows are not persisted,
        as in the reference)."""
        self.index.write(os.path.join(self.folder, "index.bin"))
        p = self._docs_path()
        os.makedirs(p, exist_ok=True)
        if not self.HAMMING_ONLY:
            np.save(os.path.join(p, "q.npy"), self._q.view().cpu().numpy())
            if self.LOCAL:
                np.save(os.path.join(p, "minmax.npy"), self._mm.view().cpu().numpy())
        with open(os.path.join(p, "texts.json"), "w") as f:
            json.dump({str(a): b for a, b in self.texts.items()}, f)
        logger.info("FAISS index saved to disk.")

    def __len__(self):
        return self.index.ntotal

    def __contains__(self, doc_id) -> bool:
        return int(doc_id) in self.texts

    # -- documents ---------------------------------------------------------------------
    def _embed(self, texts, input_type: str = "search_document") -> dict:
        return self.provider.embed_int16(texts) if self.HAMMING_ONLY else self.provider.embed_floats(texts)

    def _codes(self, X):
        """ubinary codes (+ quantised rows) of a device batch in one ``vrq_encode`` launch; the
        integer classes threshold at the float64 mean, exact for int8 as for int16 rows."""
        if self.HAMMING_ONLY and X.dtype != torch.int16:
            X = X.to(torch.int16)
        return Q.encode(self.MODE, X, self.limit if self.GLOBAL else 1.0, self.device)

    def add_vectors(self, doc_ids, X, docs=None, save: bool = False) -> None:
        """Append embeddings (f32[m, d]; i16[m, d] for VectorDBInt16) without HTTP: one ``vrq_encode``
        launch computes the ubinary codes and the quantised rows of the whole batch."""
        ids = np.asarray(doc_ids.cpu() if isinstance(doc_ids, torch.Tensor) else doc_ids, dtype=np.int64).reshape(-1)
        X = as_device_tensor(X, self.VEC_DTYPE, self.device).reshape(ids.shape[0], self.embedding_dim)
        e = self._codes(X)
        self.index.add_with_ids(e["codes"], ids)
        if not self.HAMMING_ONLY:
            self._q.append(e["q"])
            if self.LOCAL:
                self._mm.append(e["minmax"])
            self._f.append(X)
            self._float_ids.update(ids.tolist())
        if docs is None:
            docs = [""] * ids.shape[0]
        for i, d in zip(ids.tolist(), docs):
            self.texts[i] = d
        if save:
            self.save()

    def add_documents(self, doc_ids: List[int], docs: List[str], batch_size: int = 64, save: bool = True):
        if len(doc_ids) != len(docs):
            raise ValueError("doc_ids and docs must have the same length.")
        for doc_id in doc_ids:                          # remove duplicates (e.g. VectorDBInt8Global.py:170-173)
            if int(doc_id) in self.texts:
                self.remove_document(doc_id, save=False)
        for start in range(0, len(docs), batch_size):
            bi, bd = doc_ids[start:start + batch_size], docs[start:start + batch_size]
            emb = self._embed(bd)
            if not emb:
                logger.error(f"Embedding generation failed for batch: {bd}")
                continue
            if self.HAMMING_ONLY:   # VectorDBInt16.py:191-206: docs without an embedding are skipped
                keep = [j for j, t in enumerate(bd) if t in emb]
                if not keep:
                    continue
                self.add_vectors([bi[j] for j in keep], np.stack([emb[bd[j]] for j in keep]),
                                 [bd[j] for j in keep])
                continue
            # `[embeddings[doc]['ubinary'] for doc in batch_docs]` raises KeyError for a text whose
            # embedding failed (VectorDBInt8Global.py:186-189); so does this
            self.add_vectors(bi, np.stack([emb[t] for t in bd]), bd)
        if save:
            self.save()

    def remove_document(self, doc_id: int, save: bool = True):
        if int(doc_id) in self.texts:
            keep = self.index.id_map != int(doc_id)
            self.index._compact(keep)
            if not self.HAMMING_ONLY:
                self._q.keep(keep)
                if self.LOCAL:
                    self._mm.keep(keep)
                self._f.keep(keep)
            del self.texts[int(doc_id)]
            self._float_ids.discard(int(doc_id))
            logger.info(f"Document {doc_id} removed.")
        else:
            logger.warning(f"Document {doc_id} not found in the database.")
        if save:
            self.save()

    # -- search ------------------------------------------------------------------------
    def search_vectors(self, query, k: int = 10, binary_oversample: int = 10, compare_float32: bool = False):
        """Batched search of query embeddings (f32[nq, d]; i16[nq, d] for VectorDBInt16) on the device.
        Returns (doc_id i64[nq, kk], row i64[nq, kk], hamming i32[nq, kk], score f64[nq, kk]) with
        kk = min(k, K); rows past the candidates are -1."""
        n = self.index.ntotal
        if k < 0 or binary_oversample < 0:
            raise ValueError("k and binary_oversample must be non-negative")
        qv = as_device_tensor(query, self.VEC_DTYPE, self.device).reshape(-1, self.embedding_dim)
        qb = self._codes(qv)["codes"]
        with torch.cuda.device(self.device):
            if self.HAMMING_ONLY:
                rows, ham, sc = Q.vectordb_search("bin16", self.index.codes, None, None, qb, k, binary_oversample)
            else:
                mode = "f32" if compare_float32 else self.MODE
                src = self._f.view() if compare_float32 else self._q.view()
                rr = self.index.rescore_rows()
                rows, ham, sc = Q.vectordb_search(mode, self.index.codes, src, qv, qb, k, binary_oversample,
                                                  self._mm.view() if self.LOCAL and not compare_float32 else None,
                                                  self.limit, rr)
                if compare_float32:
                    self._check_float_rows(rows)
        ids = torch.where(rows >= 0, self.index.id_map[rows.clamp_min(0)], rows) if n else rows
        return ids, rows, ham, sc

    def _check_float_rows(self, rows):
        """``self.float_embeddings[doc_id_str]`` raises KeyError for a candidate without a float row
        (a document loaded from disk); the reference raises on the first such Phase-I hit."""
        if len(self._float_ids) == len(self.texts):
            return
        ids = self.index.id_map[rows[rows >= 0]].cpu().numpy().tolist()
        for e in ids:
            if e not in self._float_ids:
                raise KeyError(str(e))

    def search(self, query: str, k: int = 10, binary_oversample: int = 10, compare_float32: bool = False) -> List[Dict]:
        if self.index.ntotal == 0:
            logger.error("No documents indexed. Please add documents before searching.")
            return []
        emb = self._embed([query], "search_query")
        if not emb or query not in emb:
            logger.error("Query embedding generation failed. Returning empty results.")
            return []
        if self.HAMMING_ONLY:
            ids, _, ham, _ = self.search_vectors(emb[query], k, binary_oversample)
            ids, ham = ids[0].cpu().numpy(), ham[0].cpu().numpy()
            return [{"doc_id": int(i), "score": int(h), "doc": self.texts.get(int(i), "N/A")}
                    for i, h in zip(ids, ham) if i != -1]
        ids, _, _, sc = self.search_vectors(emb[query], k, binary_oversample, compare_float32)
        ids, sc = ids[0].cpu().numpy(), sc[0].cpu().numpy()
        return [{"doc_id": int(i), "score": float(s), "doc": self.texts.get(int(i), "N/A")}
                for i, s in zip(ids, sc) if i != -1]


class VectorDBInt8Global(_QuantizedVectorDB, Q.VectorDBInt8Global):
    """``VectorDBInt8Global.py:16``: int8 with one global clipping limit (±global_limit -> ±127)."""
    MODE, QKEY, QDTYPE, GLOBAL = "int8g", "emb_int8", torch.int8, True

    def __init__(self, folder: str, model: str = "snowflake-arctic-embed2", embedding_dim: int = 1024,
                 global_limit: float = 0.3, rdict_options=None, embed_url: str = DEFAULT_EMBED_URL, *,
                 provider=None, device=None):
        super().__init__(folder, model, embedding_dim, global_limit, rdict_options, embed_url, provider, device)


class VectorDBInt16Global(_QuantizedVectorDB, Q.VectorDBInt16Global):
    """``VectorDBInt16Global.py:17``: int16 with one global clipping limit (±global_limit -> ±32767)."""
    MODE, QKEY, QDTYPE, GLOBAL = "int16g", "emb_int16", torch.int16, True

    def __init__(self, folder: str, model: str = "snowflake-arctic-embed2", embedding_dim: int = 1024,
                 global_limit: float = 1.0, rdict_options=None, embed_url: str = DEFAULT_EMBED_URL, *,
                 provider=None, device=None):
        super().__init__(folder, model, embedding_dim, global_limit, rdict_options, embed_url, provider, device)


class VectorDBInt4Global(_QuantizedVectorDB, Q.VectorDBInt4Global):
    """``VectorDBInt4Global.py:16``: nibble-packed int4; the quantiser ignores the limit (reference
    bug, reproduced) while the dequantiser uses it."""
    MODE, QKEY, QDTYPE, GLOBAL = "int4g", "emb_int4", torch.int8, True

    def __init__(self, folder: str, model: str = "snowflake-arctic-embed2", embedding_dim: int = 1024,
                 global_limit: float = 0.18, rdict_options=None, embed_url: str = DEFAULT_EMBED_URL, *,
                 provider=None, device=None):
        super().__init__(folder, model, embedding_dim, global_limit, rdict_options, embed_url, provider, device)

    @property
    def limit(self) -> float:
        return float(self.config.get("global_limit", 0.18))


class VectorDBInt8(_QuantizedVectorDB, Q.VectorDBInt8):
    """``VectorDBInt8.py:15``: per-document symmetric int8 (truncating) with stored (min, max)."""
    MODE, QKEY, QDTYPE, LOCAL = "int8", "emb_int8", torch.int8, True

    def __init__(self, folder: str, model: str = "snowflake-arctic-embed2", embedding_dim: int = 1024,
                 rdict_options=None, embed_url: str = DEFAULT_EMBED_URL, *, provider=None, device=None):
        super().__init__(folder, model, embedding_dim, None, rdict_options, embed_url, provider, device)


class VectorDBInt4(_QuantizedVectorDB, Q.VectorDBInt4):
    """``VectorDBInt4.py:15``: per-document nibble-packed int4 with stored (min, max)."""
    MODE, QKEY, QDTYPE, LOCAL = "int4", "emb_int4", torch.int8, True

    def __init__(self, folder: str, model: str = "snowflake-arctic-embed2", embedding_dim: int = 1024,
                 rdict_options=None, embed_url: str = DEFAULT_EMBED_URL, *, provider=None, device=None):
        super().__init__(folder, model, embedding_dim, None, rdict_options, embed_url, provider, device)


class VectorDBInt16(_QuantizedVectorDB, Q.VectorDBInt16):
    """``VectorDBInt16.py:16``: int16 embeddings from the service thresholded to 1 bit/dimension;
    Hamming-only search."""
    MODE, QKEY, QDTYPE, HAMMING_ONLY, VEC_DTYPE = "bin16", "int16", torch.int16, True, torch.int16
    EMPTY_MSG = "To create a new database, the folder must be empty."

    def __init__(self, folder: str, model: str = "snowflake-arctic-embed2", embedding_dim: int = 1024,
                 rdict_options=None, embed_url: str = DEFAULT_EMBED_URL, *, provider=None, device=None):
        super().__init__(folder, model, embedding_dim, None, rdict_options, embed_url, provider, device)

    def _setup_config(self, folder: str, model: str, embedding_dim: int):
        super()._setup_config(folder, model, embedding_dim)
        if self.config.get("model") != model or self.config.get("embedding_dim") != embedding_dim:   # :71-76
            logger.warning("Config model/dim differs from constructor arguments. "
                           f"config={self.config}, constructor=(model={model}, dim={embedding_dim})")


class CohereVectorDBInt8(_QuantizedVectorDB):
    """``CohereVectorDBInt8.py:11``: Cohere int8 embeddings only, ``packbits(int8 > mean)`` codes
    (``:130-135``; the float64 mean of int8 rows is exact, so the ``bin16`` encode of the rows widened
    to int16 is bit-identical), Hamming-only ``search`` (``:192-235``: ``score`` = the distance) and
    ``search_rerank_cohere`` (``:237-339``): the Phase-I candidates of the gfx950 scan handed to the
    Cohere ``/v2/rerank`` service.  ``provider`` replaces the ``COHERE_EMBED_*`` HTTP client
    (``CohereInt8HTTPProvider``, which raises like the reference's constructor when the variables are
    unset); ``rerank_provider`` the ``COHERE_RERANK_*`` one (read per call, as the reference does)."""
    MODE, QKEY, QDTYPE, HAMMING_ONLY, VEC_DTYPE = "bin16", "int8", torch.int8, True, torch.int8
    EMPTY_MSG = "To create a new database, the folder must be empty."

    def __init__(self, folder: str, model: str = "embed-english-v3.0", embedding_dim: int = 1024,
                 rdict_options=None, *, provider=None, rerank_provider=None, device=None):
        if provider is None:
            from .embed import CohereInt8HTTPProvider
            provider = CohereInt8HTTPProvider(model=model, embedding_dim=embedding_dim)
        self.rerank_provider = rerank_provider
        super().__init__(folder, model, embedding_dim, None, rdict_options, None, provider, device)
        if getattr(provider, "model", None) is not None and "model" in self.config:
            provider.model = self.config["model"]     # the request posts self.config["model"] (:95)

    def _embed(self, texts, input_type: str = "search_document") -> dict:
        return self.provider.embed_int8(texts, input_type)

    def search_rerank_cohere(self, query: str, k: int = 10, binary_oversample: int = 10,
                             rerank_model: str = "rerank-english-v3.0") -> List[Dict]:
        """Phase I over the whole index (``binary_k = min(k * binary_oversample, ntotal)`` candidates
        in FAISS order, ``:281-285``), their texts (``:288-295``), one rerank request with
        ``top_n = k`` (``:307-312``) and the results mapped back through ``index`` and stably sorted
        by ``relevance_score`` descending (``:329-338``).  Every failure logs and returns ``[]``."""
        from .embed import CohereRerankHTTPProvider
        rr = self.rerank_provider if self.rerank_provider is not None else CohereRerankHTTPProvider()
        if not rr.configured():
            return []
        if self.index.ntotal == 0:
            logger.error("No documents indexed. Please add documents before searching.")
            return []
        emb = self._embed([query], "search_query")
        if not emb or query not in emb:
            logger.error("Query embedding generation failed. Returning empty results.")
            return []
        binary_k = min(k * binary_oversample, self.index.ntotal)
        hits = self.search_vectors(emb[query], binary_k, 1)[0][0].cpu().numpy().tolist() if binary_k > 0 else []
        cand_ids, cands = [], []
        for e in hits:
            if e != -1 and e in self.texts:
                cand_ids.append(int(e))
                cands.append(self.texts[e])
        if not cands:
            logger.error("No candidate documents found for reranking.")
            return []
        results = rr.rerank(query, cands, k, rerank_model)
        if not results:
            return []
        out = [{"doc_id": cand_ids[r["index"]], "score": r["relevance_score"], "doc": cands[r["index"]]}
               for r in results]
        out.sort(key=lambda x: x["score"], reverse=True)
        return out


def find_closest(db, query: str) -> Dict:
    """``find_closest_*`` helpers of the reference modules (e.g. ``VectorDBInt16.py:297-302``)."""
    results = db.search(query, k=1)
    return results[0] if results else {}
