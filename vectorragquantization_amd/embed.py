"""Embedding providers (the reference's L1 layer) -- plumbing, not the hot path.

``OllamaHTTPProvider`` reproduces the ``VectorDBInt{4,8}{,Global}`` /
``VectorDBInt16Global`` ``_generate_embeddings`` request (e.g.
``VectorDBInt8Global.py:88-128``): one POST per text of ``{"model", "input"}`` to
``embed_url`` (default ``http://localhost:11434/api/embed``), the vector taken
from ``data[0].embedding`` or ``embeddings`` (squeezed), texts whose vector is
missing or of the wrong dimension skipped with a log line.  ``Int16HTTPProvider``
is ``VectorDBInt16._generate_int16_embeddings`` (``VectorDBInt16.py:92-146``):
one POST of ``{"model", "texts", "embedding_bits": 16}`` for the whole batch.
Both return ``{text: vector}`` like the reference; quantisation happens on the
GPU for the whole batch (``vrq_encode``).

``CohereInt8HTTPProvider`` is ``CohereVectorDBInt8._generate_int8_embeddings`` (int8 only) and
``CohereRerankHTTPProvider`` the ``/v2/rerank`` call of ``search_rerank_cohere``
(``CohereVectorDBInt8.py:237-339``), both used by ``vectordb.CohereVectorDBInt8``.

``CohereHTTPProvider`` reproduces ``CohereEnhancedVectorDB._get_embeddings``
(``CohereEnhancedVectorDB.py:136-169``): one JSON POST to ``/v2/embed`` with
``model``, ``texts``, ``input_type``, ``truncate: NONE``, ``embedding_types``;
any failure is logged and ``{}`` returned.  There is no network in the build or
GPU containers, so benchmarks and tests use ``SyntheticCohereProvider``:
deterministic unit-norm float vectors from a stable hash of the text, with
``int8`` = the global-limit int8 quantiser and ``ubinary`` = packbits(x > 0)
computed by the gfx950 encode kernel (``vrq_encode`` mode ``cohere``); that
pair reproduces how Cohere's own int8/ubinary relate to its floats (SURVEY.md
section 0: packbits(float > 0) matches the real ubinary on all but 2 of
1,024,000 bits).
"""
from __future__ import annotations

import hashlib
import logging
import os

import numpy as np

logger = logging.getLogger(__name__)


class CohereHTTPProvider:
    def __init__(self, endpoint: str | None = None, api_key: str | None = None, model: str = "embed-english-v3.0"):
        endpoint = endpoint or os.environ.get("COHERE_EMBED_ENDPOINT")
        if not endpoint:
            raise Exception("COHERE_EMBED_ENDPOINT is not set in the environment.")
        if "/v2/embed" not in endpoint:
            endpoint = endpoint.rstrip("/") + "/v2/embed"
        api_key = api_key or os.environ.get("COHERE_EMBED_KEY")
        if not api_key:
            raise Exception("COHERE_EMBED_KEY is not set in the environment.")
        self.endpoint, self.api_key, self.model = endpoint, api_key, model

    def embed(self, texts, input_type: str, embedding_types) -> dict:
        import requests
        headers = {"Authorization": f"Bearer {self.api_key}", "Content-Type": "application/json"}
        payload = {"model": self.model, "texts": list(texts), "input_type": input_type,
                   "truncate": "NONE", "embedding_types": list(embedding_types)}
        try:
            r = requests.post(self.endpoint, headers=headers, json=payload)
            r.raise_for_status()
            return r.json().get("embeddings", {})
        except Exception as e:  # same contract as the reference: log + {}
            logger.error("Embedding generation failed: %s", str(e))
            return {}


class CohereInt8HTTPProvider(CohereHTTPProvider):
    """``CohereVectorDBInt8._generate_int8_embeddings`` (``CohereVectorDBInt8.py:84-128``): one POST of
    the batch asking for ``embedding_types: ["int8"]``; each text's vector is
    ``embeddings.int8[i]`` (squeezed), texts of the wrong dimension skipped with a log line."""

    def __init__(self, endpoint: str | None = None, api_key: str | None = None, model: str = "embed-english-v3.0",
                 embedding_dim: int = 1024):
        super().__init__(endpoint, api_key, model)
        self.dim = embedding_dim

    def embed_int8(self, texts, input_type: str = "search_document") -> dict:
        emb = self.embed(texts, input_type, ["int8"])
        out = {}
        if not emb:
            return out
        for i, text in enumerate(texts):
            try:
                a = np.array(emb["int8"][i], dtype=np.int8)
                if a.ndim > 1:
                    a = a[0]
                if a.shape[0] != self.dim:
                    logger.error(f"Embedding dimension mismatch for text='{text}'. "
                                 f"Got {a.shape[0]}, expected {self.dim}. Skipping.")
                    continue
                out[text] = a
            except Exception as ex:   # the reference logs and skips the text
                logger.error(f"Error processing int8 embedding for text='{text}': {ex}")
        return out


class CohereRerankHTTPProvider:
    """The Cohere ``/v2/rerank`` call of ``CohereVectorDBInt8.search_rerank_cohere``
    (``CohereVectorDBInt8.py:256-326``).  Endpoint and key come from ``COHERE_RERANK_ENDPOINT`` /
    ``COHERE_RERANK_KEY`` when not given; ``/v2/rerank`` is appended unless the endpoint already ends
    with it.  ``rerank`` POSTs ``{"model", "query", "top_n", "documents"}`` with a Bearer key and
    returns the response's ``results`` list (``[{"index", "relevance_score"}, ...]``), or ``None``
    after logging when the call fails or the response has no results -- the reference then
    returns ``[]``."""

    def __init__(self, endpoint: str | None = None, api_key: str | None = None):
        self.endpoint = endpoint if endpoint is not None else os.environ.get("COHERE_RERANK_ENDPOINT")
        if self.endpoint and not self.endpoint.endswith("/v2/rerank"):
            self.endpoint = self.endpoint.rstrip("/") + "/v2/rerank"
        self.api_key = api_key if api_key is not None else os.environ.get("COHERE_RERANK_KEY")

    def configured(self) -> bool:
        if not self.endpoint:
            logger.error("COHERE_RERANK_ENDPOINT not set in the environment.")
            return False
        if not self.api_key:
            logger.error("COHERE_RERANK_KEY not set in the environment.")
            return False
        return True

    def rerank(self, query: str, documents, top_n: int, model: str = "rerank-english-v3.0"):
        import requests
        headers = {"Authorization": f"Bearer {self.api_key}", "Content-Type": "application/json"}
        payload = {"model": model, "query": query, "top_n": top_n, "documents": list(documents)}
        logger.info("Calling Cohere rerank API at %s", self.endpoint)
        try:
            r = requests.post(self.endpoint, headers=headers, json=payload)
            r.raise_for_status()
            data = r.json()
        except Exception as e:
            logger.error("Rerank API call failed: %s", str(e))
            return None
        results = data.get("results")
        if not results:
            logger.error("Rerank response missing 'results'.")
            return None
        return results


class OllamaHTTPProvider:
    def __init__(self, embed_url: str = "http://localhost:11434/api/embed", model: str = "snowflake-arctic-embed2",
                 embedding_dim: int = 1024):
        self.embed_url, self.model, self.dim = embed_url, model, embedding_dim

    def embed_floats(self, texts) -> dict:
        import requests
        out = {}
        for text in texts:
            try:
                r = requests.post(self.embed_url, json={"model": self.model, "input": text})
                r.raise_for_status()
                data = r.json()
                if "data" in data and data["data"]:
                    e = np.array(data["data"][0]["embedding"], dtype=np.float32)
                elif "embeddings" in data and data["embeddings"]:
                    e = np.array(data["embeddings"], dtype=np.float32)
                else:
                    logger.warning(f"No embedding generated for text: {text}")
                    continue
                if e.ndim > 1:
                    e = e[0]
                if e.shape[0] != self.dim:
                    logger.error(f"Unexpected embedding dimension: {e.shape[0]}. Expected: {self.dim}. "
                                 f"Skipping '{text}'.")
                    continue
                out[text] = e
            except Exception as ex:  # the reference logs and skips the text
                logger.error(f"Failed to generate embedding for text: '{text}'. Error: {ex}")
        return out


class Int16HTTPProvider:
    def __init__(self, embed_url: str = "http://localhost:11434/api/embed", model: str = "snowflake-arctic-embed2",
                 embedding_dim: int = 1024):
        self.embed_url, self.model, self.dim = embed_url, model, embedding_dim

    def embed_int16(self, texts) -> dict:
        import requests
        out = {}
        if not texts:
            return out
        try:
            r = requests.post(self.embed_url, json={"model": self.model, "texts": list(texts), "embedding_bits": 16})
            r.raise_for_status()
        except Exception as ex:
            logger.error(f"Int16 embedding generation failed: {ex}")
            return out
        emb = r.json().get("embeddings", [])
        if len(emb) != len(texts):
            logger.error(f"Mismatch: got {len(emb)} embeddings for {len(texts)} texts.")
            return out
        for i, text in enumerate(texts):
            a = np.array(emb[i], dtype=np.int16)
            if a.shape[0] != self.dim:
                logger.error(f"Dimension mismatch for text={text}. Got {a.shape[0]}, expected {self.dim}")
                continue
            out[text] = a
        return out


class TableProvider:
    """Offline provider for tests and benchmarks: ``{text: vector}`` lookups (float32 or int16
    vectors), texts not in the table skipped like a failed request."""

    def __init__(self, table: dict):
        self.table = table

    def embed_floats(self, texts) -> dict:
        return {t: np.asarray(self.table[t], dtype=np.float32) for t in texts if t in self.table}

    def embed_int16(self, texts) -> dict:
        return {t: np.asarray(self.table[t], dtype=np.int16) for t in texts if t in self.table}

    def embed_int8(self, texts, input_type: str = "search_document") -> dict:
        return {t: np.asarray(self.table[t], dtype=np.int8) for t in texts if t in self.table}


def text_seed(text: str) -> int:
    """Stable (process-independent) 64-bit seed of a text (the reference's mock
    used the salted ``hash()``, embedding_service.py:17-38, which is not reproducible)."""
    return int.from_bytes(hashlib.blake2b(text.encode("utf-8"), digest_size=8).digest(), "little")


class SyntheticCohereProvider:
    """Deterministic stand-in for Cohere ``embed-english-v3.0`` (d = 1024)."""

    def __init__(self, dim: int = 1024, int8_limit: float = 0.1, device=None):
        self.dim = dim
        self.int8_limit = int8_limit
        self.device = device

    def float_embeddings(self, texts) -> np.ndarray:
        out = np.empty((len(texts), self.dim), dtype=np.float32)
        for i, t in enumerate(texts):
            v = np.random.default_rng(text_seed(t)).standard_normal(self.dim)
            out[i] = v / np.linalg.norm(v)
        return out

    def embed(self, texts, input_type: str, embedding_types) -> dict:
        from .quant import encode
        F = self.float_embeddings(texts)
        res = {}
        if "float" in embedding_types:
            res["float"] = F
        if "int8" in embedding_types or "ubinary" in embedding_types:
            e = encode("cohere", F, self.int8_limit, self.device)
            if "int8" in embedding_types:
                res["int8"] = e["q"]
            if "ubinary" in embedding_types:
                res["ubinary"] = e["codes"]
        return res
