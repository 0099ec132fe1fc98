"""Embedding providers (the reference's L1 layer) -- plumbing, not the hot path.

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
