"""Deterministic stand-ins for the Cohere HTTP services (no network anywhere), shared by the fixture
generator (run against the reference's ``CohereVectorDBInt8``) and the tests (run against the
product), so both sides see the same service answers.

``fake_rerank`` plays ``POST /v2/rerank``: relevance = a stable hash of (query, document) quantised
to 1/16 (frequent ties), the ``top_n`` best by (relevance desc, index asc), returned in DESCENDING
index order -- not sorted by relevance -- so the client's own stable sort
(``CohereVectorDBInt8.py:338``) decides the order of tied results."""
from __future__ import annotations

import hashlib


def rerank_score(query: str, doc: str) -> float:
    h = hashlib.blake2b((query + "\x00" + doc).encode("utf-8"), digest_size=8).digest()
    return (int.from_bytes(h, "little") % 16) / 16.0


def fake_rerank(query: str, documents, top_n: int):
    sc = [rerank_score(query, d) for d in documents]
    best = sorted(range(len(documents)), key=lambda i: (-sc[i], i))[:top_n]
    return [{"index": i, "relevance_score": sc[i]} for i in sorted(best, reverse=True)]


class Resp:
    def __init__(self, d):
        self._d = d

    def raise_for_status(self):
        pass

    def json(self):
        return self._d


class FakeCohereRequests:
    """``requests`` for the Cohere classes: ``/v2/embed`` with ``embedding_types: ["int8"]`` answers
    from ``table`` ({text: int8 vector}; an unknown text fails the whole request like an HTTP error),
    ``/v2/rerank`` answers with ``fake_rerank``.  Every payload is recorded in ``calls``."""

    def __init__(self, table):
        self.table = table
        self.calls = []

    def post(self, url, headers=None, json=None, **kw):
        self.calls.append((url, dict(headers or {}), json))
        if url.endswith("/v2/rerank"):
            return Resp({"id": "fake", "results": fake_rerank(json["query"], json["documents"], json["top_n"])})
        for t in json["texts"]:
            if t not in self.table:
                raise RuntimeError(f"no embedding for {t!r}")
        return Resp({"embeddings": {"int8": [self.table[t].tolist() for t in json["texts"]]}})
