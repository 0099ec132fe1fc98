"""CohereVectorDBInt8 + Cohere rerank on the CPU: the oracle restatement
against the golden tables the reference's own ``add_documents`` / ``search`` /
``search_rerank_cohere`` produced (tests/golden/make_golden.py ``cohere_int8``, Cohere services =
tests/golden/fake_services.py), and the product's HTTP clients (``CohereInt8HTTPProvider``,
``CohereRerankHTTPProvider``) against the fake services: payloads, URL/env handling and the
log-and-return-[] failures of ``CohereVectorDBInt8.py:84-128,256-326``.  Phase I is Hamming-only,
so every comparison is exact."""
import sys

import numpy as np
import pytest

from oracle import oracle_np as O
from tests.golden.fake_services import FakeCohereRequests, fake_rerank

SEARCHES = {"k10": (10, 10), "k5": (5, 3), "k30": (30, 2)}


def _oracle_db(G):
    X = G["X8"].astype(np.int16)           # the float64 mean of int8 == of the same values as int16
    ids = G["ids"].tolist()
    db = O.QuantVectorDB("bin16")
    for s in range(0, len(ids), 64):
        db.add(ids[s:s + 64], X[s:s + 64])
    db.remove(ids[10])
    db.remove(ids[11])
    db.add([ids[11], 9001, 9001], np.stack([X[12], X[5], X[6]]))
    texts = {e: f"t{i}" for i, e in enumerate(ids)}
    texts.pop(ids[10])
    texts.update({ids[11]: "t12", 9001: "t6"})
    return db, texts


def test_oracle_cohere_int8_matches_reference_golden(golden_cohere_int8):
    G = golden_cohere_int8
    db, texts = _oracle_db(G)
    assert np.array_equal(db.index.id_map, G["id_map"]) and np.array_equal(db.index.xb, G["codes"])
    Q = G["Q8"].astype(np.int16)
    for cname, (k, osb) in SEARCHES.items():
        for j in range(Q.shape[0]):
            got = db.search(Q[j], k, osb)
            c = int(G[f"search_{cname}_cnt"][j])
            assert [e for e, _ in got] == G[f"search_{cname}_ids"][j, :c].tolist()
            assert [s for _, s in got] == G[f"search_{cname}_score"][j, :c].tolist()
            # rerank: all min(k*os, ntotal) Phase-I candidates go to the service, in FAISS order
            cand = [e for e, _ in db.search(Q[j], k * osb, 1)]
            sent = G[f"rerank_{cname}_sent"][j]
            assert cand == sent[sent != -1].tolist()
            docs = [texts[e] for e in cand]
            r = O.rerank_results(cand, docs, fake_rerank(f"q{j}", docs, k))
            c = int(G[f"rerank_{cname}_cnt"][j])
            assert [h["doc_id"] for h in r] == G[f"rerank_{cname}_ids"][j, :c].tolist()
            assert [h["score"] for h in r] == G[f"rerank_{cname}_score"][j, :c].tolist()


def test_golden_rerank_exercises_stable_ties(golden_cohere_int8):
    """The fake service returns tied relevance scores out of order: the fixtures must contain ties so
    the client's stable sort is actually pinned."""
    G = golden_cohere_int8
    sc = G["rerank_k10_score"]
    assert sum(int(np.any(np.diff(row[np.isfinite(row)]) == 0)) for row in sc) >= 4


def test_rerank_provider_payload_and_failures(monkeypatch):
    from vectorragquantization_amd.embed import CohereRerankHTTPProvider
    fake = FakeCohereRequests({})
    monkeypatch.setitem(sys.modules, "requests", fake)
    monkeypatch.delenv("COHERE_RERANK_ENDPOINT", raising=False)
    monkeypatch.delenv("COHERE_RERANK_KEY", raising=False)
    assert not CohereRerankHTTPProvider().configured()
    monkeypatch.setenv("COHERE_RERANK_ENDPOINT", "https://h.invalid/")
    assert not CohereRerankHTTPProvider().configured()               # key still missing
    monkeypatch.setenv("COHERE_RERANK_KEY", "kk")
    p = CohereRerankHTTPProvider()
    assert p.configured() and p.endpoint == "https://h.invalid/v2/rerank"
    assert CohereRerankHTTPProvider("https://h.invalid/v2/rerank", "x").endpoint == "https://h.invalid/v2/rerank"
    docs = ["alpha", "beta", "gamma", "delta"]
    res = p.rerank("query", docs, 2, "rerank-english-v3.0")
    assert res == fake_rerank("query", docs, 2)
    url, hdr, payload = fake.calls[-1]
    assert url == "https://h.invalid/v2/rerank" and hdr["Authorization"] == "Bearer kk"
    assert payload == {"model": "rerank-english-v3.0", "query": "query", "top_n": 2, "documents": docs}

    class Broken:
        def post(self, *a, **kw):
            raise RuntimeError("down")
    monkeypatch.setitem(sys.modules, "requests", Broken())
    assert p.rerank("query", docs, 2) is None

    class Empty:
        def post(self, *a, **kw):
            from tests.golden.fake_services import Resp
            return Resp({"results": []})
    monkeypatch.setitem(sys.modules, "requests", Empty())
    assert p.rerank("query", docs, 2) is None


def test_int8_embed_provider(monkeypatch):
    from vectorragquantization_amd.embed import CohereInt8HTTPProvider
    v = np.arange(-512, 512).astype(np.int8)
    fake = FakeCohereRequests({"a": v, "b": v[::-1].copy()})
    monkeypatch.setitem(sys.modules, "requests", fake)
    monkeypatch.delenv("COHERE_EMBED_ENDPOINT", raising=False)
    with pytest.raises(Exception, match="COHERE_EMBED_ENDPOINT"):
        CohereInt8HTTPProvider()
    p = CohereInt8HTTPProvider("https://e.invalid", "ek", "embed-english-v3.0", 1024)
    out = p.embed_int8(["a", "b"], "search_query")
    assert np.array_equal(out["a"], v) and out["b"].dtype == np.int8
    url, hdr, payload = fake.calls[-1]
    assert url == "https://e.invalid/v2/embed"
    assert payload == {"model": "embed-english-v3.0", "texts": ["a", "b"], "input_type": "search_query",
                       "truncate": "NONE", "embedding_types": ["int8"]}
    assert p.embed_int8(["a", "missing"]) == {}                     # a failed request -> {}
    p.dim = 512
    assert p.embed_int8(["a"]) == {}                                # wrong dimension -> skipped
