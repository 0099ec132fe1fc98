"""GPU parity of ``vectorragquantization_amd.vectordb.CohereVectorDBInt8``:
the reference's add/remove/search/search_rerank_cohere sequence through the product's own HTTP
clients, with ``requests`` replaced by the same fake Cohere services the golden generator used
(tests/golden/fake_services.py), must reproduce the reference's tables exactly -- index layout,
Hamming search (ids, distances), the documents sent to the reranker (Phase-I order) and the
reranked ids/scores.  Also on the reference's persisted ``db_cohere_int8`` folder."""
import os
import shutil
import sys

import numpy as np
import pytest
import torch

from tests.golden.fake_services import FakeCohereRequests

pytestmark = pytest.mark.gpu
SEARCHES = {"k10": (10, 10), "k5": (5, 3), "k30": (30, 2)}
REF_DB = os.path.join(os.path.dirname(__file__), "golden", "ref_db", "db_cohere_int8")


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from vectorragquantization_amd import _native
    _native.load()
    return torch.device("cuda", 0)


def _services(monkeypatch, table):
    fake = FakeCohereRequests(table)
    monkeypatch.setitem(sys.modules, "requests", fake)
    monkeypatch.setenv("COHERE_EMBED_ENDPOINT", "https://embed.invalid")
    monkeypatch.setenv("COHERE_EMBED_KEY", "embed-key")
    monkeypatch.setenv("COHERE_RERANK_ENDPOINT", "https://rerank.invalid")
    monkeypatch.setenv("COHERE_RERANK_KEY", "rerank-key")
    return fake


def _check(db, fake, G, prefix, queries, table):
    for j in range(queries.shape[0]):
        table[f"{prefix}q{j}"] = queries[j]
    for cname, (k, osb) in SEARCHES.items():
        for j in range(queries.shape[0]):
            qt = f"{prefix}q{j}"
            r = db.search(qt, k=k, binary_oversample=osb)
            c = int(G[f"{prefix}search_{cname}_cnt"][j])
            assert [h["doc_id"] for h in r] == G[f"{prefix}search_{cname}_ids"][j, :c].tolist(), (cname, j)
            assert [h["score"] for h in r] == G[f"{prefix}search_{cname}_score"][j, :c].tolist(), (cname, j)
            fake.calls.clear()
            r = db.search_rerank_cohere(qt, k=k, binary_oversample=osb)
            url, hdr, payload = fake.calls[-1]
            assert url == "https://rerank.invalid/v2/rerank" and hdr["Authorization"] == "Bearer rerank-key"
            assert payload["top_n"] == k and payload["query"] == qt and payload["model"] == "rerank-english-v3.0"
            sent = G[f"{prefix}rerank_{cname}_sent"][j]
            assert payload["documents"] == [db.texts[e] for e in sent[sent != -1].tolist()]
            c = int(G[f"{prefix}rerank_{cname}_cnt"][j])
            assert [h["doc_id"] for h in r] == G[f"{prefix}rerank_{cname}_ids"][j, :c].tolist(), (cname, j)
            assert [h["score"] for h in r] == G[f"{prefix}rerank_{cname}_score"][j, :c].tolist(), (cname, j)
            assert all(h["doc"] == db.texts[h["doc_id"]] for h in r)


def test_cohere_int8_vs_reference_golden(golden_cohere_int8, dev, monkeypatch, tmp_path):
    from vectorragquantization_amd.vectordb import CohereVectorDBInt8
    G = golden_cohere_int8
    X8 = G["X8"]
    texts = [f"t{i}" for i in range(X8.shape[0])]
    table = {t: X8[i] for i, t in enumerate(texts)}
    fake = _services(monkeypatch, table)
    db = CohereVectorDBInt8(str(tmp_path / "db"), device=dev)
    ids = G["ids"].tolist()
    db.add_documents(ids, texts, batch_size=64, save=False)
    assert fake.calls[0][2]["input_type"] == "search_document"
    db.remove_document(ids[10], save=False)
    db.remove_document(ids[11], save=False)
    db.add_documents([ids[11], 9001, 9001], ["t12", "t5", "t6"], save=False)
    assert np.array_equal(db.index.id_map.cpu().numpy(), G["id_map"])
    assert np.array_equal(db.index.codes.cpu().numpy(), G["codes"])
    _check(db, fake, G, "", G["Q8"], table)
    # save -> reopen keeps the index and the texts
    db.save()
    db2 = CohereVectorDBInt8(str(tmp_path / "db"), device=dev)
    assert len(db2) == len(db) and db2.texts == db.texts
    _check(db2, fake, G, "", G["Q8"], table)


def test_cohere_int8_opens_reference_folder(golden_cohere_int8, dev, monkeypatch, tmp_path):
    from vectorragquantization_amd.vectordb import CohereVectorDBInt8
    G = golden_cohere_int8
    table = {}
    fake = _services(monkeypatch, table)
    folder = str(tmp_path / "db_cohere_int8")
    shutil.copytree(REF_DB, folder)
    db = CohereVectorDBInt8(folder, device=dev)
    assert len(db) == int(G["real_ntotal"]) == 1000 and len(db.texts) == 1000
    _check(db, fake, G, "real_", G["real_Q8"], table)


def test_cohere_int8_rerank_failures(golden_cohere_int8, dev, monkeypatch, tmp_path):
    """Every failure of ``search_rerank_cohere`` logs and returns [] (``CohereVectorDBInt8.py:256-326``)."""
    from vectorragquantization_amd.vectordb import CohereVectorDBInt8
    G = golden_cohere_int8
    table = {f"t{i}": G["X8"][i] for i in range(100)}
    table["q"] = G["X8"][3]
    _services(monkeypatch, table)
    db = CohereVectorDBInt8(str(tmp_path / "db"), device=dev)
    assert db.search_rerank_cohere("q") == []                       # empty index
    db.add_documents(list(range(100)), [f"t{i}" for i in range(100)], save=False)
    assert len(db.search_rerank_cohere("q", k=5)) == 5
    assert db.search_rerank_cohere("unknown query") == []           # embedding failed
    assert db.search_rerank_cohere("q", k=0) == []                  # no candidates
    monkeypatch.delenv("COHERE_RERANK_KEY")
    assert db.search_rerank_cohere("q") == []
