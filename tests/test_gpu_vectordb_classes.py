"""GPU parity of the VectorDB* class surface (BASELINE config 1's harness):
``vectorragquantization_amd.vectordb.VectorDBInt{4,8,16}{,Global}`` run the reference's own
add/remove/search sequence and must reproduce the golden tables that each reference class produced
(tests/golden/make_golden.py ``vectordb_synth`` / ``vectordb_real``), for both ``compare_float32``
values, with the tie-certified check of tests/test_vectordb_golden.py (Hamming exact; float32-dot
scores within 1e-5 relative; a different id at a position only if its score ties the reference's).
Real data: the reference's persisted 1000-document folders (tests/golden/ref_db/) opened through the
product's RocksDict reader."""
import os
import shutil

import numpy as np
import pytest
import torch

from tests.test_vectordb_golden import SEARCHES, TAGS, check_table, oracle_db, row_score

pytestmark = pytest.mark.gpu

CLASSES = {"int8g": "VectorDBInt8Global", "int16g": "VectorDBInt16Global", "int4g": "VectorDBInt4Global",
           "int8": "VectorDBInt8", "int4": "VectorDBInt4", "bin16": "VectorDBInt16"}
REF_DB = os.path.join(os.path.dirname(__file__), "golden", "ref_db")
FOLDERS = {"int8g": "db_int8_global", "int16g": "db_int16_global", "int4g": "db_int4_global", "int8": "db_int8",
           "int4": "db_int4", "bin16": "db_int16"}


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from vectorragquantization_amd import _native
    _native.load()
    return torch.device("cuda", 0)


def _cls(tag):
    from vectorragquantization_amd import vectordb
    return getattr(vectordb, CLASSES[tag])


def _build(tag, G, folder, dev):
    from vectorragquantization_amd.embed import TableProvider
    X = G["X16"] if tag == "bin16" else G["F"]
    texts = [f"t{i}" for i in range(X.shape[0])]
    ids = G["ids"].tolist()
    db = _cls(tag)(folder, provider=TableProvider({t: X[i] for i, t in enumerate(texts)}), device=dev)
    db.add_documents(ids, texts, batch_size=64, save=False)
    db.remove_document(ids[10], save=False)
    db.remove_document(ids[11], save=False)
    db.add_documents([ids[11], 9001, 9001], ["t12", "t5", "t6"], save=False)
    return db


def _run(db, tag, Qv, k, osb, cf):
    if tag == "bin16":
        ids, _, ham, sc = db.search_vectors(Qv, k, osb)
    else:
        ids, _, ham, sc = db.search_vectors(Qv, k, osb, cf)
    torch.cuda.synchronize()
    return ids.cpu().numpy(), sc.cpu().numpy()


@pytest.mark.parametrize("tag", list(TAGS))
def test_vectordb_class_vs_reference_golden(golden_vdb, dev, tag, tmp_path):
    G = golden_vdb
    db = _build(tag, G, str(tmp_path / "db"), dev)
    assert np.array_equal(db.index.id_map.cpu().numpy(), G[f"{tag}_id_map"])
    assert np.array_equal(db.index.codes.cpu().numpy(), G[f"{tag}_codes"])
    ref = oracle_db(G, tag)                                    # tie certification only
    Qv = G["Q16"] if tag == "bin16" else G["QF"]
    for cname, (k, osb) in SEARCHES.items():
        for cf in ((False,) if tag == "bin16" else (False, True)):
            key = f"{tag}_{cname}_{'f32' if cf else 'q'}"
            gi, gs = _run(db, tag, Qv, k, osb, cf)
            check_table(gi, gs, G[f"{key}_ids"], G[f"{key}_score"], G[f"{key}_cnt"],
                        lambda q, e: row_score(ref, Qv[q], e, cf), exact=tag == "bin16")
    # the single-query surface returns the reference's dicts
    r = db.search("t3", k=5) if tag == "bin16" else db.search("t3", k=5, compare_float32=True)
    assert [set(h) for h in r] == [{"doc_id", "score", "doc"}] * 5
    assert r[0]["doc_id"] == int(G["ids"][3]) and r[0]["doc"] == "t3"     # ties row 400; lower row first


@pytest.mark.parametrize("tag", list(TAGS))
def test_vectordb_class_save_reopen(golden_vdb, dev, tag, tmp_path):
    """save() -> reopen: same index, same quantised search; compare_float32 raises KeyError afterwards,
    as the reference's in-memory float_embeddings does."""
    G = golden_vdb
    folder = str(tmp_path / "db")
    db = _build(tag, G, folder, dev)
    db.save()
    db2 = _cls(tag)(folder, provider=db.provider, device=dev)
    assert len(db2) == len(db) and np.array_equal(db2.index.id_map.cpu().numpy(), db.index.id_map.cpu().numpy())
    Qv = G["Q16"] if tag == "bin16" else G["QF"]
    a = _run(db, tag, Qv, 10, 10, False)
    b = _run(db2, tag, Qv, 10, 10, False)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    if tag != "bin16":
        with pytest.raises(KeyError):
            db2.search_vectors(Qv[:2], 10, 10, compare_float32=True)
    with pytest.raises(Exception, match="contains files, but no config.json"):
        os.remove(os.path.join(folder, "config.json"))
        _cls(tag)(folder, provider=db.provider, device=dev)


@pytest.mark.parametrize("tag", list(TAGS))
def test_vectordb_class_opens_reference_folder(golden_vdb_real, dev, tag, tmp_path):
    """The reference's persisted folder (index.bin + RocksDict SST) opens with all 1000 documents and
    search reproduces the reference's own search on it; compare_float32=True raises KeyError like it."""
    from vectorragquantization_amd.embed import TableProvider
    G = golden_vdb_real
    folder = str(tmp_path / FOLDERS[tag])
    shutil.copytree(os.path.join(REF_DB, FOLDERS[tag]), folder)
    db = _cls(tag)(folder, provider=TableProvider({}), device=dev)
    assert len(db) == 1000 and len(db.texts) == 1000
    Qv = G["Q16"] if tag == "bin16" else G["QF"]
    for cname, (k, osb) in SEARCHES.items():
        key = f"{tag}_{cname}_q"
        gi, gs = _run(db, tag, Qv, k, osb, False)

        def score_of(q, e):
            from oracle import oracle_np as O
            r = int(np.nonzero(db.index.id_map.cpu().numpy() == e)[0][-1])
            qrow = db._q.view()[r:r + 1].cpu().numpy()
            mm = db._mm.view()[r:r + 1].cpu().numpy() if db.LOCAL else None
            row = O.dequantize(tag, qrow, mm, db.limit)
            s = float(O.dequant_scores(Qv[q:q + 1], row)[0, 0])
            return s, float(np.abs(Qv[q].astype(np.float64) * row[0].astype(np.float64)).sum())
        check_table(gi, gs, G[f"{key}_ids"], G[f"{key}_score"], G[f"{key}_cnt"], score_of, exact=tag == "bin16")
        if tag != "bin16":
            with pytest.raises(KeyError):
                db.search_vectors(Qv[:1], k, osb, compare_float32=True)
    r = db.search("not in the table")          # failed embedding -> [] like the reference
    assert r == []


def test_config1_vectordb_int8_global_10k(dev, tmp_path):
    """BASELINE config 1: VectorDBInt8Global over 10k synthetic d=1024 vectors -- the int8 rows and
    codes bit-exact against the reference encoders' restatement, and 100 searches (k=10,
    binary_oversample=10) against the restated search, scores within 1e-6 relative."""
    from oracle import oracle_np as O
    from vectorragquantization_amd.embed import TableProvider
    rng = np.random.default_rng(1)
    n = 10_000
    C = rng.standard_normal((128, 1024)) / 32.0
    F = (C[rng.integers(0, 128, n)] + (0.5 / 32.0) * rng.standard_normal((n, 1024))).astype(np.float32)
    texts = [f"d{i}" for i in range(n)]
    table = {t: F[i] for i, t in enumerate(texts)}
    Q = (F[rng.integers(0, n, 100)] + 0.004 * rng.standard_normal((100, 1024))).astype(np.float32)
    table.update({f"q{j}": Q[j] for j in range(100)})
    db = _cls("int8g")(str(tmp_path / "c1"), provider=TableProvider(table), device=dev)
    db.add_documents(list(range(n)), texts, batch_size=64, save=False)
    codes, q8, _ = O.encode_batch("int8g", F, 0.3)
    assert np.array_equal(db.index.codes.cpu().numpy(), codes)
    assert np.array_equal(db._q.view().cpu().numpy(), q8)
    ref = O.QuantVectorDB("int8g", 0.3)
    ref.add(list(range(n)), F)
    for j in range(100):
        got = db.search(f"q{j}", k=10, binary_oversample=10)
        exp = ref.search(Q[j], 10, 10)
        assert [h["doc_id"] for h in got] == [e for e, _ in exp]
        assert np.allclose([h["score"] for h in got], [s for _, s in exp], rtol=1e-6, atol=0)
