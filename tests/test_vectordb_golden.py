"""VectorDB* classes: the oracle restatement ``oracle_np.QuantVectorDB`` against
the golden tables made by running each reference class's own ``add_documents`` / ``remove_document``
/ ``search`` (both ``compare_float32`` values; tests/golden/make_golden.py ``vectordb_synth``), and the
shared tie-certified table check the GPU tests use (tests/test_gpu_vectordb_classes.py).

Parity bar: Phase I (Hamming ranks, FAISS order) is exact, so every query sees the same candidates;
scores are the float32 dot within 1e-5 relative (with the float32 summation floor near zero), and a
position may hold a different doc id only when that doc's score ties the reference's score at that
position (Python's stable sort of float32-rounded values)."""
import numpy as np
import pytest

from oracle import oracle_np as O

TAGS = {"int8g": 0.3, "int16g": 1.0, "int4g": 0.18, "int8": 0.0, "int4": 0.0, "bin16": 0.0}
SEARCHES = {"k10": (10, 10), "k5": (5, 3), "k30": (30, 2)}


def oracle_db(G, tag):
    X = G["X16"] if tag == "bin16" else G["F"]
    ids = G["ids"].tolist()
    db = O.QuantVectorDB(tag, TAGS[tag])
    for s in range(0, len(ids), 64):
        db.add(ids[s:s + 64], X[s:s + 64])
    db.remove(ids[10])
    db.remove(ids[11])
    db.add([ids[11], 9001, 9001], np.stack([X[12], X[5], X[6]]))
    return db


def row_score(db, qv, e, cf32):
    """(oracle score, float32 summation scale) of doc id e for query qv."""
    q, mm, f = db.store[e]
    row = np.asarray(f, np.float32).reshape(1, -1) if cf32 else \
        O.dequantize(db.mode, q.reshape(1, -1), None if mm is None else mm.reshape(1, 2), db.limit)
    s = float(O.dequant_scores(np.asarray(qv, np.float32).reshape(1, -1), row)[0, 0])
    return s, float(np.abs(np.asarray(qv, np.float64) * row[0].astype(np.float64)).sum())


def check_table(got_ids, got_sc, ref_ids, ref_sc, ref_cnt, score_of, exact=False, max_swapped_frac=0.25):
    """Tie-certified comparison of ranked result tables ([nq, k]; ``score_of(q, id) -> (s, scale)``).
    Returns the number of queries whose id order differs from the reference."""
    nq = ref_ids.shape[0]
    swapped = 0
    for q in range(nq):
        c = int(ref_cnt[q])
        gi, gs = got_ids[q][got_ids[q] != -1], got_sc[q][got_ids[q] != -1]
        assert gi.shape[0] == c, (q, gi.shape[0], c)
        ri, rs = ref_ids[q, :c], ref_sc[q, :c]
        if exact:
            assert np.array_equal(gi, ri) and np.array_equal(gs, rs), q
            continue
        for p in range(c):
            s, scale = score_of(q, int(gi[p]))
            tol = 1e-5 * max(abs(rs[p]), 1e-2 * scale)
            assert abs(gs[p] - rs[p]) <= tol, (q, p, gs[p], rs[p])
            assert abs(s - rs[p]) <= tol, (q, p, int(gi[p]), int(ri[p]), s, rs[p])   # a swap is a tie
        if not np.array_equal(gi, ri):
            swapped += 1
    assert swapped <= max(2, int(max_swapped_frac * nq)), swapped
    return swapped


@pytest.mark.parametrize("tag", list(TAGS))
def test_oracle_vectordb_matches_reference_golden(golden_vdb, tag):
    G = golden_vdb
    db = oracle_db(G, tag)
    assert np.array_equal(db.index.id_map, G[f"{tag}_id_map"])
    assert np.array_equal(db.index.xb, G[f"{tag}_codes"])
    Qv = G["Q16"] if tag == "bin16" else G["QF"]
    for cname, (k, osb) in SEARCHES.items():
        for cf in ((False,) if tag == "bin16" else (False, True)):
            key = f"{tag}_{cname}_{'f32' if cf else 'q'}"
            got = [db.search(Qv[j], k, osb, cf) for j in range(Qv.shape[0])]
            gi = np.full((Qv.shape[0], k), -1, np.int64)
            gs = np.full((Qv.shape[0], k), np.nan)
            for j, r in enumerate(got):
                for p, (e, s) in enumerate(r):
                    gi[j, p], gs[j, p] = e, s
            check_table(gi, gs, G[f"{key}_ids"], G[f"{key}_score"], G[f"{key}_cnt"],
                        lambda q, e: row_score(db, Qv[q], e, cf), exact=tag == "bin16")


def test_vectordb_real_golden_shape(golden_vdb_real):
    """The reference's own search on its persisted folders: every float class answers all queries with
    compare_float32=False and raises KeyError with compare_float32=True (no float rows on disk)."""
    G = golden_vdb_real
    for tag in TAGS:
        assert int(G[f"{tag}_ntotal"]) == 1000
        for cname, (k, _) in SEARCHES.items():
            assert np.all(G[f"{tag}_{cname}_q_cnt"] == k)
            if tag != "bin16":
                assert np.all(G[f"{tag}_{cname}_f32_keyerror"] == 1)
