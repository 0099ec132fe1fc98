"""Pin the CPU oracle to the golden vectors produced by the reference's own code
(tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest

from oracle import oracle_np as O
from tests.conftest import oracle_knn


@pytest.mark.parametrize("d", [1024, 384])
def test_encoders_match_reference(golden, d):
    g = golden["encoders"]
    X = g[f"x_{d}"]
    for tag in ("l03", "l01", "l10", "ltie"):
        lim = float(g[f"limit_{tag}"])
        for x, r8, r16, r4 in zip(X, g[f"int8g_{tag}_{d}"], g[f"int16g_{tag}_{d}"], g[f"int4g_{tag}_{d}"]):
            assert np.array_equal(O.quantize_int8_global(x, lim), r8)
            assert np.array_equal(O.quantize_int16_global(x, lim), r16)
            assert np.array_equal(O.quantize_int4_global(x, lim), r4)
    for i, x in enumerate(X):
        q, a, b = O.quantize_int8_local(x)
        assert np.array_equal(q, g[f"int8_{d}"][i])
        assert (float(a), float(b)) == tuple(g[f"int8_minmax_{d}"][i])
        q, a, b = O.quantize_int4_local(x)
        assert np.array_equal(q, g[f"int4_{d}"][i])
        assert (a, b) == tuple(g[f"int4_minmax_{d}"][i])
        for name in ("int8g", "int16g", "int4g", "int8", "int4"):
            assert np.array_equal(O.to_binary(x), g[f"bin_{name}_{d}"][i])
    for x, ref in zip(g[f"x16_{d}"], g[f"bin16_{d}"]):
        assert np.array_equal(O.to_binary(x), ref)


def test_encoder_golden_covers_edge_cases(golden):
    g = golden["encoders"]
    X = g["x_1024"]
    # exact half-way ties were generated (limit 127/64 -> scale 64): rounding must be half-even
    t = X[-4].astype(np.float64) * 64.0
    assert np.all(np.abs(t - np.round(t)) == 0.5)
    # flat vectors quantise to zeros (VectorDBInt4.py:133-135, VectorDBInt8.py:121-122)
    assert np.all(g["int4_1024"][43] == 0) and np.all(g["int8_1024"][44] == 0)  # zeros, constant 0.125


def _oracle_db(codes, int8, ids):
    idx = O.IndexBinaryIDMap2(1024)
    idx.add_with_ids(codes, ids)
    return idx, {int(e): int8[i] for i, e in enumerate(ids)}, {int(e): "" for e in ids}


@pytest.mark.parametrize("tag", ["k10", "k50", "k7"])
def test_three_phase_oracle_matches_reference_synth(golden, tag):
    g = golden["search_synth"]
    k, osb, osi = (int(v) for v in g[f"{tag}_params"])
    idx, x8, tx = _oracle_db(g["codes"], g["int8"], g["ids"])
    for q in range(g["qf"].shape[0]):
        res = O.three_phase_search(idx, x8, tx, g["qf"][q], g["qb"][q], k, osb, osi)
        n = int(g[f"{tag}_cnt"][q])
        assert len(res) == n
        assert [h["doc_id"] for h in res] == g[f"{tag}_ids"][q][:n].tolist()
        assert [h["score_hamming"] for h in res] == g[f"{tag}_ham"][q][:n].tolist()
        assert np.array_equal([h["score_binary"] for h in res], g[f"{tag}_bin"][q][:n])
        assert np.array_equal([h["score_cosine"] for h in res], g[f"{tag}_cos"][q][:n])


def test_three_phase_batch_oracle_matches_reference(golden):
    g = golden["search_synth"]
    out = O.three_phase_batch(g["codes"], g["int8"], g["ids"], g["qf"], g["qb"], 10, 10, 3)
    for q, o in enumerate(out):
        n = int(g["k10_cnt"][q])
        assert o["doc_id"].tolist() == g["k10_ids"][q][:n].tolist()
        assert np.array_equal(o["binary"], g["k10_bin"][q][:n])
        assert np.array_equal(o["cosine"], g["k10_cos"][q][:n])


def test_three_phase_oracle_matches_reference_small_removed(golden):
    """remove_document + re-add with a duplicate id (add_documents dedupe, :190-192)."""
    g = golden["search_synth"]
    idx = O.IndexBinaryIDMap2(1024)
    idx.add_with_ids(g["small_codes"], g["small_rows_ids"])
    x8 = {int(e): g["small_int8"][i] for i, e in enumerate(g["small_rows_ids"])}
    tx = {int(e): "" for e in g["small_rows_ids"]}
    for q in range(g["qf"].shape[0]):
        res = O.three_phase_search(idx, x8, tx, g["qf"][q], g["qb"][q], 10, 10, 3)
        assert [h["doc_id"] for h in res] == g["small_ids"][q].tolist()
        assert np.array_equal([h["score_cosine"] for h in res], g["small_cos"][q])


@pytest.mark.parametrize("tag", ["k10", "k50"])
def test_three_phase_oracle_matches_reference_real_data(golden, tag):
    g = golden["search_real"]
    ids = np.arange(1000, dtype=np.int64)
    idx, x8, tx = _oracle_db(g["codes"], g["int8"], ids)
    k = 10 if tag == "k10" else 50
    for q in range(0, g["qf"].shape[0], 7):
        res = O.three_phase_search(idx, x8, tx, g["qf"][q], g["qb"][q], k, 10, 3)
        assert [h["doc_id"] for h in res] == g[f"{tag}_ids"][q].tolist()
        assert np.array_equal([h["score_cosine"] for h in res], g[f"{tag}_cos"][q])


def test_real_data_recall_and_sign_bits(golden):
    g = golden["search_real"]
    # Cohere ubinary == packbits(float > 0) except 2 bits
    assert int(g["sign_bits_mismatch"]) == 2
    rec = np.mean([len(set(a) & set(b)) / 10 for a, b in zip(g["k10_ids"], g["gt_float_top10"])])
    assert abs(rec - 0.988) < 1e-9


def test_c_oracle_matches_numpy_faiss_restatement(oracle_lib):
    rng = np.random.default_rng(3)
    # few distinct codes -> massive distance ties: the (dist, row) order is what is tested
    base = rng.integers(0, 256, (40, 128), dtype=np.uint8)
    codes = base[rng.integers(0, 40, 3000)]
    q = np.concatenate([base[:3], rng.integers(0, 256, (5, 128), dtype=np.uint8)])
    for k in (1, 7, 100, 1000, 3000, 3500):
        D1, I1 = O.binary_flat_search(codes, q, k)
        D2, I2 = oracle_knn(oracle_lib, codes, q, k)
        assert np.array_equal(D1, D2) and np.array_equal(I1, I2)


def test_binary_flat_search_against_brute_force_definition():
    rng = np.random.default_rng(5)
    codes = rng.integers(0, 256, (500, 128), dtype=np.uint8)
    q = rng.integers(0, 256, (3, 128), dtype=np.uint8)
    D, I = O.binary_flat_search(codes, q, 20)
    bits = np.unpackbits(codes, axis=1)
    for j in range(3):
        dist = (bits != np.unpackbits(q[j])).sum(1)
        order = sorted(range(500), key=lambda r: (dist[r], r))[:20]
        assert I[j].tolist() == order
        assert D[j].tolist() == [int(dist[r]) for r in order]


DEQ_KEYS = ["int8g_l03", "int8g_l01", "int8g_l10", "int16g_l03", "int16g_l01", "int16g_l10",
            "int4g_l03", "int4g_l01", "int4g_l10", "int8", "int4"]


def deq_inputs(E, key):
    """(mode, codes, minmax, limit) of a dequant fixture key, from the encoder fixture it was built on."""
    mode, _, tag = key.partition("_")
    if mode in ("int8", "int4"):
        return mode, E[f"{mode}_1024"], E[f"{mode}_minmax_1024"], 0.0
    return mode, E[f"{mode}_{tag}_1024"], None, float(E[f"limit_{tag}"])


def score_close(got, ref, q, deq):
    """float32-dot parity: 1e-5 relative, with the float32 summation floor near zero."""
    scale = np.abs(q.astype(np.float64) * deq.astype(np.float64)).sum()
    return np.abs(got - ref) <= 1e-5 * np.maximum(np.abs(ref), 1e-2 * scale)


@pytest.mark.parametrize("key", DEQ_KEYS)
def test_dequantize_oracle_matches_reference(golden, key):
    """VectorDB*._dequantize_* (the reference's own methods, golden) == the oracle restatement, bit for bit;
    the rescoring expression float(np.dot(q, row)) within the float32-dot tolerance."""
    E, G = golden["encoders"], golden["dequant"]
    mode, q, mm, lim = deq_inputs(E, key)
    D = O.dequantize(mode, q, mm, lim)
    assert np.array_equal(D, G[key])
    S = O.dequant_scores(G["qf"], D)
    for qi in range(G["qf"].shape[0]):
        assert np.all(score_close(S[qi], G[f"score_{key}"][qi], G["qf"][qi], D))


@pytest.mark.parametrize("k", [10, 50])
def test_flat_ip_oracle_matches_reference_real_data(golden, k):
    """IndexFlatIP restatement driven by the reference's own CohereVectorDBFloat (add in batches,
    remove, re-add, search, stable re-sort) on its persisted float data: identical labels and
    scores; and the restated scores agree with a plain float32 BLAS product (FAISS's sgemm path)
    within the float32 summation error."""
    g = golden["flat_real"]
    idx = O.IndexFlatIPIDMap(1024)
    for s in range(0, 1000, 64):
        idx.add_with_ids(g["xf"][s:s + 64], np.arange(s, min(s + 64, 1000)))
    idx.remove_ids([5])
    idx.remove_ids([17])
    idx.add_with_ids(g["xf"][5:6], [5])
    assert np.array_equal(idx.id_map, g["row_ids"])
    D, L = idx.search(g["qf"], k)
    assert np.array_equal(L, g[f"k{k}_ids"])
    assert np.array_equal(D.astype(np.float64), g[f"k{k}_score"])
    S32 = (g["qf"] @ idx.xb.T).astype(np.float64)
    bound = 1e-6 * (np.abs(g["qf"]) @ np.abs(idx.xb).T)
    S = O.flat_ip_scores(idx.xb, g["qf"])
    assert np.all(np.abs(S - S32) <= bound)


def test_flat_ip_search_definition_small():
    """flat_ip_search on a tiny case by brute force: ties by lower row, k > n truncated."""
    rng = np.random.default_rng(3)
    F = rng.standard_normal((9, 1024)).astype(np.float32)
    F[4] = F[1]
    F[7] = 0.0
    Q = np.stack([F[1], np.zeros(1024, np.float32), -F[2]])
    sc, rows = O.flat_ip_search(F, Q, 20)
    assert rows.shape == (3, 9)
    assert rows[0][:2].tolist() == [1, 4]
    assert rows[1].tolist() == list(range(9))
    for q in range(3):
        exact = [float(np.float32(np.dot(Q[q].astype(np.float64), F[r].astype(np.float64)))) for r in rows[q]]
        assert sc[q].tolist() == exact
