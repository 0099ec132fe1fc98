"""GPU parity: libvrq.so kernels on cuda:0 vs the CPU oracle and the reference golden vectors.

Bit-exact for everything integer (codes, int8/int16/int4, Hamming ranks, row
indices, Phase-II float64 scores -- exact sums); Phase-III cosine within 1e-5
relative (north star), with result ORDER checked exactly against the reference
stable-sort rule applied to the GPU's own scores.
"""
import numpy as np
import pytest
import torch

from oracle import oracle_np as O
from tests.conftest import oracle_knn

pytestmark = pytest.mark.gpu

COS_RTOL = 1e-5


def cos_close(got, ref, q, x):
    """1e-5 relative, with the float32-summation floor for near-zero scores: NumPy's sdot and
    the GPU's correctly rounded dot may differ by ~1e-7 * sum|q_i x_i| (cancellation)."""
    if np.isinf(ref) or np.isinf(got):
        return got == ref
    scale = np.abs(q.astype(np.float64) * x.astype(np.float64)).sum() / max(np.linalg.norm(x), 1e-300)
    return abs(got - ref) <= COS_RTOL * max(abs(ref), 1e-2 * scale)


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from vectorragquantization_amd import _native
    _native.load()
    return torch.device("cuda", 0)


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


# ----------------------------------------------------------------------------- encoders
@pytest.mark.parametrize("d", [1024, 384])
def test_encoders_bit_exact_vs_reference_golden(golden, dev, d):
    from vectorragquantization_amd.quant import encode
    g = golden["encoders"]
    X = g[f"x_{d}"]
    for tag in ("l03", "l01", "l10", "ltie"):
        lim = float(g[f"limit_{tag}"])
        r = encode("int8g", X, lim, dev)
        assert np.array_equal(r["q"].cpu().numpy(), g[f"int8g_{tag}_{d}"])
        assert np.array_equal(r["codes"].cpu().numpy(), g[f"bin_int8g_{d}"])
        assert np.array_equal(encode("int16g", X, lim, dev)["q"].cpu().numpy(), g[f"int16g_{tag}_{d}"])
        assert np.array_equal(encode("int4g", X, lim, dev)["q"].cpu().numpy(), g[f"int4g_{tag}_{d}"])
    r = encode("int8", X, 1.0, dev)
    assert np.array_equal(r["q"].cpu().numpy(), g[f"int8_{d}"])
    assert np.array_equal(r["minmax"].cpu().numpy(), g[f"int8_minmax_{d}"])
    r = encode("int4", X, 1.0, dev)
    assert np.array_equal(r["q"].cpu().numpy(), g[f"int4_{d}"])
    assert np.array_equal(r["minmax"].cpu().numpy(), g[f"int4_minmax_{d}"])
    assert np.array_equal(r["codes"].cpu().numpy(), g[f"bin_int4_{d}"])
    assert np.array_equal(encode("bin16", g[f"x16_{d}"], 1.0, dev)["codes"].cpu().numpy(), g[f"bin16_{d}"])


@pytest.mark.parametrize("d", [1024, 768, 1000, 128, 8])
def test_encoders_random_batches_vs_oracle(dev, d):
    from vectorragquantization_amd.quant import encode
    rng = np.random.default_rng(d)
    X = (rng.standard_normal((300, d)) * rng.uniform(0.01, 2.0, (300, 1))).astype(np.float32)
    for mode in ("int8g", "int16g", "int4g", "int8", "int4", "cohere"):
        c, q, mm = O.encode_batch(mode, X, 0.3)
        r = encode(mode, X, 0.3, dev)
        assert np.array_equal(r["codes"].cpu().numpy(), c), mode
        assert np.array_equal(r["q"].cpu().numpy(), q), mode
        if mm is not None:
            assert np.array_equal(r["minmax"].cpu().numpy(), mm), mode


def test_encoders_persistent_loop_d1024(dev):
    """d = 1024 runs the persistent encoder (each wave loops over vectors, the next one's 4 KiB in
    flight): 9001 vectors = more than one vector per wave, an odd tail, flat rows (min == max), exact
    ties with the mean, values beyond the global limit; bit-exact against the oracle in every mode."""
    from vectorragquantization_amd.quant import encode
    rng = np.random.default_rng(77)
    n = 9001
    X = (rng.standard_normal((n, 1024)) * rng.uniform(0.01, 2.0, (n, 1))).astype(np.float32)
    X[17] = 0.25                                   # flat row: scale 0, mean == every element
    X[4000, :512] = 1.0                            # half the elements exactly at the top
    X[4000, 512:] = -1.0
    X[8999] = np.round(X[8999] * 8) / 8            # many repeated values
    for mode in ("int8g", "int16g", "int4g", "int8", "int4", "cohere"):
        c, q, mm = O.encode_batch(mode, X, 0.3)
        r = encode(mode, X, 0.3, dev)
        assert np.array_equal(r["codes"].cpu().numpy(), c), mode
        assert np.array_equal(r["q"].cpu().numpy(), q), mode
        if mm is not None:
            assert np.array_equal(r["minmax"].cpu().numpy(), mm), mode


def test_int8_norms_exact(dev):
    from vectorragquantization_amd.quant import int8_row_norms
    rng = np.random.default_rng(1)
    x = rng.integers(-128, 128, (777, 1024)).astype(np.int8)
    x[5] = 0
    got = int8_row_norms(_t(x, dev)).cpu().numpy()
    assert np.array_equal(got, O.int8_row_norms(x))


def test_reference_static_encoder_surface(dev):
    from vectorragquantization_amd import quant as Q
    x = np.random.default_rng(2).standard_normal(1024).astype(np.float32) * 0.05
    assert np.array_equal(Q.VectorDBInt8Global._quantize_to_int8(x, 0.3), O.quantize_int8_global(x, 0.3))
    assert np.array_equal(Q.VectorDBInt8Global._to_binary(x), O.to_binary(x))
    q, a, b = Q.VectorDBInt8._quantize_to_int8(x)
    q0, a0, b0 = O.quantize_int8_local(x)
    assert np.array_equal(q, q0) and a == a0 and b == b0
    q, a, b = Q.VectorDBInt4._quantize_to_int4(x)
    q0, a0, b0 = O.quantize_int4_local(x)
    assert np.array_equal(q, q0) and (a, b) == (a0, b0)


# ----------------------------------------------------------------------------- Phase I
def _hamming_gpu(codes, q, k, dev, row_offset=0):
    from vectorragquantization_amd import _native as N
    lib = N.load()
    codes_t, q_t = _t(codes, dev), _t(q, dev)
    nq = q.shape[0]
    D = torch.empty((nq, k), dtype=torch.int32, device=dev)
    R = torch.empty((nq, k), dtype=torch.int64, device=dev)
    ws = torch.empty((max(8, lib.vrq_hamming_topk_workspace_size(codes.shape[0], 128, nq, k)),),
                     dtype=torch.uint8, device=dev)
    rc = lib.vrq_hamming_topk(N.ptr(codes_t), codes.shape[0], 128, row_offset, N.ptr(q_t), nq, k, N.ptr(D),
                              N.ptr(R), N.ptr(ws), ws.numel(), N.stream_handle(dev))
    N.check(rc, "hamming_topk")
    torch.cuda.synchronize()
    return D.cpu().numpy(), R.cpu().numpy()


@pytest.mark.parametrize("n,nq,k", [(1, 1, 1), (37, 3, 100), (4096, 5, 100), (5000, 8, 100),
                                    (50_001, 16, 100), (50_000, 9, 7), (20_000, 2, 1024),
                                    (20_000, 33, 500), (300_000, 4, 100)])
def test_hamming_topk_vs_faiss_restatement(dev, oracle_lib, n, nq, k):
    rng = np.random.default_rng(n + nq + k)
    codes = rng.integers(0, 256, (n, 128), dtype=np.uint8)
    q = rng.integers(0, 256, (nq, 128), dtype=np.uint8)
    q[0] = codes[n // 2]                            # exact hit (dist 0)
    D0, I0 = oracle_knn(oracle_lib, codes, q, k)
    D1, I1 = _hamming_gpu(codes, q, k, dev)
    assert np.array_equal(D0, D1)
    assert np.array_equal(I0, I1)


def test_hamming_topk_heavy_ties_and_offset(dev, oracle_lib):
    rng = np.random.default_rng(11)
    base = rng.integers(0, 256, (25, 128), dtype=np.uint8)
    codes = base[rng.integers(0, 25, 120_000)]      # every distance occurs thousands of times
    q = np.concatenate([base[:4], rng.integers(0, 256, (4, 128), dtype=np.uint8)])
    for k in (1, 100, 1000):
        D0, I0 = oracle_knn(oracle_lib, codes, q, k)
        D1, I1 = _hamming_gpu(codes, q, k, dev, row_offset=5_000_000)
        assert np.array_equal(D0, D1)
        assert np.array_equal(I0 + 5_000_000, I1)


def test_hamming_topk_all_identical_rows(dev, oracle_lib):
    codes = np.full((70_000, 128), 0x5A, dtype=np.uint8)
    q = np.zeros((3, 128), dtype=np.uint8)
    D0, I0 = oracle_knn(oracle_lib, codes, q, 100)
    D1, I1 = _hamming_gpu(codes, q, 100, dev)
    assert np.array_equal(D0, D1) and np.array_equal(I0, I1)
    assert I1[0].tolist() == list(range(100))


# ----------------------------------------------------------------------------- 3-phase
def _search3(codes, x8, qf, qb, k, osb, osi, dev, flags=0, row_offset=0, remap=None):
    from vectorragquantization_amd.enhanced import search3
    from vectorragquantization_amd.quant import int8_row_norms
    x8_t = _t(x8, dev)
    norms = int8_row_norms(x8_t)
    K = min(k * osb, codes.shape[0])
    out = search3(_t(codes, dev), x8_t, norms, _t(qf.astype(np.float32), dev), _t(qb, dev), k, K, k * osi,
                  flags, row_offset, None if remap is None else _t(remap, dev))
    torch.cuda.synchronize()
    return [o.cpu().numpy() for o in out]


def _ref_semantics(qf, qb, codes, x8, rows):
    """Reference-semantics scores of the given internal rows for one query: Hamming distance (FAISS),
    Phase-II ``float(q . (2*unpackbits-1))`` (f64, :290) and Phase-III ``float(q . int8) / norm`` with
    NumPy's float32 dot exactly as the reference computes it (:308-313)."""
    rows = np.asarray(rows, dtype=np.int64)
    ham = np.unpackbits(codes[rows] ^ qb[None, :], axis=1).sum(1).astype(np.int64)
    pm = 2 * np.unpackbits(codes[rows], axis=1).astype(np.int32) - 1
    s2 = np.array([float(qf.dot(p)) for p in pm], dtype=np.float64)
    s3 = np.empty(rows.shape[0], dtype=np.float64)
    for j, r in enumerate(rows.tolist()):
        nrm = np.linalg.norm(x8[r])
        s3[j] = -np.inf if nrm == 0 else float(qf.dot(x8[r])) / nrm
    return ham, s2, s3


def _cos_tol(ref, q, x):
    """cos_close's bound: 1e-5 relative, floored by the float32-summation error of the dot."""
    if np.isinf(ref):
        return 0.0
    scale = np.abs(q.astype(np.float64) * x.astype(np.float64)).sum() / max(np.linalg.norm(x), 1e-300)
    return COS_RTOL * max(abs(ref), 1e-2 * scale)


def _certify(qf, qb, codes, x8, rows, dist, s2, s3, ref_rows):
    """One query's GPU result (internal rows, in final order) against the reference's final rows.

    Every GPU result must carry exactly the reference-semantics Hamming distance and Phase-II score of
    its row and a Phase-III score within the cosine tolerance.  If the rows differ from the reference's,
    the difference must lie inside Phase-III tie groups: position by position the two lists' reference
    scores agree within the tolerance (each list is the stable top-k of the same K3 candidates), and every
    row in only one of the lists has a reference score within the tolerance of the boundary (k-th)
    score.  Returns True for an identical list, False for a certified tie permutation."""
    ham, r2, r3 = _ref_semantics(qf, qb, codes, x8, rows)
    assert np.array_equal(dist, ham), "Hamming distances differ from the reference semantics"
    assert np.array_equal(s2, r2), "Phase-II scores are not bit-exact"
    for j, r in enumerate(rows.tolist()):
        assert cos_close(s3[j], r3[j], qf, x8[r])
    if np.array_equal(rows, ref_rows):
        return True
    assert rows.shape[0] == ref_rows.shape[0]
    _, _, t3 = _ref_semantics(qf, qb, codes, x8, ref_rows)
    for j in range(rows.shape[0]):
        tol = _cos_tol(r3[j], qf, x8[rows[j]]) + _cos_tol(t3[j], qf, x8[ref_rows[j]])
        assert abs(r3[j] - t3[j]) <= tol or (np.isinf(r3[j]) and r3[j] == t3[j]), \
            f"position {j}: a different row with a non-tied score"
    edge = t3[-1]
    for r in set(rows.tolist()) ^ set(ref_rows.tolist()):
        v = _ref_semantics(qf, qb, codes, x8, [r])[2][0]
        assert abs(v - edge) <= 2 * _cos_tol(edge, qf, x8[r]) + _cos_tol(v, qf, x8[r]), \
            "a row outside the reference top-k that is not tied with its k-th score"
    return False


# at most this fraction of queries may differ from the reference by a certified Phase-III tie permutation
MAX_TIE_FRAC = 0.05


def _check_against_table(cnt, rows, dist, s2, s3, ids, g, tag, codes, x8, qf, qb):
    """GPU result vs the reference's own search() output (golden table): identical ids, Hamming
    distances and Phase-II scores and cosine scores within 1e-5 rel, or a certified Phase-III tie
    permutation (``_certify``), on at most MAX_TIE_FRAC of the queries."""
    row_of = {int(e): r for r, e in enumerate(ids.tolist())}  # IDMap2 rev_map: last add wins
    ties = 0
    for q in range(cnt.shape[0]):
        n = int(g[f"{tag}_cnt"][q])
        assert int(cnt[q]) == n
        ref_ids = g[f"{tag}_ids"][q][:n]
        ref_rows = rows[q][:n] if np.array_equal(ids[rows[q][:n]], ref_ids) else \
            np.array([row_of[int(e)] for e in ref_ids], dtype=np.int64)
        same = _certify(qf[q], qb[q], codes, x8, rows[q][:n], dist[q][:n], s2[q][:n], s3[q][:n], ref_rows)
        if same:
            assert np.array_equal(dist[q][:n], g[f"{tag}_ham"][q][:n])
            assert np.array_equal(s2[q][:n], g[f"{tag}_bin"][q][:n])
            np.testing.assert_allclose(s3[q][:n], g[f"{tag}_cos"][q][:n], rtol=COS_RTOL)
        ties += not same
    assert ties <= MAX_TIE_FRAC * cnt.shape[0], f"{ties} of {cnt.shape[0]} queries differ by Phase-III ties"
    return ties


@pytest.mark.parametrize("tag", ["k10", "k50", "k7"])
def test_search3_vs_reference_golden_synth(golden, dev, tag):
    g = golden["search_synth"]
    k, osb, osi = (int(v) for v in g[f"{tag}_params"])
    cnt, rows, dist, s2, s3 = _search3(g["codes"], g["int8"], g["qf"], g["qb"], k, osb, osi, dev)
    _check_against_table(cnt, rows, dist, s2, s3, g["ids"], g, tag, g["codes"], g["int8"], g["qf"], g["qb"])


def test_search3_vs_reference_golden_small_with_removals(golden, dev):
    g = golden["search_synth"]
    cnt, rows, dist, s2, s3 = _search3(g["small_codes"], g["small_int8"], g["qf"], g["qb"], 10, 10, 3, dev)
    _check_against_table(cnt, rows, dist, s2, s3, g["small_rows_ids"], g, "small", g["small_codes"],
                         g["small_int8"], g["qf"], g["qb"])


@pytest.mark.parametrize("tag,k", [("k10", 10), ("k50", 50)])
def test_search3_vs_reference_golden_real_cohere_data(golden, dev, tag, k):
    g = golden["search_real"]
    cnt, rows, dist, s2, s3 = _search3(g["codes"], g["int8"], g["qf"], g["qb"], k, 10, 3, dev)
    ties = _check_against_table(cnt, rows, dist, s2, s3, np.arange(1000), g, tag, g["codes"], g["int8"], g["qf"],
                                g["qb"])
    assert ties == 0  # the real data has no Phase-III near-ties at these queries
    if k == 10:
        rec = np.mean([len(set(rows[q]) & set(g["gt_float_top10"][q])) / 10 for q in range(rows.shape[0])])
        assert rec >= 0.98


def _stable_desc(scores):
    return sorted(range(len(scores)), key=lambda j: -scores[j])


def test_search3_vs_oracle_synthetic(dev):
    rng = np.random.default_rng(21)
    n, nq = 20_000, 48
    C = rng.standard_normal((64, 1024)) / 32.0
    F = C[rng.integers(0, 64, n)] + (0.6 / 32.0) * rng.standard_normal((n, 1024))
    F = (F / np.linalg.norm(F, axis=1, keepdims=True)).astype(np.float32)
    F[17] = F[3]                                          # duplicate rows -> ties in every phase
    codes, x8, _ = O.encode_batch("cohere", F, 0.1)
    qf = F[rng.integers(0, n, nq)] + (0.3 / 32.0) * rng.standard_normal((nq, 1024))
    qf = (qf / np.linalg.norm(qf, axis=1, keepdims=True)).astype(np.float32)
    qb, _, _ = O.encode_batch("cohere", qf, 0.1)
    ids = np.arange(n, dtype=np.int64)
    ref = O.three_phase_batch(codes, x8, ids, qf, qb, 10, 10, 3)
    cnt, rows, dist, s2, s3 = _search3(codes, x8, qf, qb, 10, 10, 3, dev)
    # Phase I exactly (via PHASE1_ONLY)
    c1, r1, d1, _, _ = _search3(codes, x8, qf, qb, 10, 10, 3, dev, flags=1)
    ties = 0
    for q in range(nq):
        o = ref[q]
        assert np.array_equal(r1[q], o["p1_rows"]) and np.array_equal(d1[q], o["p1_dist"])
        # final rows identical, or a certified Phase-III tie permutation (bounded below)
        assert int(cnt[q]) == len(o["row"])
        same = _certify(qf[q], qb[q], codes, x8, rows[q], dist[q], s2[q], s3[q], o["row"])
        if same:
            assert np.array_equal(s2[q], o["binary"])
            np.testing.assert_allclose(s3[q], o["cosine"], rtol=COS_RTOL)
        ties += not same
    assert ties <= MAX_TIE_FRAC * nq


def test_shard_mode_and_merge_equal_single_index(dev):
    from vectorragquantization_amd.dist import merge_shards
    rng = np.random.default_rng(4)
    n, nq, k = 30_000, 40, 10
    F = rng.standard_normal((n, 1024)).astype(np.float32) * 0.03
    F[100:200] = F[0:100]                                   # cross-shard duplicates
    codes, x8, _ = O.encode_batch("cohere", F, 0.1)
    qf = (F[rng.integers(0, n, nq)] + 0.01 * rng.standard_normal((nq, 1024))).astype(np.float32)
    qb, _, _ = O.encode_batch("cohere", qf, 0.1)
    full = _search3(codes, x8, qf, qb, k, 10, 3, dev)
    for S in (2, 3, 5):
        bounds = np.linspace(0, n, S + 1).astype(int)
        parts = []
        for s in range(S):
            a, b = bounds[s], bounds[s + 1]
            K = min(k * 10, n)
            from vectorragquantization_amd.enhanced import search3
            from vectorragquantization_amd.quant import int8_row_norms
            x8t = _t(x8[a:b], dev)
            parts.append(search3(_t(codes[a:b], dev), x8t, int8_row_norms(x8t), _t(qf, dev), _t(qb, dev), k, K,
                                 k * 3, 2, int(a)))
        st = [torch.stack([p[i] for p in parts]) for i in range(5)]
        oc, orow, od, o2, o3, src = merge_shards(st[0], st[1], st[2], st[3], st[4], k, k * 3)
        torch.cuda.synchronize()
        assert np.array_equal(oc.cpu().numpy(), full[0])
        assert np.array_equal(orow.cpu().numpy(), full[1])
        assert np.array_equal(od.cpu().numpy(), full[2])
        assert np.array_equal(o2.cpu().numpy(), full[3])
        assert np.array_equal(o3.cpu().numpy(), full[4])


def test_rescore_entry_points(dev):
    from vectorragquantization_amd import _native as N
    from vectorragquantization_amd.quant import int8_row_norms
    rng = np.random.default_rng(8)
    n = 500
    F = rng.standard_normal((n, 1024)).astype(np.float32) * 0.03
    codes, x8, _ = O.encode_batch("cohere", F, 0.1)
    qf = rng.standard_normal((3, 1024)).astype(np.float32) * 0.03
    cand = rng.integers(-1, n, (3, 20)).astype(np.int64)
    x8_t, qf_t, codes_t, cand_t = _t(x8, dev), _t(qf, dev), _t(codes, dev), _t(cand, dev)  # keep alive
    norms = int8_row_norms(x8_t)
    out2 = torch.empty((3, 20), dtype=torch.float64, device=dev)
    out3 = torch.empty((3, 20), dtype=torch.float64, device=dev)
    lib = N.load()
    N.check(lib.vrq_rescore_binary(N.ptr(qf_t), 3, 1024, N.ptr(codes_t), n, N.ptr(cand_t), 20, N.ptr(out2),
                                   N.stream_handle(dev)), "rb")
    N.check(lib.vrq_rescore_int8_cosine(N.ptr(qf_t), 3, 1024, N.ptr(x8_t), N.ptr(norms), n, N.ptr(cand_t), 20,
                                        N.ptr(out3), N.stream_handle(dev)), "rc")
    torch.cuda.synchronize()
    o2, o3 = out2.cpu().numpy(), out3.cpu().numpy()
    for q in range(3):
        for j in range(20):
            r = cand[q, j]
            if r < 0:
                assert np.isnan(o2[q, j]) and np.isnan(o3[q, j])
                continue
            pm = 2 * np.unpackbits(codes[r]).astype(np.int32) - 1
            assert o2[q, j] == float(qf[q].dot(pm))
            nrm = np.linalg.norm(x8[r])
            ref = -np.inf if nrm == 0 else float(qf[q].dot(x8[r])) / nrm
            assert cos_close(o3[q, j], ref, qf[q], x8[r])


# ----------------------------------------------------------------------------- host surface
def test_binary_index_faiss_protocol(dev):
    from vectorragquantization_amd.index import BinaryIndexIDMap2
    rng = np.random.default_rng(9)
    codes = rng.integers(0, 256, (3000, 128), dtype=np.uint8)
    ids = rng.permutation(10_000)[:3000].astype(np.int64)
    a, b = BinaryIndexIDMap2(1024, dev), O.IndexBinaryIDMap2(1024)
    for s in range(0, 3000, 700):
        a.add_with_ids(codes[s:s + 700], ids[s:s + 700])
        b.add_with_ids(codes[s:s + 700], ids[s:s + 700])
    q = codes[[5, 17, 2999]]
    for k in (1, 10, 100):
        Da, La = a.search(q, k)
        Db, Lb = b.search(q, k)
        assert np.array_equal(Da, Db) and np.array_equal(La, Lb)
    assert np.array_equal(a.reconstruct(ids[17]), b.reconstruct(ids[17]))
    rm = ids[::3]
    assert a.remove_ids(rm) == b.remove_ids(rm)
    assert a.ntotal == b.ntotal
    Da, La = a.search(q, 50)
    Db, Lb = b.search(q, 50)
    assert np.array_equal(Da, Db) and np.array_equal(La, Lb)
    c = BinaryIndexIDMap2.from_bytes(a.to_bytes(), dev)
    assert np.array_equal(c.codes.cpu().numpy(), a.codes.cpu().numpy())
    assert np.array_equal(c.id_map.cpu().numpy(), a.id_map.cpu().numpy())


def test_enhanced_db_end_to_end(tmp_path, dev):
    from vectorragquantization_amd.embed import SyntheticCohereProvider
    from vectorragquantization_amd.enhanced import CohereEnhancedVectorDB
    prov = SyntheticCohereProvider(device=dev)
    db = CohereEnhancedVectorDB(str(tmp_path / "db"), provider=prov, device=dev)
    texts = [f"document number {i} about topic {i % 17}" for i in range(700)]
    ids = list(range(100, 800))
    db.add_documents(ids, texts, batch_size=64, save=False)
    db.add_documents([105, 106], ["replacement five", "replacement six"], save=False)   # dedupe path
    db.remove_document(110, save=False)
    assert len(db) == 699
    # oracle: same embeddings through the restated reference
    idx = O.IndexBinaryIDMap2(1024)
    x8d, txd = {}, {}
    F = prov.float_embeddings
    all_ids = db.index.id_map.cpu().numpy()
    idx.add_with_ids(db.index.codes.cpu().numpy(), all_ids)
    x8_all = db._x8.view().cpu().numpy()
    for r, e in enumerate(all_ids):
        x8d[int(e)] = x8_all[r]
        txd[int(e)] = db.texts[int(e)]
    for query in ("topic 3", "replacement five", "document number 42 about topic 8"):
        got = db.search(query, k=10)
        qf = F([query])[0]
        ref = O.three_phase_search(idx, x8d, txd, qf, O.to_binary_sign(qf), 10, 10, 3)
        assert [h["doc_id"] for h in got] == [h["doc_id"] for h in ref]
        assert [h["score_hamming"] for h in got] == [h["score_hamming"] for h in ref]
        assert [h["doc"] for h in got] == [h["doc"] for h in ref]
        np.testing.assert_allclose([h["score_cosine"] for h in got], [h["score_cosine"] for h in ref],
                                   rtol=COS_RTOL)
    db.save()
    db2 = CohereEnhancedVectorDB(str(tmp_path / "db"), provider=prov, device=dev)
    assert len(db2) == 699
    assert db2.search("topic 3", k=5) == db.search("topic 3", k=5)
    assert CohereEnhancedVectorDB(str(tmp_path / "empty"), provider=prov, device=dev).search("x") == []
