"""GPU parity of the exact IndexFlatIP top-k (vrq_flat_ip_topk / FloatIndexIDMap /
CohereVectorDBFloat) against the oracle restatement (oracle.flat_ip_search) and
the reference's own CohereVectorDBFloat run on its persisted 1000-document data (flat_real.npz).

Scores are the float32 inner product as the exact float64 dot rounded once (both sides); rows and
order are compared exactly -- (score desc, row asc) -- except where two scores are within one
float32 ulp (a float64 summation-order difference can flip such a rounding).  Tolerance on the
scores: 1 float32 ulp (<< the 1e-5 relative bar of north_star)."""
import numpy as np
import pytest
import torch

from oracle import oracle_np as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from vectorragquantization_amd import _native
    _native.load()
    return torch.device("cuda", 0)


def _corpus(rng, n, nclus=64):
    C = rng.standard_normal((nclus, 1024)) / 32.0
    F = C[rng.integers(0, nclus, n)] + (0.6 / 32.0) * rng.standard_normal((n, 1024))
    return (F / np.linalg.norm(F, axis=1, keepdims=True)).astype(np.float32)


def _queries(rng, F, nq):
    qf = F[rng.integers(0, F.shape[0], nq)] + (0.3 / 32.0) * rng.standard_normal((nq, 1024))
    return (qf / np.linalg.norm(qf, axis=1, keepdims=True)).astype(np.float32)


def _ulp(x):
    return np.spacing(np.abs(np.asarray(x, np.float32))).astype(np.float64)


def _check(F, qf, k, cnt, rows, sc, row_offset=0):
    S = O.flat_ip_scores(F, qf)
    ref_sc, ref = O.flat_ip_search(F, qf, k)
    m = min(k, F.shape[0])
    for q in range(qf.shape[0]):
        assert cnt[q] == m, (q, cnt[q])
        r = rows[q, :m] - row_offset
        assert np.all(rows[q, m:] == -1)
        assert np.all(np.abs(sc[q, :m] - S[q, r]) <= _ulp(S[q, r])), q   # GPU score of ITS row
        assert np.all(np.abs(sc[q, :m] - ref_sc[q]) <= _ulp(ref_sc[q])), q  # the k-th values agree
        if not np.array_equal(r, ref[q]):
            bad = np.nonzero(r != ref[q])[0]
            assert np.all(np.abs(S[q, r[bad]] - S[q, ref[q][bad]]) <= _ulp(S[q, ref[q][bad]])), (q, bad)
        assert np.all(np.diff(sc[q, :m]) <= 0), q


def _index(F, dev, batch=None):
    from vectorragquantization_amd.flat import FloatIndexIDMap
    idx = FloatIndexIDMap(1024, dev)
    b = batch or F.shape[0]
    for s in range(0, F.shape[0], b):
        idx.add_with_ids(F[s:s + b], np.arange(s, min(s + b, F.shape[0])))
    return idx


def _search(idx, qf, k, flags=0):
    cnt, rows, sc = idx.search_rows(qf, k, flags)
    torch.cuda.synchronize()
    return cnt.cpu().numpy(), rows.cpu().numpy(), sc.cpu().numpy()


@pytest.mark.parametrize("k", [10, 100])
def test_flat_ip_vs_oracle_matrix_path(dev, k):
    from vectorragquantization_amd import _native as N
    rng = np.random.default_rng(21)
    n, nq = 70_000, 300
    F = _corpus(rng, n)
    F[4000] = F[123]                              # exact duplicates -> tied scores, row order decides
    F[61000] = F[123]
    qf = _queries(rng, F, nq)
    qf[3] = F[123]
    idx = _index(F, dev, batch=20_000)            # bounds accumulate over several prepare batches
    cnt, rows, sc = _search(idx, qf, k, N.VRQ_GEMM_NO_FALLBACK)  # the matrix-core path alone must serve it
    _check(F, qf, k, cnt, rows, sc)


def test_flat_ip_edge_cases(dev):
    rng = np.random.default_rng(22)
    n = 5000
    F = _corpus(rng, n)
    F[10] = 0.0                                   # zero row: score exactly 0
    F[11] *= 1e-33                                # below the int8 path's scale floor: all residual
    F[12] *= 40.0                                 # a large row widens the corpus bound
    F[13:20] = F[12] * -1.0                       # negative scores, ties
    qf = _queries(rng, F, 40)
    qf[0] = 0.0                                   # zero query: every score 0 -> rows 0..k-1
    qf[1] = -F[12] / 40.0
    idx = _index(F, dev, batch=999)
    for k in (1, 7, 64):
        cnt, rows, sc = _search(idx, qf, k)
        _check(F, qf, k, cnt, rows, sc)
    small = _index(F[:5], dev)                     # n < k
    cnt, rows, sc = _search(small, qf[:8], 10)
    _check(F[:5], qf[:8], 10, cnt, rows, sc)


def test_flat_ip_prepare_operands(dev):
    """x8 / inv_scale / bounds of vrq_flat_ip_prepare: b = clamp(rint(x * 127 / max|x|)) and the
    bounds dominate every row's ||s b|| and ||x - s b||."""
    from vectorragquantization_amd.flat import flat_ip_prepare
    rng = np.random.default_rng(23)
    F = _corpus(rng, 3000)
    F[5] = 0.0
    bounds = torch.zeros(2, dtype=torch.float64, device=dev)
    x8, inv = flat_ip_prepare(torch.from_numpy(F).to(dev), bounds)
    x8, inv, b = x8.cpu().numpy(), inv.cpu().numpy(), bounds.cpu().numpy()
    mx = np.abs(F).max(axis=1).astype(np.float64)
    live = mx >= 1e-30
    want = np.clip(np.rint(F.astype(np.float64) * (127.0 / np.where(live, mx, 1.0))[:, None]), -127, 127)
    want[~live] = 0
    assert np.array_equal(x8, want.astype(np.int8))
    assert np.allclose(inv[live], 127.0 / mx[live], rtol=1e-15) and np.all(inv[~live] == 1.0)
    s = np.where(live, mx / 127.0, 0.0)[:, None]
    assert b[0] >= np.linalg.norm(s * want, axis=1).max()
    assert b[1] >= np.linalg.norm(F.astype(np.float64) - s * want, axis=1).max()
    assert b[1] <= 1.001 * np.linalg.norm(F.astype(np.float64) - s * want, axis=1).max() + 1e-300


def test_flat_ip_real_data_vs_reference(dev, golden):
    """The reference's CohereVectorDBFloat on its own persisted data (add in 64-doc batches, remove
    ids 5 and 17, re-add 5): same labels, order and scores."""
    g = golden["flat_real"]
    F = g["xf"]
    from vectorragquantization_amd.flat import FloatIndexIDMap
    idx = FloatIndexIDMap(1024, dev)
    for s in range(0, 1000, 64):
        idx.add_with_ids(F[s:s + 64], np.arange(s, min(s + 64, 1000)))
    idx.remove_ids(np.array([5]))
    idx.remove_ids(np.array([17]))
    idx.add_with_ids(F[5:6], np.array([5]))
    assert np.array_equal(idx.id_map.cpu().numpy(), g["row_ids"])
    Fr = F[g["row_ids"]]
    for k in (10, 50):
        D, L = idx.search(g["qf"], k)
        ref_ids, ref_sc = g[f"k{k}_ids"], g[f"k{k}_score"]
        S = O.flat_ip_scores(Fr, g["qf"])
        for q in range(g["qf"].shape[0]):
            assert np.all(np.abs(D[q] - ref_sc[q]) <= _ulp(ref_sc[q])), q
            if not np.array_equal(L[q], ref_ids[q]):
                bad = np.nonzero(L[q] != ref_ids[q])[0]
                row = {int(e): j for j, e in enumerate(g["row_ids"])}
                a = S[q, [row[int(e)] for e in L[q][bad]]]
                b = S[q, [row[int(e)] for e in ref_ids[q][bad]]]
                assert np.all(np.abs(a - b) <= _ulp(b)), (q, bad)


def test_cohere_vector_db_float_surface(dev, tmp_path):
    """CohereVectorDBFloat: add_documents / search dicts / remove / save -> reload (index.faiss)."""
    from vectorragquantization_amd.embed import SyntheticCohereProvider
    from vectorragquantization_amd.flat import CohereVectorDBFloat
    prov = SyntheticCohereProvider()
    docs = [f"document number {i} about topic {i % 7}" for i in range(300)]
    db = CohereVectorDBFloat(str(tmp_path / "db"), provider=prov, device=dev)
    db.add_documents(list(range(300)), docs, batch_size=64, save=True)
    assert len(db) == 300
    res = db.search("document number 42 about topic 0", k=5)
    F = prov.float_embeddings(docs)
    q = prov.float_embeddings(["document number 42 about topic 0"])
    sc, rows = O.flat_ip_search(F, q, 5)
    assert [r["doc_id"] for r in res] == rows[0].tolist()
    assert all(abs(r["score"] - s) <= 1e-6 for r, s in zip(res, sc[0]))
    assert res[0]["doc"] == docs[rows[0][0]]
    db.remove_document(int(rows[0][0]))
    assert len(db) == 299 and int(rows[0][0]) not in [r["doc_id"] for r in db.search(docs[0], k=50)]
    db2 = CohereVectorDBFloat(str(tmp_path / "db"), provider=prov, device=dev)
    assert len(db2) == 299
    assert db2.search(docs[3], k=3) == db.search(docs[3], k=3)


@pytest.mark.parametrize("order", ["random", "cluster_sorted"])
def test_flat_ip_1m_clustered_served_without_fallback(dev, order):
    """1M clustered rows (4096 clusters of ~244: the dense sample holds only a few rows of a query's
    cluster, so the sampled threshold admits far more rows than a candidate list holds).  The
    overflowing queries must be served by the retry pass (threshold raised to the k-th exact score
    among the recorded candidates), not by the one-workgroup full-scan fallback: VRQ_GEMM_NO_FALLBACK
    makes any fallback query an error.  Exact against a float64 matmul (ties within one f32 ulp).
    ``cluster_sorted`` stores the rows in cluster order (the sample's chunks then miss most clusters)."""
    from vectorragquantization_amd import _native as N
    from vectorragquantization_amd.flat import flat_ip_prepare, flat_ip_topk
    g = torch.Generator(device=dev).manual_seed(77)
    n, nq, k = 1_000_000, 128, 10
    cent = torch.randn((4096, 1024), generator=g, device=dev)
    cid = torch.randint(0, 4096, (n,), generator=g, device=dev)
    if order == "cluster_sorted":
        cid = torch.sort(cid).values
    xf = torch.empty((n, 1024), dtype=torch.float32, device=dev)
    for s0 in range(0, n, 1 << 18):
        e = min(n, s0 + (1 << 18))
        b = cent[cid[s0:e]] + 0.7 * torch.randn((e - s0, 1024), generator=g, device=dev)
        xf[s0:e] = b / b.norm(dim=1, keepdim=True)
    qi = torch.randint(0, n, (nq,), generator=g, device=dev)
    qf = xf[qi] + (0.3 / 32.0) * torch.randn((nq, 1024), generator=g, device=dev)
    qf = (qf / qf.norm(dim=1, keepdim=True)).contiguous()
    bounds = torch.zeros((2,), dtype=torch.float64, device=dev)
    x8, inv = flat_ip_prepare(xf, bounds)
    cnt, rows, sc = flat_ip_topk(xf, x8, inv, bounds, qf, k, flags=N.VRQ_GEMM_NO_FALLBACK)
    torch.cuda.synchronize()
    assert bool((cnt == k).all())
    S = (qf.double() @ xf.double().T).float().double()          # the f32-rounded exact dot
    ref_sc, ref = torch.topk(S, k, dim=1)
    got = torch.gather(S, 1, rows)
    ulp = torch.from_numpy(_ulp(ref_sc.cpu().numpy())).to(dev)
    assert bool((torch.abs(sc - got) <= ulp).all())               # each returned score is its row's
    assert bool((torch.abs(sc - ref_sc) <= ulp).all())            # the k best values
    assert bool((torch.diff(sc, dim=1) <= 0).all())
