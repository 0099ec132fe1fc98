"""GPU parity of the matrix-core Phase-I scan (hamming_mfma.hip) against the FAISS restatement.

The matrix-core path must return exactly what the wavefront scan and FAISS return: the
K smallest (dist, row) pairs, ties broken by row.  Cases cover ragged row counts, batches
that are not multiples of the 256-query workgroup, K = 1 and K = 128 (the path's bound), heavy
ties, the candidate-list overflow that triggers the exact rescan (including dist == T ties
taken in row order), the stage-split ABI, and the full three-phase search agreeing between
the two scans bit for bit.
"""
import numpy as np
import pytest
import torch

from oracle import oracle_np as O
from tests.conftest import oracle_knn

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from vectorragquantization_amd import _native
    _native.load()
    return torch.device("cuda", 0)


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _phase1(codes, qb, K, dev, scan, row_offset=0):
    """vrq_search3 in PHASE1_ONLY mode with an explicit scan selection -> (dist, rows)."""
    from vectorragquantization_amd import _native as N
    from vectorragquantization_amd.enhanced import search3
    n, nq = codes.shape[0], qb.shape[0]
    flags = N.VRQ_SEARCH_PHASE1_ONLY | {"valu": N.VRQ_SEARCH_SCAN_VALU, "mfma": N.VRQ_SEARCH_SCAN_MFMA,
                                        "auto": 0}[scan]
    x8 = torch.empty((1, 1024), dtype=torch.int8, device=dev)
    norms = torch.empty((1,), dtype=torch.float64, device=dev)
    qf = torch.zeros((nq, 1024), dtype=torch.float32, device=dev)
    cnt, rows, dist, _, _ = search3(_t(codes, dev), x8, norms, qf, _t(qb, dev), K, K, K, flags, row_offset)
    torch.cuda.synchronize()
    return cnt.cpu().numpy(), dist.cpu().numpy(), rows.cpu().numpy()


def _near(rng, base, nflip):
    """Copies of `base` rows with exactly nflip distinct bits flipped each."""
    out = base.copy()
    bits = np.unpackbits(out, axis=1)
    for i in range(out.shape[0]):
        pos = rng.choice(1024, nflip, replace=False)
        bits[i, pos] ^= 1
    return np.packbits(bits, axis=1)


@pytest.mark.parametrize("n,nq,K", [(65_536, 1, 100), (70_001, 300, 100), (200_000, 130, 10),
                                    (131_072, 257, 128), (100_003, 128, 1), (500_000, 520, 100),
                                    # the row-split small-batch kernel K1r: MB = 1, 2, 4
                                    (80_000, 20, 100), (90_017, 33, 100), (120_000, 64, 128), (150_001, 100, 50)])
@pytest.mark.parametrize("scan", ["mfma", "valu"])
def test_mfma_phase1_vs_faiss_restatement(dev, oracle_lib, n, nq, K, scan):
    rng = np.random.default_rng(n * 7 + nq + K)
    codes = rng.integers(0, 256, (n, 128), dtype=np.uint8)
    src = rng.integers(0, n, nq)
    qb = _near(rng, codes[src], 40)                      # every query has a close neighbour
    qb[0] = codes[n - 1]                                  # exact hit on the very last row
    codes[rng.integers(0, n, 64)] = qb[-1]                # duplicates of one query across the corpus
    D0, I0 = oracle_knn(oracle_lib, codes, qb, K)
    c, D1, I1 = _phase1(codes, qb, K, dev, scan)
    assert np.array_equal(c, np.full(nq, K))
    assert np.array_equal(D0, D1)
    assert np.array_equal(I0, I1)


def test_mfma_auto_selection_in_hamming_topk(dev, oracle_lib):
    """vrq_hamming_topk picks the matrix-core scan on its own (K <= 128, n >= 65536)."""
    from vectorragquantization_amd.index import BinaryIndexIDMap2
    rng = np.random.default_rng(5)
    n, nq = 150_000, 200
    codes = rng.integers(0, 256, (n, 128), dtype=np.uint8)
    qb = _near(rng, codes[rng.integers(0, n, nq)], 100)
    idx = BinaryIndexIDMap2(1024, dev)
    idx.add_with_ids(codes, np.arange(n) * 3 + 1)
    D1, L1 = idx.search(qb, 50)
    D0, I0 = oracle_knn(oracle_lib, codes, qb, 50)
    assert np.array_equal(D0, D1) and np.array_equal(I0 * 3 + 1, L1)


@pytest.mark.parametrize("nq", [8, 40, 64, 600])     # K1r MB = 1, the lean MB = 2 kernel; K1s
def test_mfma_heavy_ties(dev, oracle_lib, nq):
    rng = np.random.default_rng(11)
    base = rng.integers(0, 256, (25, 128), dtype=np.uint8)
    codes = base[rng.integers(0, 25, 120_000)]            # every distance occurs thousands of times
    qb = np.concatenate([base[:4], rng.integers(0, 256, (nq - 4, 128), dtype=np.uint8)])
    for K in (1, 100, 128):
        D0, I0 = oracle_knn(oracle_lib, codes, qb, K)
        _, D1, I1 = _phase1(codes, qb, K, dev, "mfma", row_offset=5_000_000)
        assert np.array_equal(D0, D1)
        assert np.array_equal(I0 + 5_000_000, I1)


@pytest.mark.parametrize("nq", [130, 600])             # K1m MB = 2; K1s (512-query blocks)
def test_mfma_candidate_overflow_exact_rescan(dev, oracle_lib, nq):
    """Query 0's neighbours fill rows [S, n): far more rows beat its threshold than a candidate
    list holds, so its lists overflow and the corpus is rescanned exactly.  Those rows hold 50
    exact copies (dist 0) and otherwise rows at dist exactly 3, so with K = 100 the answer is
    the 50 copies plus the FIRST 50 dist-3 rows in row order."""
    rng = np.random.default_rng(9)
    n, K = 100_000, 100
    S = 32_768
    codes = rng.integers(0, 256, (n, 128), dtype=np.uint8)
    qb = rng.integers(0, 256, (nq, 128), dtype=np.uint8)
    suffix = _near(rng, np.repeat(qb[:1], n - S, axis=0), 3)
    copies = rng.choice(n - S, 50, replace=False)
    suffix[copies] = qb[0]
    codes[S:] = suffix
    qb[2] = codes[S + 17]                                 # another query, near the suffix too
    D0, I0 = oracle_knn(oracle_lib, codes, qb, K)
    _, D1, I1 = _phase1(codes, qb, K, dev, "mfma")
    assert np.array_equal(D0, D1)
    assert np.array_equal(I0, I1)
    assert (D1[0] == 0).sum() == 50 and (D1[0] == 3).sum() == 50


def test_mfma_stage_split_equals_full_scan(dev, oracle_lib):
    from vectorragquantization_amd import _native as N
    lib = N.load()
    rng = np.random.default_rng(3)
    n, nq, K = 90_000, 140, 100
    codes = rng.integers(0, 256, (n, 128), dtype=np.uint8)
    qb = _near(rng, codes[rng.integers(0, n, nq)], 60)
    c_t, q_t = _t(codes, dev), _t(qb, dev)
    st = N.stream_handle(dev)
    ws = torch.zeros((lib.vrq_search3_workspace_size(n, 1024, nq, K),), dtype=torch.uint8, device=dev)
    cnt = torch.empty((nq,), dtype=torch.int32, device=dev)
    rows = torch.empty((nq, K), dtype=torch.int64, device=dev)
    dist = torch.empty((nq, K), dtype=torch.int32, device=dev)
    base = N.VRQ_SEARCH_PHASE1_ONLY | N.VRQ_SEARCH_SCAN_MFMA
    for stage in (N.VRQ_SCAN_STAGE_PREFIX, N.VRQ_SCAN_STAGE_MATRIX, N.VRQ_SCAN_STAGE_RECHECK,
                  N.VRQ_SCAN_STAGE_SUFFIX):
        N.check(lib.vrq_search3_scan(N.ptr(c_t), n, 1024, N.ptr(q_t), nq, K, base | stage, N.ptr(ws), ws.numel(),
                                     st), "scan stage")
    N.check(lib.vrq_search3_finish(N.ptr(c_t), None, None, None, n, 1024, 0, None, nq, K, K, K, base, N.ptr(cnt),
                                   N.ptr(rows), N.ptr(dist), None, None, N.ptr(ws), ws.numel(), st), "finish")
    torch.cuda.synchronize()
    D0, I0 = oracle_knn(oracle_lib, codes, qb, K)
    assert np.array_equal(D0, dist.cpu().numpy()) and np.array_equal(I0, rows.cpu().numpy())


def test_mfma_and_valu_three_phase_identical(dev):
    """Full 3-phase outputs (rows, dist, s2, s3) are bit-identical between the two scans."""
    from vectorragquantization_amd import _native as N
    from vectorragquantization_amd.enhanced import search3
    from vectorragquantization_amd.quant import int8_row_norms
    rng = np.random.default_rng(21)
    n, nq = 120_000, 256
    C = rng.standard_normal((64, 1024)) / 32.0
    F = (C[rng.integers(0, 64, n)] + (0.6 / 32.0) * rng.standard_normal((n, 1024))).astype(np.float32)
    codes, x8, _ = O.encode_batch("cohere", F, 0.1)
    qf = (F[rng.integers(0, n, nq)] + (0.3 / 32.0) * rng.standard_normal((nq, 1024))).astype(np.float32)
    qb, _, _ = O.encode_batch("cohere", qf, 0.1)
    x8_t = _t(x8, dev)
    norms = int8_row_norms(x8_t)
    outs = {}
    for name, fl in (("valu", N.VRQ_SEARCH_SCAN_VALU), ("mfma", N.VRQ_SEARCH_SCAN_MFMA), ("auto", 0)):
        o = search3(_t(codes, dev), x8_t, norms, _t(qf, dev), _t(qb, dev), 10, 100, 30, fl)
        torch.cuda.synchronize()
        outs[name] = [x.cpu().numpy() for x in o]
    for a, b, c in zip(outs["valu"], outs["mfma"], outs["auto"]):
        assert np.array_equal(a, b, equal_nan=True) and np.array_equal(a, c, equal_nan=True)


@pytest.mark.parametrize("nq", [200, 64, 40, 600])  # K1m MB = 2; the lean MB = 2 K1r (full and partial); K1s
def test_mfma_hit_staging_overflow(dev, oracle_lib, nq):
    """Up to 64 queries (one wave's worth) and the whole suffix clustered around one code: every tile
    gives a wave thousands of hits, more than its LDS staging holds, so the lists are marked overflowed
    and those queries are rescanned exactly; the other queries keep the fast path.  At 40 and 64 queries
    this runs the lean K1r kernel's per-n-block stage overflow, spare-slot clamp and capc + 1 marking."""
    rng = np.random.default_rng(17)
    n, K = 100_000, 100
    S = 32_768
    base = rng.integers(0, 256, (1, 128), dtype=np.uint8)
    codes = rng.integers(0, 256, (n, 128), dtype=np.uint8)
    codes[S:] = _near(rng, np.repeat(base, n - S, axis=0), 6)
    qb = rng.integers(0, 256, (nq, 128), dtype=np.uint8)
    nh = min(nq, 64)
    qb[:nh] = _near(rng, np.repeat(base, nh, axis=0), 4)
    D0, I0 = oracle_knn(oracle_lib, codes, qb, K)
    _, D1, I1 = _phase1(codes, qb, K, dev, "mfma")
    assert np.array_equal(D0, D1)
    assert np.array_equal(I0, I1)


def _sample_rows(n, nq, K=100):
    """Rows of the dense threshold sample, from the library's own plan (vrq_scan_sample_plan): tile
    i = c * T + t of the sample starts at row i * ts (64-row tiles spread over the corpus; for <= 64
    queries the row-split kernel's own sample pass)."""
    from vectorragquantization_amd import _native as N
    info = np.zeros(8, np.int64)
    N.check(N.load().vrq_scan_sample_plan(n, 1024, nq, K, 0, info.ctypes.data), "sample plan")
    chunks, crows, ts = int(info[1]), int(info[2]), int(info[4])
    tiles = chunks * (crows // 64)
    return (np.arange(tiles)[:, None] * ts + np.arange(64)[None, :]).reshape(-1)


@pytest.mark.parametrize("nq", [300, 100, 50, 600])
def test_mfma_sampled_threshold_rerun(dev, oracle_lib, nq):
    """The thresholded pass runs with the sampled tau_s = d_(j)+1 (j < K) of the dense sample.
    Queries 0 and nq - 10 (two different 256-query blocks at nq = 300; the one block of the
    row-split kernel at nq = 100) get 70 near copies (dist <= 20) on sample
    rows and 40 more at dist 30 off the sample, none elsewhere: d_(j) falls among the near
    copies, the dist-30 copies miss tau_s, the check finds C = 70 < K and the re-run with tau_p
    must recover the first 30 of them in row order.  The other queries take the fast path."""
    rng = np.random.default_rng(23)
    n, K = 100_000, 100
    codes = rng.integers(0, 256, (n, 128), dtype=np.uint8)
    qb = _near(rng, codes[rng.integers(0, n, nq)], 50)
    samp = _sample_rows(n, nq)
    off = np.setdiff1d(np.arange(n), samp)
    for q in (0, nq - 10):
        near = rng.choice(samp, 70, replace=False)
        codes[near] = _near(rng, np.repeat(qb[q:q + 1], 70, axis=0), int(rng.integers(5, 21)))
        far = rng.choice(off, 40, replace=False)
        codes[far] = _near(rng, np.repeat(qb[q:q + 1], 40, axis=0), 30)
    D0, I0 = oracle_knn(oracle_lib, codes, qb, K)
    _, D1, I1 = _phase1(codes, qb, K, dev, "mfma")
    assert (D0[0] == 30).sum() == 30 and (D0[nq - 10] == 30).sum() == 30
    assert np.array_equal(D0, D1)
    assert np.array_equal(I0, I1)


@pytest.mark.parametrize("nq", [40, 130, 520])
def test_mfma_cluster_ordered_corpus(dev, oracle_lib, nq):
    """Corpus stored in cluster order (1000 contiguous near-copies of each centre): a query's whole
    neighbourhood sits in one chunk and in few lane rows of the sample, so the sample pass's lane
    minima collapse many near rows into one value each (looser tau_s / tau_p).  The result must
    still be exactly the FAISS order (recheck + re-run + suffix); covers K1r (40 queries), the
    MB = 2 (130) and MB = 4 (520) instances of K1m."""
    rng = np.random.default_rng(4242 + nq)
    ncl, per = 300, 1000
    centres = rng.integers(0, 256, (ncl, 128), dtype=np.uint8)
    bits = np.unpackbits(np.repeat(centres, per, axis=0), axis=1)
    flips = rng.random(bits.shape) < rng.uniform(0.01, 0.06, (bits.shape[0], 1))
    codes = np.packbits(bits ^ flips, axis=1)
    qb = _near(rng, centres[rng.integers(0, ncl, nq)], 12)
    D0, I0 = oracle_knn(oracle_lib, codes, qb, 100)
    c, D1, I1 = _phase1(codes, qb, 100, dev, "mfma")
    assert np.array_equal(c, np.full(nq, 100))
    assert np.array_equal(D0, D1)
    assert np.array_equal(I0, I1)
