"""Edge paths of K1m's MB = 4 instance -- the kernel config 4's headline runs -- against the FAISS restatement.

K1s takes every large-batch pass of at most 2^32 (query, row) pairs, so the small-n cases of
test_gpu_mfma.py no longer reach K1m MB = 4.  These cases use n = 4.2M rows and nq >= 1024, i.e.
n * nq > 2^32, assert that ``vrq_scan_plan`` reports K1m with 4 M-blocks per wave (kind 0, MB 4), and
stress the exact-fallback paths the FAISS semantics depend on (CohereEnhancedVectorDB.py:267-275:
strict-< heap insert, (dist, row) order under ties):

* heavy ties (every distance occurs ~170K times);
* candidate-list overflow -> exact rescan, with dist == T ties taken in row order;
* LDS hit-staging overflow (a whole wave of 128 queries and more, with thousands of hits per tile);
* the sampled tau_s failing for two queries in different 512-query blocks -> re-run with tau_p;
* a corpus stored in cluster order (the sample's lane minima collapse near rows).

Each test checks the planted queries plus a spread sample of the others bit for bit (rows and
distances) against the C restatement of ``hammings_knn_hc`` over all rows.
"""
import numpy as np
import pytest
import torch

from tests.conftest import oracle_knn

pytestmark = pytest.mark.gpu

N_BIG = 4_200_007          # n * 1024 = 4.30e9 > 2^32: K1m, not K1s
NQ = 1024


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from vectorragquantization_amd import _native
    _native.load()
    return torch.device("cuda", 0)


def _plan(n, nq, K):
    from vectorragquantization_amd import _native as N
    info = np.zeros(12, np.int64)
    N.check(N.load().vrq_scan_plan(n, 1024, nq, K, 0, info.ctypes.data), "plan")
    return info


def _assert_k1m4(n, nq, K=100):
    info = _plan(n, nq, K)
    assert (int(info[0]), int(info[1])) == (0, 4), "shape does not run K1m MB = 4"
    return info


def _phase1(codes_t, qb, K, dev, row_offset=0):
    """vrq_search3 PHASE1_ONLY with the library's own scan choice -> (count, dist, rows)."""
    from vectorragquantization_amd import _native as N
    from vectorragquantization_amd.enhanced import search3
    nq = qb.shape[0]
    x8 = torch.empty((1, 1024), dtype=torch.int8, device=dev)
    norms = torch.empty((1,), dtype=torch.float64, device=dev)
    qf = torch.zeros((nq, 1024), dtype=torch.float32, device=dev)
    q_t = torch.from_numpy(np.ascontiguousarray(qb)).to(dev)
    cnt, rows, dist, _, _ = search3(codes_t, x8, norms, qf, q_t, K, K, K, N.VRQ_SEARCH_PHASE1_ONLY, row_offset)
    torch.cuda.synchronize()
    return cnt.cpu().numpy(), dist.cpu().numpy(), rows.cpu().numpy()


def _paths(codes_t, qb, K):
    """Which fallback paths a query took: run PREFIX + MATRIX + RECHECK through the stage-split ABI and read
    the per-(query, chunk) list lengths (> capc: overflowed, rescanned exactly by the suffix stage) and the
    per-query re-run flags from the workspace (offsets from vrq_scan_plan).  -> (overflowed[nq], rerun[nq])"""
    from vectorragquantization_amd import _native as N
    lib = N.load()
    n, nq = codes_t.shape[0], qb.shape[0]
    flags = N.VRQ_SEARCH_PHASE1_ONLY
    info = _plan(n, nq, K)
    ws = torch.zeros((int(info[11]),), dtype=torch.uint8, device=codes_t.device)
    q_t = torch.from_numpy(np.ascontiguousarray(qb)).to(codes_t.device)
    st = N.stream_handle(codes_t.device)
    for stage in (N.VRQ_SCAN_STAGE_PREFIX, N.VRQ_SCAN_STAGE_MATRIX, N.VRQ_SCAN_STAGE_RECHECK):
        N.check(lib.vrq_search3_scan(N.ptr(codes_t), n, 1024, N.ptr(q_t), nq, K, flags | stage, N.ptr(ws), ws.numel(),
                                     st), "scan stage")
    torch.cuda.synchronize()
    nch, capc, off_cnt, off_tau = (int(info[i]) for i in (3, 4, 6, 7))
    cnt = ws[off_cnt:off_cnt + 4 * nq * nch].view(torch.int32).view(nq, nch).cpu().numpy()
    qa = (4 * nq + 255) & ~255
    rerun = ws[off_tau + 2 * qa:off_tau + 2 * qa + 4 * nq].view(torch.int32).cpu().numpy()
    return (cnt > capc).any(axis=1), rerun != 0


def _flip(rng, rows, nflip):
    """Copies of `rows` with exactly nflip distinct bits flipped each (vectorised for millions of rows)."""
    m = rows.shape[0]
    out = np.empty((m, 128), np.uint8)                   # C-contiguous (rows may be a broadcast view)
    out[...] = rows
    pos = rng.integers(0, 1024, (m, nflip))
    while True:                                          # distinct positions per row
        s = np.sort(pos, axis=1)
        bad = (np.diff(s, axis=1) == 0).any(axis=1) if nflip > 1 else np.zeros(m, bool)
        if not bad.any():
            break
        pos[bad] = rng.integers(0, 1024, (int(bad.sum()), nflip))
    flat = out.reshape(-1)
    base = np.arange(m, dtype=np.int64) * 128
    for c in range(nflip):                               # one position per row per step: unique indices
        flat[base + (pos[:, c] >> 3)] ^= (0x80 >> (pos[:, c] & 7)).astype(np.uint8)
    return out


def _check(oracle_lib, codes, qb, K, dist, rows, qsel, row_offset=0):
    D0, I0 = oracle_knn(oracle_lib, codes, qb[qsel], K, threads=16)
    assert np.array_equal(D0, dist[qsel])
    assert np.array_equal(I0 + row_offset, rows[qsel])
    return D0, I0


def _sel(planted, nq, extra=48):
    return np.unique(np.concatenate([np.asarray(planted, np.int64),
                                     np.linspace(0, nq - 1, extra).round().astype(np.int64)]))


def test_k1m4_heavy_ties(dev, oracle_lib):
    """Every row is one of 25 codes: every list overflows and every query is rescanned exactly; the
    K-list must be the first rows of each distance in row order (plus a row offset, as a shard has)."""
    rng = np.random.default_rng(11)
    base = rng.integers(0, 256, (25, 128), dtype=np.uint8)
    codes = base[rng.integers(0, 25, N_BIG)]
    qb = np.concatenate([base[:4], _flip(rng, base[4:8], 40),
                         rng.integers(0, 256, (NQ - 8, 128), dtype=np.uint8)])
    _assert_k1m4(N_BIG, NQ)
    codes_t = torch.from_numpy(codes).to(dev)
    ovf, _ = _paths(codes_t, qb, 100)
    assert ovf.all(), "every query's lists must overflow on an all-ties corpus"
    for K in (1, 100, 128):
        c, D1, I1 = _phase1(codes_t, qb, K, dev, row_offset=5_000_000)
        assert np.array_equal(c, np.full(NQ, K))
        _check(oracle_lib, codes, qb, K, D1, I1, _sel(range(8), NQ, 56), row_offset=5_000_000)


def test_k1m4_candidate_overflow_exact_rescan(dev, oracle_lib):
    """400K rows of the corpus sit at distance exactly 3 from query 0 (50 of them exact copies): far
    more rows beat its threshold than its lists hold, so the corpus is rescanned exactly and the answer
    is the 50 copies plus the FIRST 50 dist-3 rows in row order.  Query 2 is a row of that region."""
    rng = np.random.default_rng(9)
    K, R0, R = 100, 1_300_000, 400_000
    codes = rng.integers(0, 256, (N_BIG, 128), dtype=np.uint8)
    qb = rng.integers(0, 256, (NQ, 128), dtype=np.uint8)
    region = _flip(rng, np.broadcast_to(qb[:1], (R, 128)), 3)
    region[rng.choice(R, 50, replace=False)] = qb[0]
    codes[R0:R0 + R] = region
    qb[2] = codes[R0 + 17]
    qb[700] = codes[R0 + R - 5]                            # the second 512-query block too
    _assert_k1m4(N_BIG, NQ, K)
    codes_t = torch.from_numpy(codes).to(dev)
    ovf, _ = _paths(codes_t, qb, K)
    assert ovf[[0, 2, 700]].all() and not ovf[[1, 3]].any()
    c, D1, I1 = _phase1(codes_t, qb, K, dev)
    assert np.array_equal(c, np.full(NQ, K))
    D0, _ = _check(oracle_lib, codes, qb, K, D1, I1, _sel([0, 1, 2, 3, 700], NQ))
    assert (D1[0] == 0).sum() == 50 and (D1[0] == 3).sum() == 50


def test_k1m4_hit_staging_overflow(dev, oracle_lib):
    """A 300K-row region clustered around one code and 138 queries near it (all 128 queries of block 0's
    first wave, and 10 in the second query block): every tile of the region gives those waves thousands
    of hits, more than the per-wave LDS stage holds, so their lists are marked overflowed and rescanned
    exactly while the other queries keep the fast path."""
    rng = np.random.default_rng(17)
    K, R0, R = 100, 2_000_000, 300_000
    base = rng.integers(0, 256, (1, 128), dtype=np.uint8)
    codes = rng.integers(0, 256, (N_BIG, 128), dtype=np.uint8)
    codes[R0:R0 + R] = _flip(rng, np.broadcast_to(base, (R, 128)), 6)
    qb = rng.integers(0, 256, (NQ, 128), dtype=np.uint8)
    planted = np.concatenate([np.arange(128), np.arange(600, 610)])
    qb[planted] = _flip(rng, np.broadcast_to(base, (planted.size, 128)), 4)
    _assert_k1m4(N_BIG, NQ, K)
    codes_t = torch.from_numpy(codes).to(dev)
    ovf, _ = _paths(codes_t, qb, K)
    # (an unplanted query's list may also overflow by chance under its sampled tau_s: exact either way)
    assert ovf[planted].all() and ovf.sum() <= planted.size + 8
    c, D1, I1 = _phase1(codes_t, qb, K, dev)
    assert np.array_equal(c, np.full(NQ, K))
    _check(oracle_lib, codes, qb, K, D1, I1, _sel(planted, NQ))
    assert (I1[planted] >= R0).all() and (I1[planted] < R0 + R).all()


def _sample_rows(n, nq, K):
    """Rows of the dense threshold sample, from the library's own plan (vrq_scan_sample_plan): tile
    i = c * T + t of the sample starts at row i * ts."""
    from vectorragquantization_amd import _native as N
    info = np.zeros(8, np.int64)
    N.check(N.load().vrq_scan_sample_plan(n, 1024, nq, K, 0, info.ctypes.data), "sample plan")
    chunks, crows, ts = int(info[1]), int(info[2]), int(info[4])
    tiles = chunks * (crows // 64)
    return (np.arange(tiles, dtype=np.int64)[:, None] * ts + np.arange(64)[None, :]).reshape(-1)


@pytest.mark.parametrize("nq", [NQ, 1100])
def test_k1m4_sampled_threshold_rerun(dev, oracle_lib, nq):
    """Queries 0 and nq - 10 (different 512-query blocks) get 70 near copies on sample rows and 40 more at
    dist 30 off the sample: tau_s = d'_(j) + 1 falls among the near copies, the check finds fewer than K
    admitted rows, and the query block's re-run with tau_p must recover the first 30 dist-30 rows in
    row order.  1100 queries: a ragged third query block."""
    rng = np.random.default_rng(23 + nq)
    K = 100
    info = _assert_k1m4(N_BIG, nq, K)
    assert int(info[9]) < K, "the plan must take the sampled threshold"
    codes = rng.integers(0, 256, (N_BIG, 128), dtype=np.uint8)
    qb = _flip(rng, codes[rng.integers(0, N_BIG, nq)], 50)
    samp = _sample_rows(N_BIG, nq, K)
    assert samp.max() < N_BIG and np.unique(samp).size == samp.size
    insamp = np.zeros(N_BIG, bool)
    insamp[samp] = True
    planted = [0, nq - 10]
    near_all = rng.choice(samp, 140, replace=False)       # disjoint row sets for the two queries
    far_all = rng.integers(0, N_BIG, 400)
    far_all = rng.permutation(np.unique(far_all[~insamp[far_all]]))[:80]
    assert far_all.size == 80
    for i, q in enumerate(planted):
        near = near_all[70 * i:70 * (i + 1)]
        codes[near] = _flip(rng, np.repeat(qb[q:q + 1], 70, axis=0), int(rng.integers(5, 21)))
        far = far_all[40 * i:40 * (i + 1)]
        codes[far] = _flip(rng, np.repeat(qb[q:q + 1], 40, axis=0), 30)
    codes_t = torch.from_numpy(codes).to(dev)
    _, rerun = _paths(codes_t, qb, K)
    assert rerun[planted].all(), "the planted queries must fail tau_s and re-run with tau_p"
    c, D1, I1 = _phase1(codes_t, qb, K, dev)
    assert np.array_equal(c, np.full(nq, K))
    D0, _ = _check(oracle_lib, codes, qb, K, D1, I1, _sel(planted, nq))
    assert (D1[0] == 30).sum() == 30 and (D1[nq - 10] == 30).sum() == 30


def test_k1m4_cluster_ordered_corpus(dev, oracle_lib):
    """4200 clusters of 1000 contiguous near-copies (32 or 64 flipped bits on average): a query's whole
    neighbourhood sits in one chunk and in few lane rows of the sample (looser tau_s / tau_p).  The result
    must still be exactly the FAISS order."""
    rng = np.random.default_rng(4242)
    ncl, per = 4200, 1000
    centres = rng.integers(0, 256, (ncl, 128), dtype=np.uint8)
    codes = np.empty((N_BIG, 128), np.uint8)
    codes[:ncl * per] = np.repeat(centres, per, axis=0)
    codes[ncl * per:] = rng.integers(0, 256, (N_BIG - ncl * per, 128), dtype=np.uint8)
    m = ncl * per
    flips = rng.integers(0, 256, (m, 128), dtype=np.uint8)
    for _ in range(3):                                    # bit density 1/16
        flips &= rng.integers(0, 256, (m, 128), dtype=np.uint8)
    tight = np.repeat(rng.random(ncl) < 0.5, per)         # half the clusters: density 1/32
    flips[tight] &= rng.integers(0, 256, (int(tight.sum()), 128), dtype=np.uint8)
    codes[:m] ^= flips
    del flips
    qb = _flip(rng, centres[rng.integers(0, ncl, NQ)], 12)
    _assert_k1m4(N_BIG, NQ)
    c, D1, I1 = _phase1(torch.from_numpy(codes).to(dev), qb, 100, dev)
    assert np.array_equal(c, np.full(NQ, 100))
    _check(oracle_lib, codes, qb, 100, D1, I1, _sel([], NQ, 128))
