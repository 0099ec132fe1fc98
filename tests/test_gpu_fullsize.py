"""BASELINE configs 3 and 5 checked at their full benchmark shapes (not only at test sizes).

* Config 3 -- Phase I only over 100M uniform random 1024-bit codes (CohereEnhancedVectorDB.py:267-268,
  north_star target "top-10 ids identical to the CPU reference at N = 100M"): the matrix-core
  small-batch scan (K1r) at nq = 1, 8 and 64, K = 100, against the C restatement of FAISS
  hammings_knn_hc over every row.  Every (dist, row) of the top-K must be identical.
* Config 2 -- the 3-phase search over 1M rows with the full nq = 1024 batch, i.e. the MB = 4 instance
  of the large-batch matrix-core scan (K1s) the config-2 bench runs: 32 sampled queries against the
  FAISS restatement (Phase I, every (dist, row) of the top-K) and the reference Phases II/III
  (CohereEnhancedVectorDB.py:267-322).
* Config 5 -- exhaustive Phase-II / Phase-III top-k over 10M x 1024 rows, nq = 1024 (four 256-query
  blocks per chunk, the retry path at scale), with the exact fallback OFF (VRQ_GEMM_NO_FALLBACK):
  a sample of 16 queries against the reference scores of EVERY row, computed in float64 on the GPU
  with torch as the checker (CohereEnhancedVectorDB.py:283-293 and :302-318).
"""
import ctypes

import numpy as np
import pytest
import torch

from tests.conftest import oracle_knn

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from vectorragquantization_amd import _native
    _native.load()
    return torch.device("cuda", 0)


@pytest.mark.timeout(300)
def test_config3_100m_phase1_identical_to_cpu_reference(dev, oracle_lib):
    from vectorragquantization_amd import _native as N
    from vectorragquantization_amd import synth
    from vectorragquantization_amd.enhanced import search3
    n, K = 100_000_000, 100
    codes = synth.random_codes(n, device=dev)
    qb64, _ = synth.flip_queries(codes, 64)
    lib = N.load()
    got = {}
    for nq in (1, 8, 64):
        pre = ctypes.c_int64(-1)
        kind = lib.vrq_scan_kind(n, 1024, nq, K, N.VRQ_SEARCH_PHASE1_ONLY, ctypes.byref(pre))
        assert kind == N.VRQ_SCAN_KIND_MFMA and pre.value == 0, (nq, kind)  # the K1r matrix-core scan
        qb = qb64[:nq].contiguous()
        qf = torch.zeros((nq, 1024), dtype=torch.float32, device=dev)
        x8 = torch.empty((1, 1024), dtype=torch.int8, device=dev)
        nrm = torch.empty((1,), dtype=torch.float64, device=dev)
        cnt, rows, d, _, _ = search3(codes, x8, nrm, qf, qb, 10, K, 30, N.VRQ_SEARCH_PHASE1_ONLY)
        got[nq] = (cnt.cpu().numpy(), rows.cpu().numpy(), d.cpu().numpy())
    codes_h = codes.cpu().numpy()
    del codes
    torch.cuda.empty_cache()
    D, I = oracle_knn(oracle_lib, codes_h, qb64.cpu().numpy(), K, threads=16)
    del codes_h
    for nq, (cnt, rows, d) in got.items():
        assert (cnt == K).all(), nq
        assert np.array_equal(d, D[:nq]), f"nq={nq}: Hamming distances differ from the CPU reference"
        assert np.array_equal(rows, I[:nq]), f"nq={nq}: rows differ from the CPU reference"
        assert np.array_equal(rows[:, :10], I[:nq, :10])


def _exact_scores(mode, q64, codes, x8, norms, chunk=1 << 19):
    """Reference scores of every row for the sampled queries, float64 on the GPU (checker):
    Phase II  q . (2*unpackbits(code) - 1) summed in float64;
    Phase III float32(q . int8) / ||int8||_2, -inf for a zero norm."""
    n = codes.shape[0]
    out = torch.empty((q64.shape[0], n), dtype=torch.float64, device=q64.device)
    sh = torch.arange(7, -1, -1, device=q64.device, dtype=torch.uint8)
    for a in range(0, n, chunk):
        b = min(n, a + chunk)
        if mode == "binary":
            bits = ((codes[a:b, :, None] >> sh) & 1).reshape(b - a, 1024).to(torch.float64)
            out[:, a:b] = q64 @ (2.0 * bits - 1.0).T
        else:
            dot = (q64 @ x8[a:b].to(torch.float64).T).to(torch.float32).to(torch.float64)
            nr = norms[a:b]
            out[:, a:b] = torch.where(nr == 0, torch.full_like(dot, -float("inf")), dot / nr)
    return out


@pytest.mark.timeout(300)
def test_config5_full_shape_vs_exact_scores(dev):
    from vectorragquantization_amd import _native as N
    from vectorragquantization_amd import synth
    from vectorragquantization_amd.enhanced import gemm_topk
    n, nq, k = 10_000_000, 1024, 10
    sh = synth.make_corpus(n, device=dev)
    codes, x8, norms = sh["codes"], sh["x8"], sh["norms"]
    qf, _, _ = synth.make_queries(n, nq, device=dev)
    sample = torch.arange(5, nq, nq // 16, device=dev)[:16]  # spread over the four query blocks
    q64 = qf[sample].to(torch.float64)
    for mode in ("binary", "int8_cosine"):
        cnt, rows, sc = gemm_topk(mode, qf, k, codes=codes, x8=x8, norms=norms, flags=N.VRQ_GEMM_NO_FALLBACK)
        assert bool((cnt == k).all()), mode
        S = _exact_scores(mode, q64, codes, x8, norms)
        r, s = rows[sample], sc[sample]
        got = torch.gather(S, 1, r)
        # each returned score is its row's reference score: Phase III bit-exact; Phase II equal up to
        # the float64 summation order of the checker's GEMM (0 or 1 ulp)
        tol = torch.abs(got) * 2.0 ** -52 if mode == "binary" else torch.zeros_like(got)
        assert bool((torch.abs(s - got) <= tol).all()), mode
        # the reference order: the k largest scores, ties by row ascending (stable sort over rows)
        kth = torch.topk(S, k, dim=1).values[:, -1:]
        for i in range(sample.shape[0]):
            cand = torch.nonzero(S[i] >= kth[i] - (abs(float(kth[i])) * 2.0 ** -50)).flatten()
            cs = S[i, cand]
            o = sorted(range(cand.shape[0]), key=lambda j: (-float(cs[j]), int(cand[j])))[:k]
            ref_rows = cand[o]
            if not torch.equal(ref_rows, r[i]):
                # only certified near-ties (within the checker's summation slack) may swap
                diff = torch.nonzero(ref_rows != r[i]).flatten()
                gap = torch.abs(S[i, ref_rows[diff]] - S[i, r[i][diff]])
                assert bool((gap <= torch.abs(S[i, ref_rows[diff]]) * 2.0 ** -50).all()), (mode, i)
        del S
    del sh, codes, x8, norms
    torch.cuda.empty_cache()


@pytest.mark.timeout(300)
def test_config2_1m_batch_1024_vs_reference(dev, oracle_lib):
    from oracle import oracle_np as O
    from tests.test_gpu_parity import MAX_TIE_FRAC, _certify
    from vectorragquantization_amd import _native as N
    from vectorragquantization_amd import synth
    from vectorragquantization_amd.enhanced import search3
    n, nq, k, K, K3 = 1_000_000, 1024, 10, 100, 30
    lib = N.load()
    info = np.zeros(12, np.int64)
    N.check(lib.vrq_scan_plan(n, 1024, nq, K, 0, info.ctypes.data), "plan")
    assert int(info[0]) == 2 and int(info[1]) == 4, info[:2]  # K1s, 512-query blocks
    sh = synth.make_corpus(n, device=dev)
    codes, x8, norms = sh["codes"], sh["x8"], sh["norms"]
    qf, qb, _ = synth.make_queries(n, nq, device=dev)
    cnt, rows, dist, s2, s3 = (t.cpu().numpy() for t in search3(codes, x8, norms, qf, qb, k, K, K3, 0))
    c1, r1, d1, _, _ = (t.cpu().numpy() for t in search3(codes, x8, norms, qf, qb, k, K, K3,
                                                          N.VRQ_SEARCH_PHASE1_ONLY))
    torch.cuda.synchronize()
    sample = np.arange(3, nq, nq // 32)[:32]                 # spread over the four 256-query blocks
    codes_h, x8_h = codes.cpu().numpy(), x8.cpu().numpy()
    qf_h, qb_h = qf.cpu().numpy()[sample], qb.cpu().numpy()[sample]
    D, I = oracle_knn(oracle_lib, codes_h, qb_h, K, threads=16)
    assert (c1[sample] == K).all()
    assert np.array_equal(d1[sample], D) and np.array_equal(r1[sample], I)
    ref = O.three_phase_batch(codes_h, x8_h, np.arange(n, dtype=np.int64), qf_h, qb_h, k, K // k, K3 // k,
                              phase1=(D, I))
    ties = 0
    for j, q in enumerate(sample.tolist()):
        assert int(cnt[q]) == k
        same = _certify(qf_h[j], qb_h[j], codes_h, x8_h, rows[q], dist[q], s2[q], s3[q], ref[j]["row"])
        if same:
            assert np.array_equal(s2[q], ref[j]["binary"])
        ties += not same
    assert ties <= MAX_TIE_FRAC * len(sample) + 1
