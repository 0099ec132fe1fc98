"""GPU parity of the exhaustive matrix-core Phase-II / Phase-III top-k (vrq_gemm_topk, BASELINE
config 5) against the oracle's reference scores over every row (oracle.exhaustive_scores).

Phase II is bit-exact (rows, order and float64 scores).  Phase III scores are the correctly
rounded float32 dot over the float64 norm (the fused search's definition): checked bit-exact
against that restatement, the rows and order exactly.  Edge cases: duplicate rows (exact ties),
zero-norm rows (-inf), a zero query (everything tied -> exact fallback), n < k, row_offset, query
padding, and the stage split."""
import numpy as np
import pytest
import torch

from oracle import oracle_np as O

pytestmark = pytest.mark.gpu

NOFB = 128  # VRQ_GEMM_NO_FALLBACK: an unserved query is an error (the matrix path alone must serve the batch)


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from vectorragquantization_amd import _native
    _native.load()
    return torch.device("cuda", 0)


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _corpus(rng, n, nclus=64):
    C = rng.standard_normal((nclus, 1024)) / 32.0
    F = C[rng.integers(0, nclus, n)] + (0.6 / 32.0) * rng.standard_normal((n, 1024))
    F = (F / np.linalg.norm(F, axis=1, keepdims=True)).astype(np.float32)
    return F


def _queries(rng, F, nq):
    qf = F[rng.integers(0, F.shape[0], nq)] + (0.3 / 32.0) * rng.standard_normal((nq, 1024))
    return (qf / np.linalg.norm(qf, axis=1, keepdims=True)).astype(np.float32)


def _run(mode, qf, k, dev, codes=None, x8=None, row_offset=0, flags=0, lib=None):
    from vectorragquantization_amd.enhanced import gemm_topk
    from vectorragquantization_amd.quant import int8_row_norms
    c_t = _t(codes, dev) if codes is not None else None
    x_t = _t(x8, dev) if x8 is not None else None
    nrm = int8_row_norms(x_t) if x_t is not None else None
    cnt, rows, sc = gemm_topk(mode, _t(qf, dev), k, codes=c_t, x8=x_t, norms=nrm, row_offset=row_offset, flags=flags,
                              lib=lib)
    torch.cuda.synchronize()
    return cnt.cpu().numpy(), rows.cpu().numpy(), sc.cpu().numpy()


def _check(mode, qf, k, cnt, rows, sc, codes=None, x8=None, row_offset=0):
    S = O.exhaustive_scores(mode, qf, codes=codes, x8=x8)
    ref = O.exhaustive_topk(S, k)
    n = S.shape[1]
    for q in range(qf.shape[0]):
        m = min(k, n)
        assert cnt[q] == m
        assert np.array_equal(rows[q, :m] - row_offset, ref[q]), (mode, q)
        assert np.array_equal(sc[q, :m], S[q, ref[q]]), (mode, q)
        assert np.all(rows[q, m:] == -1)


@pytest.mark.parametrize("mode", ["binary", "int8_cosine"])
def test_gemm_topk_vs_oracle(dev, mode):
    rng = np.random.default_rng(5)
    n, nq, k = 70_000, 200, 10                    # > the 32768-row sample; two query blocks + padding
    F = _corpus(rng, n)
    F[4000] = F[123]                              # exact duplicates -> tied scores, row order decides
    F[61000] = F[123]
    codes, x8, _ = O.encode_batch("cohere", F, 0.1)
    qf = _queries(rng, F, nq)
    qf[7] = F[123]                                # a query whose top rows are the tied duplicates
    cnt, rows, sc = _run(mode, qf, k, dev, codes=codes, x8=x8, row_offset=1000, flags=NOFB)  # matrix path alone
    _check(mode, qf, k, cnt, rows, sc, codes=codes, x8=x8, row_offset=1000)


@pytest.mark.parametrize("k", [1, 100])
def test_gemm_topk_k_range(dev, k):
    rng = np.random.default_rng(11 + k)
    n, nq = 40_000, 130
    F = _corpus(rng, n, 16)
    codes, x8, _ = O.encode_batch("cohere", F, 0.1)
    qf = _queries(rng, F, nq)
    for mode in ("binary", "int8_cosine"):
        cnt, rows, sc = _run(mode, qf, k, dev, codes=codes, x8=x8, flags=NOFB)
        _check(mode, qf, k, cnt, rows, sc, codes=codes, x8=x8)


def test_gemm_topk_edge_cases(dev):
    """zero-norm rows (-inf, they fill the top-k only when too few finite rows exist), a zero query
    (every score tied -> exact fallback, lowest rows first), n < k, odd sizes."""
    rng = np.random.default_rng(2)
    n, nq, k = 1000, 5, 10
    F = _corpus(rng, n, 8)
    codes, x8, _ = O.encode_batch("cohere", F, 0.1)
    x8[10:20] = 0                                  # zero-norm rows
    qf = _queries(rng, F, nq)
    qf[1] = 0.0                                    # zero query
    for mode in ("binary", "int8_cosine"):
        cnt, rows, sc = _run(mode, qf, k, dev, codes=codes, x8=x8)
        _check(mode, qf, k, cnt, rows, sc, codes=codes, x8=x8)
    # n < k, and a corpus whose rows are mostly zero-norm (-inf results in row order)
    small = x8[:7].copy()
    small[2:6] = 0
    cnt, rows, sc = _run("int8_cosine", qf, k, dev, x8=small)
    _check("int8_cosine", qf, k, cnt, rows, sc, x8=small)
    cnt, rows, sc = _run("binary", qf, k, dev, codes=codes[:3])
    _check("binary", qf, k, cnt, rows, sc, codes=codes[:3])


@pytest.mark.parametrize("nq", [3, 300])
def test_gemm_topk_all_identical_rows(dev, nq):
    """Every row identical: all scores tie, the sampled threshold admits every row -> list overflow
    -> exact fallback, which must return rows 0..k-1.  nq = 300 floods the thresholded pass with a
    whole 256-query block plus a partial one: every (query, row) of every tile is a hit, so the hit
    stage, the per-chunk list counters and the list appends all run at their capacity bounds."""
    rng = np.random.default_rng(9)
    n, k = 50_000, 10
    F = np.repeat(_corpus(rng, 1), n, axis=0)
    codes, x8, _ = O.encode_batch("cohere", F, 0.1)
    qf = _queries(rng, _corpus(rng, 100), nq)
    for mode in ("binary", "int8_cosine"):
        cnt, rows, sc = _run(mode, qf, k, dev, codes=codes, x8=x8)
        assert np.array_equal(rows, np.tile(np.arange(k), (nq, 1))), mode
        _check(mode, qf, k, cnt, rows, sc, codes=codes, x8=x8)


def test_gemm_topk_stage_split(dev):
    from vectorragquantization_amd import _native as N
    from vectorragquantization_amd.enhanced import gemm_topk
    from vectorragquantization_amd.quant import int8_row_norms
    rng = np.random.default_rng(3)
    n, nq, k = 80_000, 64, 10
    F = _corpus(rng, n)
    _, x8, _ = O.encode_batch("cohere", F, 0.1)
    qf = _queries(rng, F, nq)
    x_t, q_t = _t(x8, dev), _t(qf, dev)
    nrm = int8_row_norms(x_t)
    full = gemm_topk("int8_cosine", q_t, k, x8=x_t, norms=nrm)
    ws = torch.empty((N.load().vrq_gemm_topk_workspace_size(3, n, 1024, nq, k),), dtype=torch.uint8, device=dev)
    for st in (N.VRQ_GEMM_STAGE_SAMPLE, N.VRQ_GEMM_STAGE_MAIN, N.VRQ_GEMM_STAGE_FINISH):
        part = gemm_topk("int8_cosine", q_t, k, x8=x_t, norms=nrm, flags=st, workspace=ws)
    torch.cuda.synchronize()
    for a, b in zip(full, part):
        assert torch.equal(a, b)


def test_gemm_topk_many_candidates(dev):
    """k = 1000 leaves more than one finish batch (1024 rows) of candidates per query: the finish
    kernel's running top-k walks them in several batches (checked on the lists the MAIN stage leaves);
    the fallback stays off."""
    from vectorragquantization_amd import _native as N
    from vectorragquantization_amd.enhanced import gemm_topk
    from vectorragquantization_amd.quant import int8_row_norms
    lib = N.load()
    rng = np.random.default_rng(17)
    n, nq, k = 200_000, 40, 1000
    F = _corpus(rng, n, 32)
    codes, x8, _ = O.encode_batch("cohere", F, 0.1)
    qf = _queries(rng, F, nq)
    c_t, x_t, q_t = _t(codes, dev), _t(x8, dev), _t(qf, dev)
    nrm = int8_row_norms(x_t)
    for mode in ("binary", "int8_cosine"):
        m = {"binary": N.VRQ_GEMM_BINARY, "int8_cosine": N.VRQ_GEMM_INT8_COSINE}[mode]
        plan, lay = np.zeros(8, np.int64), np.zeros(8, np.int64)
        N.check(lib.vrq_gemm_topk_plan(m, n, 1024, nq, k, plan.ctypes.data), "plan")
        N.check(lib.vrq_gemm_topk_layout(m, n, 1024, nq, k, lay.ctypes.data), "layout")
        nch, capc, off_cnt = int(plan[1]), int(plan[2]), int(lay[2])
        ws = torch.zeros((int(plan[6]),), dtype=torch.uint8, device=dev)
        for st in (N.VRQ_GEMM_STAGE_SAMPLE, N.VRQ_GEMM_STAGE_MAIN):
            gemm_topk(mode, q_t, k, codes=c_t, x8=x_t, norms=nrm, flags=st, workspace=ws)
        torch.cuda.synchronize()
        cnt = ws[off_cnt:off_cnt + 4 * nq * nch].view(torch.int32).view(nq, nch)
        assert int(cnt.clamp(max=capc).sum(1).min()) > 1024, mode
        cnt_, rows, sc = _run(mode, qf, k, dev, codes=codes, x8=x8, flags=NOFB)
        _check(mode, qf, k, cnt_, rows, sc, codes=codes, x8=x8)
