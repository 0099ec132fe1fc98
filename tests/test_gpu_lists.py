"""GPU checks of the intermediate every matrix-core pass writes: the per-(query, chunk) candidate lists.

The top-K tests only see a wrong list entry if it reaches the top-K, which for a rare corruption
(round 3: a register copied before its LDS read landed gave ~1 in 10^4 K1r candidates a stale-row
distance, and a green GPUTEST) depends on luck.  Here every entry of every list is checked against
the true value, and every list against the exact set of rows it must hold:

* Phase-I scans (hamming_mfma.hip), FAISS semantics of CohereEnhancedVectorDB.py:267-268: after the
  PREFIX + MATRIX (+ RECHECK) stages, list (q, chunk) must be exactly the rows r of the chunk with
  dist(q, r) < tau(q) (tau = the threshold the pass ran with: tau_s, or tau_p for re-run queries), each
  once, with its exact distance in the key.  Every K1r instance (MB = 1, the lean MB = 2, MB = 4) and
  both K1m instances (MB = 2, MB = 4) and K1s, 4M+ uniform rows (ragged: the last tile is partial).
* The dense sample pass (PREFIX): every u16 lane minimum equals min(dist - pc(q)) + 1024 over the
  sample rows that lane holds.
* K5 (gemm_topk.hip, CohereEnhancedVectorDB.py:283-293 / :302-318 scored against every row): after the
  SAMPLE + MAIN stages every (query, chunk) list holds exactly the rows whose matrix-core value passes
  the query's threshold (Phase II: the exact integer rule; Phase III: up to the f32 rounding band of
  u = f32(A) * rcp(f32(norm))), row ids inside their chunk, no duplicates.

True distances come from an exact fp32 GEMM of 0/1 bit matrices (integers <= 1024), true matrix-core
values from an exact float64 GEMM of the int8 pieces: test infrastructure only, no product code.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

KEY_ROW_BITS = 40


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from vectorragquantization_amd import _native
    _native.load()
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.set_float32_matmul_precision("highest")
    return torch.device("cuda", 0)


def _al(x):
    return (x + 255) & ~255


def _bits(c):
    """u8[m, 128] -> f32[m, 1024] 0/1 (np.unpackbits order)."""
    sh = torch.arange(7, -1, -1, device=c.device, dtype=torch.uint8)
    return ((c[:, :, None] >> sh) & 1).reshape(c.shape[0], -1).float()


def _dist(codes, qb, block=1 << 19):
    """Exact Hamming distances i16[nq, n] (pc(q) + pc(r) - 2 <q, r>, all integers in f32)."""
    nq, n = qb.shape[0], codes.shape[0]
    qbits = _bits(qb)
    pcq = qbits.sum(1)
    out = torch.empty((nq, n), dtype=torch.int16, device=codes.device)
    for r0 in range(0, n, block):
        cb = _bits(codes[r0:r0 + block])
        d = pcq[:, None] + cb.sum(1)[None, :] - 2.0 * (qbits @ cb.T)
        out[:, r0:r0 + block] = d.to(torch.int16)
    return out


def _corpus(n, nq, dev, seed):
    from vectorragquantization_amd import synth
    codes = synth.random_codes(n, device=dev, seed=seed)
    qb, _ = synth.flip_queries(codes, nq, seed=seed + 1)
    g = torch.Generator(device=dev)
    g.manual_seed(seed + 2)
    qb[::7] = torch.randint(0, 256, qb[::7].shape, generator=g, device=dev, dtype=torch.uint8)  # some far queries
    return codes, qb


def _scan_stages(codes, qb, K, stages):
    from vectorragquantization_amd import _native as N
    lib = N.load()
    n, nq = codes.shape[0], qb.shape[0]
    flags = N.VRQ_SEARCH_PHASE1_ONLY | N.VRQ_SEARCH_SCAN_MFMA
    info = np.zeros(12, np.int64)
    N.check(lib.vrq_scan_plan(n, 1024, nq, K, flags, info.ctypes.data), "plan")
    ws = torch.zeros((int(info[11]),), dtype=torch.uint8, device=codes.device)
    st = N.stream_handle(codes.device)
    for stage in stages:
        N.check(lib.vrq_search3_scan(N.ptr(codes), n, 1024, N.ptr(qb), nq, K, flags | stage, N.ptr(ws), ws.numel(),
                                     st), "scan stage")
    torch.cuda.synchronize()
    return info, ws


# (nq, instance): K1r MB = 1 (<= 32 queries), the lean MB = 2 (33..64), MB = 4 (65..128); K1m MB = 2
# (129..511); >= 512: K1s (kind 2) up to 2^32 (query, row) pairs per pass, K1m MB = 4 above
SCAN_CASES = [(8, (1, 1)), (40, (1, 2)), (64, (1, 2)), (128, (1, 4)), (256, (0, 2)), (1024, (2, 4)), (1536, (0, 4))]


@pytest.mark.parametrize("nq,inst", SCAN_CASES)
def test_scan_candidate_lists_exact(dev, nq, inst):
    n = 4_194_301
    codes, qb = _corpus(n, nq, dev, 1000 + nq)
    info = check_scan_lists(codes, qb, 100)
    assert (int(info[0]), int(info[1])) == inst


def check_scan_lists(codes, qb, K, allow_overflow=False):
    """PREFIX + MATRIX + RECHECK on (codes, qb) with whatever scan the library plans; every list entry and
    every list checked against the true distances (shared with tools/k1s_check.py).  -> the plan."""
    from vectorragquantization_amd import _native as N
    dev = codes.device
    n, nq = codes.shape[0], qb.shape[0]
    info, ws = _scan_stages(codes, qb, K, (N.VRQ_SCAN_STAGE_PREFIX, N.VRQ_SCAN_STAGE_MATRIX,
                                           N.VRQ_SCAN_STAGE_RECHECK))
    cr, nch, capc, off_cand, off_cnt, off_tau, j = (int(info[i]) for i in (2, 3, 4, 5, 6, 7, 9))
    cnt = ws[off_cnt:off_cnt + 4 * nq * nch].view(torch.int32).view(nq, nch)
    cand = ws[off_cand:off_cand + 8 * nq * nch * capc].view(torch.int64).view(nq, nch, capc)
    qa = _al(4 * nq)
    tau_s = ws[off_tau:off_tau + 4 * nq].view(torch.int32).long()
    tau_p = ws[off_tau + qa:off_tau + qa + 4 * nq].view(torch.int32).long()
    rerun = ws[off_tau + 2 * qa:off_tau + 2 * qa + 4 * nq].view(torch.int32)
    tau = torch.where(rerun != 0, tau_p, tau_s if j < K else tau_p)
    assert (cnt >= 0).all(), "negative list length"
    ovf = (cnt > capc).any(dim=1)
    assert allow_overflow or not ovf.any(), "a list overflowed on uniform data"
    cnt = torch.where(ovf[:, None], torch.zeros_like(cnt), cnt)  # overflowed queries: rescanned, not checked
    D = _dist(codes, qb)
    # every listed entry: in its chunk, its key's distance is the true one, and below the threshold
    live = torch.arange(capc, device=dev)[None, None, :] < cnt[:, :, None]
    qs = torch.arange(nq, device=dev)[:, None, None].expand(nq, nch, capc)[live]
    chs = torch.arange(nch, device=dev)[None, :, None].expand(nq, nch, capc)[live]
    keys = cand[live]
    rows = keys & ((1 << KEY_ROW_BITS) - 1)
    assert ((rows >= chs * cr) & (rows < torch.clamp(chs * cr + cr, max=n))).all(), "row outside its chunk"
    d_gpu = (keys >> KEY_ROW_BITS) - 1025 + tau[qs]
    d_true = D[qs, rows].long()
    bad = torch.nonzero(d_gpu != d_true).flatten()
    assert bad.numel() == 0, (f"{bad.numel()} of {keys.numel()} listed distances wrong; first: q {int(qs[bad[0]])} "
                              f"row {int(rows[bad[0]])} gpu {int(d_gpu[bad[0]])} true {int(d_true[bad[0]])}")
    assert (d_true < tau[qs]).all()
    # every list complete: the listed (q, row) set is exactly {dist < tau}, each row once
    listed = torch.sort(qs * n + rows).values
    want = []
    for q0 in range(0, nq, 128):  # (torch.nonzero of > 2^31 elements fails: query blocks)
        below = D[q0:q0 + 128] < tau[q0:q0 + 128, None].to(torch.int16)
        below &= ~ovf[q0:q0 + 128, None]
        tq, tr = torch.nonzero(below, as_tuple=True)
        want.append((tq + q0) * n + tr)
    want = torch.cat(want)
    assert torch.equal(listed, want), f"{listed.numel()} listed vs {want.numel()} rows below the thresholds"
    # the recheck's guarantee: tau_s admitted >= K rows, or the query re-ran with tau_p
    assert ((cnt.sum(1) >= K) | ovf).all()
    return info


@pytest.mark.parametrize("nq", [8, 64, 128, 1024])
def test_scan_sample_lane_minima_exact(dev, nq):
    """Every lane minimum of the dense sample pass (K1r's own for <= 64 queries, K1m's MB = 2 instance
    above) equals the minimum of dist - pc(q) over the sample rows of that lane."""
    from vectorragquantization_amd import _native as N
    lib = N.load()
    n, K = 4_194_301, 100
    codes, qb = _corpus(n, nq, dev, 2000 + nq)
    flags = N.VRQ_SEARCH_PHASE1_ONLY | N.VRQ_SEARCH_SCAN_MFMA
    sp = np.zeros(6, np.int64)
    N.check(lib.vrq_scan_sample_plan(n, 1024, nq, K, flags, sp.ctypes.data), "sample plan")
    rows_sample, nsc, scr, sstride, ts, cols = (int(x) for x in sp)
    assert rows_sample == (1 if nq <= 64 else 0)
    assert sstride == (scr // 64) * ts and cols == 32 * nsc
    _, ws = _scan_stages(codes, qb, K, (N.VRQ_SCAN_STAGE_PREFIX,))
    dv = ws[:2 * nq * cols].view(torch.int16).view(nq, cols).int() & 0xFFFF
    T = scr // 64
    srows = (torch.arange(nsc * T, device=dev)[:, None] * ts + torch.arange(64, device=dev)[None, :]).reshape(-1)
    assert int(srows.max()) < n
    D = _dist(codes[srows], qb)                                          # [nq, nsc * T * 64]
    pcq = _bits(qb).sum(1).int()
    want = D.view(nq, nsc, T, 2, 32).amin(dim=(2, 3)).int() - pcq[:, None, None] + 1024
    assert torch.equal(dv, want.view(nq, cols))


def _ph2_perm():
    """Natural dim of each Phase-II fragment position within a 32-dim k-step (gemm_topk.hip ph2_pos)."""
    pos = []
    for d in range(32):
        b, x = d >> 3, 7 - (d & 7)
        pos.append((x >> 2) * 16 + 4 * (x & 3) + b)
    return np.array([s * 32 + pos[d] for s in range(32) for d in range(32)])


@pytest.mark.parametrize("mode", ["binary", "int8_cosine"])
def test_gemm_main_pass_lists_exact(dev, mode):
    """K5's thresholded pass: every (query, chunk) list holds exactly the rows of its chunk whose
    matrix-core value u passes the query's threshold (each once, ids in range); two query blocks plus
    padding, a ragged corpus of the SURVEY 8(d) generator."""
    from vectorragquantization_amd import _native as N
    from vectorragquantization_amd import synth
    from vectorragquantization_amd.enhanced import gemm_topk
    lib = N.load()
    n, nq, k = 2_000_003, 300, 10
    m = {"binary": N.VRQ_GEMM_BINARY, "int8_cosine": N.VRQ_GEMM_INT8_COSINE}[mode]
    sh = synth.make_corpus(n, device=dev)
    qf, _, _ = synth.make_queries(n, nq, device=dev)
    codes, x8, norms = sh["codes"], sh["x8"], sh["norms"]
    plan, lay = np.zeros(8, np.int64), np.zeros(8, np.int64)
    N.check(lib.vrq_gemm_topk_plan(m, n, 1024, nq, k, plan.ctypes.data), "plan")
    N.check(lib.vrq_gemm_topk_layout(m, n, 1024, nq, k, lay.ctypes.data), "layout")
    cr, nch, capc, ws_bytes = int(plan[0]), int(plan[1]), int(plan[2]), int(plan[6])
    nq_pad, off_thr, off_cnt, off_cand = (int(x) for x in lay[:4])
    ws = torch.zeros((ws_bytes,), dtype=torch.uint8, device=dev)
    for st in (N.VRQ_GEMM_STAGE_SAMPLE, N.VRQ_GEMM_STAGE_MAIN):
        gemm_topk(mode, qf, k, codes=codes, x8=x8, norms=norms, flags=st, workspace=ws)
    torch.cuda.synchronize()
    thr = ws[off_thr:off_thr + 4 * nq].view(torch.float32).double()
    cnt = ws[off_cnt:off_cnt + 4 * nq * nch].view(torch.int32).view(nq, nch)
    cand = ws[off_cand:off_cand + 4 * nq * nch * capc].view(torch.int32).view(nq, nch, capc).long() & 0xFFFFFFFF
    assert (cnt >= 0).all() and (cnt <= capc).all(), "a list overflowed"
    a = ws[:nq_pad * 1024].view(torch.int8).view(nq_pad, 1024)[:nq]
    if m == N.VRQ_GEMM_BINARY:
        a = a[:, torch.from_numpy(_ph2_perm()).to(dev)]
    a = a.double()
    live = torch.arange(capc, device=dev)[None, None, :] < cnt[:, :, None]
    qs = torch.arange(nq, device=dev)[:, None, None].expand(nq, nch, capc)[live]
    chs = torch.arange(nch, device=dev)[None, :, None].expand(nq, nch, capc)[live]
    rows = cand[live]
    assert ((rows >= chs * cr) & (rows < torch.clamp(chs * cr + cr, max=n))).all(), "row outside its chunk"
    listed = torch.sort(qs * n + rows).values
    assert torch.equal(listed, torch.unique(listed)), "a row listed twice"
    must, may = [], []
    for r0 in range(0, n, 1 << 19):
        r1 = min(n, r0 + (1 << 19))
        if m == N.VRQ_GEMM_BINARY:
            A = a @ _bits(codes[r0:r1]).double().T                      # exact integers
            ok = A >= torch.ceil(thr)[:, None]
            must.append(ok)
            may.append(ok)
        else:
            A = a @ x8[r0:r1].double().T                                # exact integers (|A| < 2^24)
            u = A / norms[r0:r1][None, :]                               # zero norm -> +-inf/NaN: never listed
            band = 2.0 ** -20 * u.abs() + 1e-30
            fin = norms[r0:r1][None, :] > 0
            must.append(fin & (u >= thr[:, None] + band))
            may.append(fin & (u >= thr[:, None] - band))
    must, may = torch.cat(must, 1), torch.cat(may, 1)
    in_list = torch.zeros((nq, n), dtype=torch.bool, device=dev)
    in_list[qs, rows] = True
    missing = must & ~in_list
    assert not missing.any(), f"{int(missing.sum())} rows passing the threshold are missing from the lists"
    spurious = in_list & ~may
    assert not spurious.any(), f"{int(spurious.sum())} listed rows fail the threshold"
    assert int(must.sum(1).min()) >= k
