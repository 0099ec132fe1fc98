"""Multi-rank path on CPU (gloo, world_size 2): shard plan, candidate packing, the single
all-gather collective, and -- with the CPU oracle standing in for the per-shard kernels
(test infrastructure) -- that the merged result equals the single-index reference.  The
GPU merge kernel itself (vrq_merge_shards) is checked against the single-GPU search in
tests/test_gpu_parity.py::test_shard_mode_and_merge_equal_single_index."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle_np as O
from vectorragquantization_amd import synth
from vectorragquantization_amd.dist import gather_candidates, pack_candidates, unpack_candidates


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _corpus():
    rng = np.random.default_rng(123)
    n, nq = 4000, 12
    F = rng.standard_normal((n, 1024)).astype(np.float32) * 0.03
    F[2100:2200] = F[0:100]                                  # duplicates across the two shards
    codes, x8, _ = O.encode_batch("cohere", F, 0.1)
    qf = (F[rng.integers(0, n, nq)] + 0.01 * rng.standard_normal((nq, 1024))).astype(np.float32)
    qb, _, _ = O.encode_batch("cohere", qf, 0.1)
    return codes, x8, qf, qb


def _shard_candidates(codes, x8, qf, qb, r0, r1, K):
    """Oracle stand-in for vrq_search3(..., VRQ_SEARCH_SHARD): this shard's exact top-K by
    (dist, global row) with Phase-II / Phase-III scores."""
    nq = qf.shape[0]
    cnt = np.zeros(nq, np.int32)
    rows = np.full((nq, K), -1, np.int64)
    d = np.full((nq, K), np.iinfo(np.int32).max, np.int32)
    s2 = np.full((nq, K), np.nan)
    s3 = np.full((nq, K), np.nan)
    D, I = O.binary_flat_search(codes[r0:r1], qb, K)
    norms = O.int8_row_norms(x8)
    for q in range(nq):
        m = int((I[q] >= 0).sum())
        cnt[q] = m
        for j in range(m):
            r = int(I[q, j]) + r0
            rows[q, j], d[q, j] = r, D[q, j]
            s2[q, j] = float(qf[q].dot(2 * np.unpackbits(codes[r]).astype(np.int32) - 1))
            s3[q, j] = -np.inf if norms[r] == 0 else float(qf[q].dot(x8[r])) / norms[r]
    return cnt, rows, d, s2, s3


def _merge_oracle(gc, gr, gd, g2, g3, k, K3):
    """Host restatement of vrq_merge_shards: top-K by (dist, row) -> stable s2 -> K3 -> stable s3 -> k."""
    S, nq, K = gr.shape
    out = []
    for q in range(nq):
        c = [(int(gd[s, q, p]), int(gr[s, q, p]), g2[s, q, p], g3[s, q, p])
             for s in range(S) for p in range(int(gc[s, q]))]
        c.sort(key=lambda t: (t[0], t[1]))
        c = c[:K]
        c = sorted(c, key=lambda t: -t[2])[:K3]
        c = sorted(c, key=lambda t: -t[3])[:k]
        out.append([t[1] for t in c])
    return out


def _worker(rank, world, port, result_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    codes, x8, qf, qb = _corpus()
    n, k, osb, osi = codes.shape[0], 10, 10, 3
    K = min(k * osb, n)
    r0, r1 = synth.shard_range(n, rank, world)
    cnt, rows, d, s2, s3 = _shard_candidates(codes, x8, qf, qb, r0, r1, K)
    ids = np.where(rows >= 0, rows + 7, -1)                       # external id = row + 7
    t = [torch.from_numpy(a) for a in (cnt, rows, ids, d, s2, s3)]
    buf = gather_candidates(pack_candidates(*t))                   # one collective
    gc, gr, gi, gd, g2, g3 = (x.numpy() for x in unpack_candidates(buf, world, qf.shape[0], K))
    merged = _merge_oracle(gc, gr, gd, g2, g3, k, k * osi)
    if rank == 0:
        ref = O.three_phase_batch(codes, x8, np.arange(n) + 7, qf, qb, k, osb, osi)
        ok = all(merged[q] == ref[q]["row"].tolist() for q in range(qf.shape[0]))
        # ids travel with their rows through the gather
        ok &= bool(np.all((gi[gr >= 0] == gr[gr >= 0] + 7)))
        result_q.put(ok)
    dist.barrier()
    dist.destroy_process_group()


def test_shard_ranges_cover_and_align():
    for n in (1, 63, 64, 1000, 1_000_000, 100_000_000):
        for world in (1, 2, 4, 8):
            rs = [synth.shard_range(n, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
            cs = synth.chunk_grid(n)
            assert all(a % cs == 0 or a == n for a, _ in rs)


def test_pack_unpack_roundtrip():
    nq, K, S = 5, 7, 3
    parts = []
    for s in range(S):
        g = torch.Generator().manual_seed(s)
        parts.append((torch.randint(0, K, (nq,), dtype=torch.int32, generator=g),
                      torch.randint(0, 1 << 40, (nq, K), generator=g),
                      torch.randint(0, 1 << 40, (nq, K), generator=g),
                      torch.randint(0, 1025, (nq, K), dtype=torch.int32, generator=g),
                      torch.randn((nq, K), dtype=torch.float64, generator=g),
                      torch.randn((nq, K), dtype=torch.float64, generator=g)))
    buf = torch.cat([pack_candidates(*p) for p in parts])
    out = unpack_candidates(buf, S, nq, K)
    for s in range(S):
        c, r, i, d, a, b = parts[s]
        assert torch.equal(out[0][s], c) and torch.equal(out[1][s], r) and torch.equal(out[2][s], i)
        assert torch.equal(out[3][s], d) and torch.equal(out[4][s], a) and torch.equal(out[5][s], b)


@pytest.mark.timeout(300)
def test_two_rank_gloo_sharded_search_equals_single_index():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    assert all(p.exitcode == 0 for p in procs)
    assert q.get(timeout=5) is True


def _worker_c5(rank, world, port, result_q):
    """Config 5 over 2 ranks: per-shard exact top-k (oracle stand-in for vrq_gemm_topk with the
    shard's row_offset), ONE all-gather, merge_topk_shards == the single-corpus top-k."""
    from vectorragquantization_amd.dist import gather_topk, merge_topk_shards
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    codes, x8, qf, _ = _corpus()
    x8 = x8.copy()
    x8[3000:3010] = 0                                   # zero-norm rows in shard 1
    qf = qf.copy()
    qf[0] = 0.0                                         # every score tied: row order decides
    n, k = codes.shape[0], 10
    r0, r1 = synth.shard_range(n, rank, world)
    ok = True
    for mode in ("binary", "int8_cosine"):
        for kk in (k, 3000):                            # 3000 > shard rows: -1 / NaN padding
            S = O.exhaustive_scores(mode, qf, codes=codes[r0:r1], x8=x8[r0:r1])
            top = O.exhaustive_topk(S, kk)
            rows = np.full((qf.shape[0], kk), -1, np.int64)
            sc = np.full((qf.shape[0], kk), np.nan)
            m = top.shape[1]
            rows[:, :m] = top + r0
            sc[:, :m] = np.take_along_axis(S, top, 1)
            gr, gs = gather_topk(torch.from_numpy(rows), torch.from_numpy(sc))
            cnt, mr, ms = (t.numpy() for t in merge_topk_shards(gr, gs, kk))
            if rank == 0:
                Sf = O.exhaustive_scores(mode, qf, codes=codes, x8=x8)
                ref = O.exhaustive_topk(Sf, kk)
                mm = ref.shape[1]
                ok &= bool(np.all(cnt == mm))
                ok &= np.array_equal(mr[:, :mm], ref)
                ok &= np.array_equal(ms[:, :mm], np.take_along_axis(Sf, ref, 1))
                ok &= bool(np.all(mr[:, mm:] == -1))
    if rank == 0:
        result_q.put(bool(ok))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_gloo_config5_topk_merge_equals_single_corpus():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_c5, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    assert all(p.exitcode == 0 for p in procs)
    assert q.get(timeout=5) is True


def _worker_c5_identity(rank, world, port, result_q):
    """bench.py's config-5 N > 1 identity check (c5_identity with row0/world/rank): each rank scores its
    shard with the oracle, rank 0 merges by (score desc, row asc) and compares `out` -- here the
    oracle's whole-corpus top-k (must be identical) and a copy with two ranks of one list swapped
    (must not)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    rng = np.random.default_rng(5)
    n, nq, k = 3000, 8, 10
    codes = rng.integers(0, 256, (n, 128), dtype=np.uint8)
    x8 = rng.integers(-127, 128, (n, 1024), dtype=np.int8)
    codes[1600:1700], x8[1600:1700] = codes[0:100], x8[0:100]  # exact ties across the shard boundary
    qf = (rng.standard_normal((nq, 1024)) * 0.03).astype(np.float32)
    qsel = (1, 5)
    out = {}
    for mode, m in (("binary", 2), ("int8_cosine", 3)):
        S = O.exhaustive_scores(mode, qf, codes=codes, x8=x8)
        top = O.exhaustive_topk(S, k)
        out[m] = (torch.full((nq,), k, dtype=torch.int32), torch.from_numpy(top.astype(np.int64)),
                  torch.from_numpy(np.take_along_axis(S, top, 1)))
    r0, r1 = synth.shard_range(n, rank, world)
    args = (torch.from_numpy(codes[r0:r1]), torch.from_numpy(x8[r0:r1]), torch.from_numpy(qf))
    good = bench.c5_identity(*args, out, k, 2, qsel=qsel, row0=r0, world=world, rank=rank)
    bad_out = {m: (c, r.clone(), s) for m, (c, r, s) in out.items()}
    for m in (2, 3):
        bad_out[m][1][5, [0, 1]] = bad_out[m][1][5, [1, 0]]
    bad = bench.c5_identity(*args, bad_out, k, 2, qsel=qsel, row0=r0, world=world, rank=rank)
    if rank == 0:
        ok = all(good[mo]["rows_identical"] and good[mo]["scores_identical"] for mo in ("binary", "int8_cosine"))
        ok = ok and good["rows"] == n
        ok = ok and not any(bad[mo]["rows_identical"] for mo in ("binary", "int8_cosine"))
        result_q.put(bool(ok))
    else:
        result_q.put(good is None and bad is None)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_gloo_bench_config5_identity_check():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_c5_identity, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    assert all(p.exitcode == 0 for p in procs)
    assert q.get(timeout=5) is True and q.get(timeout=5) is True
