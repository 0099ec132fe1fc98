#!/usr/bin/env python
"""bench.py -- throughput of CohereEnhancedVectorDB's three-phase search on MI355X.

Metric (BASELINE.json): queries/sec + recall@10 vs float32, d=1024 3-phase
search at 1/2/4/8 GPUs.  Default workload = BASELINE config 4: 3-phase search
over a 100M x 1024 synthetic corpus (SURVEY.md section 8(d) generator), query
batches of nq = 1024, k = 10, binary_oversample = 10, int8_oversample = 3.  The
same corpus and the same batch at every N (strong scaling): with --gpus N the
corpus is row-sharded over N ranks, each rank searches its shard and one RCCL
all_gather + vrq_merge_shards reproduces the single-index result exactly.  At
N = 1 the whole 100M-row corpus (codes 12.8 GB + int8 102.4 GB) sits in one
MI355X's HBM.

One step = one three-phase search of the whole nq-query batch:
  K1 vrq_search3_scan (Phase I Hamming scan, per-chunk exact top-K)
  K2 vrq_search3_finish (exact merge + Phase II + Phase III + stable sorts)
  [N > 1: one RCCL all_gather of the per-shard candidates + vrq_merge_shards]
Inputs are HBM-resident before the timed region.

--config c2  BASELINE config 2 (the same 3-phase search, 1M x 1024).
--config c3  Phase-I-only HBM-roofline case (100M uniform random codes, queries
             = corpus rows with 64-256 flipped bits, nq = 8 by default).
--config c5  BASELINE config 5: the batched Phase-II + Phase-III scoring of
             nq = 1024 queries against EVERY row of a 10M x 1024 corpus on the
             matrix cores (vrq_gemm_topk), top-k fused.

rank 0 prints ONE JSON line (the driver contract).
"""
from __future__ import annotations

import argparse
import ctypes
import glob
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from vectorragquantization_amd import _native as N  # noqa: E402
from vectorragquantization_amd import synth  # noqa: E402
from vectorragquantization_amd.dist import gather_candidates, merge_shards, pack_candidates, unpack_candidates  # noqa: E402

METRIC = "queries/sec + recall@10 vs float32, d=1024 3-phase search at 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0                          # MI355X spec (MI355X_MICROARCH.md)
# integer VALU peak: a wave64 v_xor_b32 / v_bcnt_u32_b32 retires every 4 SIMD cycles when the SIMD is
# saturated (measured: tools/probes/valu_probe.hip, profiles/r1_valu_probe.json) ->
# 1024 SIMDs x 64 lanes / 4 cycles x 2.4 GHz = 39.3 T lane-ops/s
VALU_PEAK_TOPS = 1024 * 64 / 4 * 2.4e9 / 1e12
# dense FP4 MFMA peak (MI355X_MICROARCH.md: ~10 PF dense): 1024 SIMDs x 4096 ops/clk x 2.4 GHz
MFMA_FP4_PEAK_TOPS = 1024 * 4096 * 2.4e9 / 1e12
I8_DENSE_PEAK_TOPS = 1024 * 2048 * 2.4e9 / 1e12  # v_mfma_i32_32x32x32_i8: 32 cycles, 2x the bf16 rate

# workload of each --config: corpus rows, queries per step, Phase-I only
CONFIGS = {
    "c4": dict(n=100_000_000, nq=1024, phase1=False,
               name="BASELINE config 4: CohereEnhancedVectorDB 3-phase search, row-sharded over N GPUs + RCCL "
                    "all_gather of per-shard top-K"),
    "c2": dict(n=1_000_000, nq=1024, phase1=False, name="BASELINE config 2: CohereEnhancedVectorDB 3-phase search"),
    "c3": dict(n=100_000_000, nq=8, phase1=True, name="BASELINE config 3: Phase-I-only Hamming top-k"),
    "c5": dict(n=10_000_000, nq=1024, phase1=False, name="BASELINE config 5: batched Phase-II + Phase-III exhaustive "
                                                          "scoring"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c4")
    ap.add_argument("--n", type=int, default=None, help="corpus rows (total over all ranks)")
    ap.add_argument("--nq", type=int, default=None, help="queries per step")
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--binary-oversample", type=int, default=10)
    ap.add_argument("--int8-oversample", type=int, default=3)
    ap.add_argument("--cpu-sample", type=int, default=None,
                    help="queries per pass of the host CPU baseline (default: sized to ~10 s of CPU work)")
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="host threads of the CPU baseline (default: OMP_NUM_THREADS, else os.cpu_count())")
    ap.add_argument("--recall-sample", type=int, default=128)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-recall", action="store_true")
    ap.add_argument("--no-encode", action="store_true", help="skip the encoder roofline leg")
    ap.add_argument("--no-phase1", action="store_true",
                    help="skip the config-3 Phase-I leg (roofline_phase1) of the default config-4 line")
    ap.add_argument("--scan", choices=["auto", "valu", "mfma"], default="auto",
                    help="Phase-I scan (auto = the library's choice for the shape)")
    ap.add_argument("--launch-probe", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_info(threads):
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"cores": threads, "host_nproc": os.cpu_count(), "cpu_model": model,
            "cores_note": "threads the baseline ran on = the box's CPU share for one GPU (OMP_NUM_THREADS); "
                          "host_nproc is the whole machine"}


def cpu_threads(a):
    if a.cpu_threads:
        return a.cpu_threads
    env = os.environ.get("OMP_NUM_THREADS", "")
    return int(env) if env.isdigit() and int(env) > 0 else (os.cpu_count() or 1)


class Pipeline:
    """One rank's search step with event-bracketed kernels on torch's current stream.

    Phase I runs the scan the library selects for this shape (``vrq_scan_kind``).  For the
    matrix-core scan its four stages are issued as four calls (``VRQ_SCAN_STAGE_*``) -- the
    same launches in the same order as one call -- so the dominant kernel
    (hamming_mfma_kernel) gets its own HIP events."""

    def __init__(self, codes, x8, norms, row0, n_total, qf, qb, k, osb, osi, world, phase1_only=False,
                 scan="auto"):
        self.lib = N.load()
        self.codes, self.x8, self.norms, self.row0 = codes, x8, norms, row0
        self.qf, self.qb = qf, qb
        self.k, self.K, self.K3 = k, min(k * osb, n_total), k * osi
        self.world = world
        self.phase1 = phase1_only
        self.flags = N.VRQ_SEARCH_PHASE1_ONLY if phase1_only else (N.VRQ_SEARCH_SHARD if world > 1 else 0)
        self.flags |= {"auto": 0, "valu": N.VRQ_SEARCH_SCAN_VALU, "mfma": N.VRQ_SEARCH_SCAN_MFMA}[scan]
        nq = qf.shape[0]
        dev = codes.device
        self.m = codes.shape[0]
        pre = ctypes.c_int64(0)
        self.kind = self.lib.vrq_scan_kind(self.m, 1024, nq, self.K, self.flags, ctypes.byref(pre))
        N.check(min(self.kind, 0), "vrq_scan_kind")
        self.prefix_rows = int(pre.value)
        ws = self.lib.vrq_search3_workspace_size(self.m, 1024, nq, self.K)
        self.ws = torch.empty((max(ws, 8),), dtype=torch.uint8, device=dev)
        kout = self.K if self.flags & (N.VRQ_SEARCH_SHARD | N.VRQ_SEARCH_PHASE1_ONLY) else k
        self.cnt = torch.empty((nq,), dtype=torch.int32, device=dev)
        self.rows = torch.empty((nq, kout), dtype=torch.int64, device=dev)
        self.dist = torch.empty((nq, kout), dtype=torch.int32, device=dev)
        self.s2 = torch.empty((nq, kout), dtype=torch.float64, device=dev)
        self.s3 = torch.empty((nq, kout), dtype=torch.float64, device=dev)
        self.ev = []
        self.final = None

    def _scan(self, extra, st):
        N.check(self.lib.vrq_search3_scan(N.ptr(self.codes), self.m, 1024, N.ptr(self.qb), self.qb.shape[0],
                                          self.K, self.flags | extra, N.ptr(self.ws), self.ws.numel(), st), "scan")

    def step(self, record: bool):
        L, st = self.lib, N.stream_handle(self.codes.device)
        e = [torch.cuda.Event(enable_timing=True) for _ in range(8)] if record else None
        rec = (lambda i: e[i].record()) if record else (lambda i: None)
        rec(0)
        if self.kind == N.VRQ_SCAN_KIND_MFMA:
            self._scan(N.VRQ_SCAN_STAGE_PREFIX, st)
            rec(1)
            self._scan(N.VRQ_SCAN_STAGE_MATRIX, st)
            rec(2)
            self._scan(N.VRQ_SCAN_STAGE_RECHECK, st)
            rec(6)
            self._scan(N.VRQ_SCAN_STAGE_SUFFIX, st)
        else:
            self._scan(0, st)
            rec(1)
            rec(2)
            rec(6)
        rec(3)
        N.check(L.vrq_search3_finish(N.ptr(self.codes), N.ptr(self.x8), N.ptr(self.norms), None, self.m, 1024,
                                     self.row0, N.ptr(self.qf), self.qf.shape[0], self.k, self.K, self.K3,
                                     self.flags, N.ptr(self.cnt), N.ptr(self.rows), N.ptr(self.dist),
                                     N.ptr(self.s2), N.ptr(self.s3), N.ptr(self.ws), self.ws.numel(), st),
                "finish")
        rec(4)
        if self.world > 1 and not self.phase1:
            nq = self.qf.shape[0]
            ids = self.rows  # external id = global row for the synthetic corpus
            local = pack_candidates(self.cnt, self.rows, ids, self.dist, self.s2, self.s3)
            self.gather_bytes = int(local.numel())
            buf = gather_candidates(local)
            rec(7)
            gc, gr, gi, gd, g2, g3 = unpack_candidates(buf, self.world, nq, self.K)
            self.final = merge_shards(gc, gr, gd, g2, g3, self.k, self.K3)
        else:
            self.final = (self.cnt, self.rows, self.dist, self.s2, self.s3)
            rec(7)
        rec(5)
        if record:
            self.ev.append(e)

    def stage_ms(self):
        """Mean ms per step of: scan (all stages), prefix stage, matrix stage, recheck stage, suffix stage,
        finish (K2), all-gather + merge (and the all-gather alone)."""
        def mean(i, j):
            return float(np.mean([ev[i].elapsed_time(ev[j]) for ev in self.ev]))
        return {"scan": mean(0, 3), "prefix": mean(0, 1), "matrix": mean(1, 2), "recheck": mean(2, 6),
                "suffix": mean(6, 3),
                "finish": mean(3, 4), "collective": mean(4, 5), "allgather": mean(4, 7)}


def recall_at_10(top_rows, qf, n_total, rank, world, dev, sample):
    """recall@10 of the 3-phase top-10 vs exact float32 inner product (CohereVectorDBFloat semantics)."""
    qs = qf[:sample]
    C = synth.centres(1024, dev)
    cs = synth.chunk_grid(n_total)
    r0, r1 = synth.shard_range(n_total, rank, world)

    def local():
        best_v = torch.full((qs.shape[0], 10), -float("inf"), device=dev)
        best_i = torch.full((qs.shape[0], 10), -1, dtype=torch.int64, device=dev)
        for c in range(r0 // cs, (r1 + cs - 1) // cs):
            a, b = c * cs, min((c + 1) * cs, n_total)
            F = synth.float_rows(a, b - a, 1024, dev, C, chunk=c)
            S = qs @ F.T
            v, i = torch.topk(torch.cat([best_v, S], 1), 10, dim=1)
            cand = torch.cat([best_i, torch.arange(a, b, device=dev).expand(qs.shape[0], -1)], 1)
            best_v, best_i = v, torch.gather(cand, 1, i)
            del F, S
        return best_v, best_i
    best_v, best_i = in_turns(local, rank, world)
    if world > 1:
        gv = [torch.empty_like(best_v) for _ in range(world)]
        gi = [torch.empty_like(best_i) for _ in range(world)]
        dist.all_gather(gv, best_v)
        dist.all_gather(gi, best_i)
        v, i = torch.topk(torch.cat(gv, 1), 10, dim=1)
        best_i = torch.gather(torch.cat(gi, 1), 1, i)
    gt = best_i.cpu().numpy()
    got = top_rows[:sample].cpu().numpy()
    return float(np.mean([len(set(a[a >= 0]) & set(b)) / 10.0 for a, b in zip(got, gt)]))


def real_data_recall(dev):
    """The same GPU search on the reference's persisted 1000-document Cohere corpus (golden fixture
    tests/golden/search_real.npz: codes from its index.bin, int8 from its RocksDB SST, queries = 100 doc float
    vectors): recall@10 vs exact float32 IP, and agreement of the top-10 ids with the reference's own
    CohereEnhancedVectorDB.search output on that data."""
    from vectorragquantization_amd.enhanced import search3
    from vectorragquantization_amd.quant import int8_row_norms
    p = os.path.join(HERE, "tests", "golden", "search_real.npz")
    if not os.path.exists(p):
        return None
    g = np.load(p)
    codes = torch.from_numpy(g["codes"]).to(dev)
    x8 = torch.from_numpy(g["int8"]).to(dev)
    qf = torch.from_numpy(g["qf"]).to(dev)
    qb = torch.from_numpy(g["qb"]).to(dev)
    cnt, rows, _, _, _ = search3(codes, x8, int8_row_norms(x8), qf, qb, 10, 100, 30)
    got = rows.cpu().numpy()
    gt = g["gt_float_top10"]
    rec = float(np.mean([len(set(a[a >= 0]) & set(b)) / 10.0 for a, b in zip(got, gt)]))
    same = float(np.mean([np.array_equal(a, b) for a, b in zip(got, g["k10_ids"])]))
    return {"recall_at_10": rec, "reference_top10_identical": same, "queries": int(got.shape[0]),
            "corpus": "reference db_cohere_enhanced (1000 real Cohere embed-english-v3.0 docs)"}


def _oracle_lib():
    import subprocess
    so = os.path.join(HERE, "oracle", "_build", "liboracle.so")
    if not os.path.exists(so):
        subprocess.check_call([os.path.join(HERE, "oracle", "build.sh")])
    lib = ctypes.CDLL(so)
    lib.oracle_hamming_knn.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                       ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    return lib


def cpu_phase1(lib, codes_h, qb, K, nthreads):
    """FAISS hammings_knn_hc restatement (C, OpenMP over queries): (D i32[nq, K], I i64[nq, K])."""
    qb = np.ascontiguousarray(qb)
    D = np.empty((qb.shape[0], K), np.int32)
    I = np.empty((qb.shape[0], K), np.int64)
    lib.oracle_hamming_knn(codes_h.ctypes.data, codes_h.shape[0], 128, qb.ctypes.data, qb.shape[0], K,
                           D.ctypes.data, I.ctypes.data, nthreads)
    return D, I


def cpu_baseline(codes_h, fetch_x8, qf_h, qb_h, k, osb, osi, threads, sample, gpu_rows=None, min_s=10.0,
                 single_sample=32):
    """Restated reference path on the host: FAISS hammings_knn_hc in C (OpenMP over queries)
    + the reference's NumPy Phase II / III per query (CohereEnhancedVectorDB.py:281-322).

    ``fetch_x8(rows)`` returns the int8 rows of the given candidates: the reference fetches each
    Phase-III candidate from its RocksDB store (:303); here they are fetched from the device copy
    between the timed Phase I and the timed Phases II/III (not timed, like the reference's HTTP).
    Returns (dict, top-10 agreement with the GPU)."""
    from oracle import oracle_np as O  # noqa: F401  (checker module; keeps the import path explicit)
    lib = _oracle_lib()
    nq = min(sample, qf_h.shape[0])
    K = min(k * osb, codes_h.shape[0])

    def phase23(q, rows, x8_of):
        rows = rows[rows >= 0]
        pm = 2 * np.unpackbits(codes_h[rows], axis=1).astype(np.int32) - 1
        s2 = pm.astype(np.float64) @ qf_h[q].astype(np.float64)
        o2 = sorted(range(rows.shape[0]), key=lambda j: -s2[j])[: k * osi]
        r3 = rows[o2]
        s3 = []
        for r in r3:
            v = x8_of[int(r)]
            nrm = np.linalg.norm(v)
            s3.append(-np.inf if nrm == 0 else float(qf_h[q].dot(v)) / nrm)
        o3 = sorted(range(len(s3)), key=lambda j: -s3[j])[:k]
        return r3[o3]

    def fetch(I):
        u = np.unique(I[I >= 0])
        X = fetch_x8(u)
        return {int(r): X[i] for i, r in enumerate(u)}

    # all host threads given: the whole sample per pass, passes repeated until ~min_s of CPU work
    qb = np.ascontiguousarray(qb_h[:nq])
    t_p1 = t_p23 = 0.0
    reps = 0
    while True:
        t0 = time.perf_counter()
        _, I = cpu_phase1(lib, codes_h, qb, K, threads)
        t1 = time.perf_counter()
        x8_of = fetch(I)
        t2 = time.perf_counter()
        out_rows = [phase23(q, I[q], x8_of) for q in range(nq)]
        t3 = time.perf_counter()
        t_p1, t_p23, reps = t_p1 + t1 - t0, t_p23 + t3 - t2, reps + 1
        if t_p1 + t_p23 >= min_s or reps >= 50:
            break
    # one core, one query per call: the reference's own behaviour (FAISS parallelises over queries only)
    n1 = min(single_sample, nq)
    t_single = 0.0
    for q in range(n1):
        t0 = time.perf_counter()
        _, I1 = cpu_phase1(lib, codes_h, qb_h[q:q + 1], K, 1)
        t1 = time.perf_counter()
        x8_of = fetch(I1)
        t2 = time.perf_counter()
        phase23(q, I1[0], x8_of)
        t_single += t1 - t0 + time.perf_counter() - t2
    parity = None
    if gpu_rows is not None:
        g = gpu_rows[:nq]
        parity = float(np.mean([np.array_equal(a, b[b >= 0]) for a, b in zip(out_rows, g)]))
    qps = nq * reps / (t_p1 + t_p23)
    out = {"value": qps, "unit": "queries/s", "kind": "port", **host_info(threads),
           "sample": f"{nq} queries of the same batch over the full {codes_h.shape[0]}-row corpus, {reps} pass(es); "
                     f"Phase I = C restatement of FAISS hammings_knn_hc (OpenMP over queries, {threads} threads, "
                     f"{t_p1:.2f} s), Phases II/III = the reference NumPy per-query code (1 thread, {t_p23:.2f} s; "
                     "candidate int8 rows fetched untimed, as the reference's RocksDB gets). FAISS itself is not "
                     "available offline.",
           "phase1_s": t_p1, "phase23_s": t_p23,
           "single_core": {"value": n1 / t_single, "unit": "queries/s", "cores": 1,
                           "sample": f"{n1} queries, one per call (nq=1), Phase I on 1 thread + NumPy II/III"}}
    return out, parity


def cpu_baseline_phase1(codes_h, qb_h, K, threads, gpu_dist, gpu_rows, min_s=10.0):
    """Config 3 baseline: the FAISS hammings_knn_hc restatement over the same queries and corpus, timed on the
    host; and the identity check of the GPU's Phase-I output against it (every (dist, row) of the top-K and
    the top-10 ids)."""
    lib = _oracle_lib()
    nq = qb_h.shape[0]
    t, reps = 0.0, 0
    D = I = None
    while t < min_s and reps < 20:
        t0 = time.perf_counter()
        D, I = cpu_phase1(lib, codes_h, qb_h, K, threads)
        t += time.perf_counter() - t0
        reps += 1
    t0 = time.perf_counter()
    cpu_phase1(lib, codes_h, qb_h[:1], K, 1)
    t1q = time.perf_counter() - t0
    ident_k = bool(np.array_equal(D, gpu_dist) and np.array_equal(I, gpu_rows))
    ident_10 = float(np.mean([np.array_equal(a[:10], b[:10]) for a, b in zip(I, gpu_rows)]))
    return {"value": nq * reps / t, "unit": "queries/s", "kind": "port", **host_info(threads),
            "sample": f"the same {nq} queries over the full {codes_h.shape[0]}-row corpus, {reps} pass(es), C "
                      f"restatement of FAISS hammings_knn_hc (OpenMP over queries, {threads} threads, {t:.2f} s)",
            "single_core": {"value": 1.0 / t1q, "unit": "queries/s", "cores": 1, "sample": "1 query (nq=1), 1 thread"},
            }, {"topK_dist_rows_identical": ident_k, "top10_ids_identical": ident_10}


def encode_roofline(dev, n=1 << 20, reps=5):
    """vrq_encode over n f32 vectors per mode against the HBM roofline (SURVEY.md 8(d) encode row).
    Algorithmic bytes per vector: the input row (4096 B f32 / 2048 B i16) + the code row (128 B) + the
    quantised row (1024 / 2048 / 512 B) + min/max (16 B, local modes)."""
    from vectorragquantization_amd.quant import encode
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    X = torch.randn((n, 1024), generator=g, device=dev) * 0.05
    X16 = (X * 3000).to(torch.int16)
    qbytes = {"int8g": 1024, "int16g": 2048, "int4g": 512, "int8": 1024 + 16, "int4": 512 + 16, "bin16": 0,
              "cohere": 1024}
    out = {}
    lib, st = N.load(), N.stream_handle(dev)
    modes = ("int8g", "int16g", "int4g", "int8", "int4", "bin16", "cohere")
    for mode in modes:  # one untimed launch of every mode first: the first timed mode otherwise runs cold
        encode(mode, X16 if mode == "bin16" else X, 0.1, dev)
    torch.cuda.synchronize()
    for mode in modes:
        inp = X16 if mode == "bin16" else X
        o = encode(mode, inp, 0.1, dev)  # warm-up launch; its outputs are the preallocated buffers below
        args = (N.ENC_MODES[mode], N.ptr(inp), n, 1024, 0.1, N.ptr(o["codes"]), N.ptr(o["q"]), N.ptr(o["minmax"]), st)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            lib.vrq_encode(*args)  # launches only: no allocation inside the window
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        del o
        b = n * ((2048 if mode == "bin16" else 4096) + 128 + qbytes[mode])
        out[mode] = {"ms": ms, "GB/s": b / (ms * 1e-3) / 1e9, "frac": b / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     "bytes_per_launch": b}
    del X, X16
    torch.cuda.empty_cache()
    return {"bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s", "vectors_per_launch": n,
            "timing": f"HIP events around {reps} back-to-back vrq_encode launches into preallocated outputs",
            "modes": out}


def pmc_traffic(tag, kernel):
    """Per-launch HBM bytes of `kernel` from a committed rocprofv3 --pmc summary under profiles/
    (FETCH_SIZE KiB x2 for gfx950 16-B-per-lane streams + WRITE_SIZE KiB; tools/summarize_profile.py),
    or None when no summary for this workload tag is committed."""
    files = sorted(glob.glob(os.path.join(HERE, "profiles", f"*{tag}*pmc*.json")), key=_round_key)
    if not files:
        return None
    try:
        d = json.load(open(files[-1]))
        return float(d["bytes_per_launch"][kernel])
    except Exception:
        return None


def pmc_clock(tag, kernel, peak, achieved_at_events):
    """The shader clock `kernel` ran at and its matrix-core busy fraction, from the committed clock pass
    (GRBM_GUI_ACTIVE / 8 per launch over its rocprofv3 duration; SQ_VALU_MFMA_BUSY_CYCLES over 1024
    SIMDs; MI355X_MICROARCH.md 'DVFS give-back'), and this run's rate as a fraction of the peak at
    that clock.  None when no clock pass is committed for this workload."""
    files = sorted(glob.glob(os.path.join(HERE, "profiles", f"*{tag}*pmc*.json")), key=_round_key)
    try:
        d = json.load(open(files[-1]))
        c = d["clock"][kernel]
        clk = float(c["eff_clock_ghz"])
        if not 0.5 <= clk <= 2.52:  # a clock outside the part's range is a measurement artefact
            return None
        return {"eff_clock_ghz": clk, "mfma_busy_frac": float(c["mfma_busy_frac"]),
                "peak_at_clock": peak * clk / 2.4, "frac_at_clock": achieved_at_events / (peak * clk / 2.4),
                "source": os.path.relpath(files[-1], HERE)}
    except Exception:
        return None


def _round_key(path):
    """Sort key of a committed profile file name r<round>[s<session>]_...: (round, session)."""
    import re
    m = re.match(r"r(\d+)(?:s(\d+))?_", os.path.basename(path))
    return (int(m.group(1)), int(m.group(2) or 0)) if m else (-1, 0)


# the K1r thresholded pass: hamming_mfma_rows_kernel<0, MB> (MB 1, 4) or its lean MB = 2 form
K1R_MAIN = ("hamming_mfma_rows_kernel<0", "hamming_mfma_rows_lean_kernel<0")


def _kname(kern):
    """Display / profile-summary name of a kernel spec (a name prefix or a tuple of them)."""
    return (kern if isinstance(kern, str) else kern[0]).split("<")[0]


def rocprof_avg_ms(tag, kernel):
    """rocprofv3 duration (ms) of `kernel` for this workload tag from the newest committed summary:
    profiles/r*_<tag>_dispatch.json (tools/trace_dispatches.py: the mean over the launches after the
    bench's untimed warm-up steps, i.e. the launches the HIP events time) or else the --stats average of
    profiles/r*_<tag>_kernel_stats.csv (every launch).  Returns (ms, source, what) or None."""
    import csv
    kernels = (kernel,) if isinstance(kernel, str) else tuple(kernel)  # name substrings, any matches
    disp = sorted(glob.glob(os.path.join(HERE, "profiles", f"r*_{tag}_dispatch.json")), key=_round_key)
    stats = sorted(glob.glob(os.path.join(HERE, "profiles", f"r*_{tag}_kernel_stats.csv")), key=_round_key)
    try:
        if disp and (not stats or _round_key(disp[-1]) >= _round_key(stats[-1])):
            d = json.load(open(disp[-1]))
            for name, v in d["kernels"].items():
                if any(k in name for k in kernels):
                    return (v["mean_after_warmup_ms"], os.path.relpath(disp[-1], HERE),
                            f"rocprofv3 --kernel-trace: mean of the {v['n_after_warmup']} launches after "
                            f"{d['warmup']} warm-up step(s), from the same bench command")
        if stats:
            for row in csv.DictReader(open(stats[-1])):
                if any(k in row["Name"] for k in kernels):
                    return (float(row["AverageNs"]) / 1e6, os.path.relpath(stats[-1], HERE),
                            "rocprofv3 --kernel-trace --stats average over every launch (warm-up included)")
    except Exception:
        return None
    return None


def rocprof_field(tag, kernel, work, unit_scale, peak, event_ms):
    """The `rocprof` sub-object of a roofline: the committed profiler duration of the same kernel and
    workload, its achieved rate and fraction, and the ratio of this run's HIP-event time to it."""
    rp = rocprof_avg_ms(tag, kernel)
    if not rp:
        return None
    ach = work / (rp[0] * 1e-3) / unit_scale
    return {"avg_ms": rp[0], "achieved": ach, "frac": ach / peak, "source": rp[1], "what": rp[2],
            "events_over_rocprof": event_ms / rp[0]}


class C5Pipeline:
    """Config 5 step: vrq_gemm_topk(BINARY) then vrq_gemm_topk(INT8_COSINE) over the shard, each as its
    three stages (sample / main / finish) bracketed by HIP events on the library's stream; N > 1: one
    all-gather of both phases' [nq, k] results + the (score desc, row asc) merge."""

    def __init__(self, codes, x8, norms, row0, qf, k, world):
        self.lib = N.load()
        self.codes, self.x8, self.norms, self.row0, self.qf, self.k, self.world = codes, x8, norms, row0, qf, k, world
        dev = codes.device
        nq, m = qf.shape[0], codes.shape[0]
        ws = max(self.lib.vrq_gemm_topk_workspace_size(mo, m, 1024, nq, k) for mo in (2, 3))
        assert ws > 0, "unsupported config-5 shape"
        self.ws = torch.empty((ws,), dtype=torch.uint8, device=dev)
        self.out = {mo: (torch.empty((nq,), dtype=torch.int32, device=dev),
                         torch.empty((nq, k), dtype=torch.int64, device=dev),
                         torch.empty((nq, k), dtype=torch.float64, device=dev)) for mo in (2, 3)}
        self.ev, self.final = [], None

    def _call(self, mode, stage, st):
        c, r, s = self.out[mode]
        N.check(self.lib.vrq_gemm_topk(mode, N.ptr(self.codes), N.ptr(self.x8), N.ptr(self.norms),
                                       self.codes.shape[0], 1024, self.row0, N.ptr(self.qf), self.qf.shape[0],
                                       self.k, stage, N.ptr(c), N.ptr(r), N.ptr(s), N.ptr(self.ws), self.ws.numel(),
                                       st), "vrq_gemm_topk")

    def step(self, record):
        st = N.stream_handle(self.codes.device)
        e = [torch.cuda.Event(enable_timing=True) for _ in range(8)] if record else None
        rec = (lambda i: e[i].record()) if record else (lambda i: None)
        i = 0
        rec(i)
        for mode in (N.VRQ_GEMM_BINARY, N.VRQ_GEMM_INT8_COSINE):
            for stage in (N.VRQ_GEMM_STAGE_SAMPLE, N.VRQ_GEMM_STAGE_MAIN, N.VRQ_GEMM_STAGE_FINISH):
                self._call(mode, stage, st)
                i += 1
                rec(i)
        if self.world > 1:
            from vectorragquantization_amd.dist import gather_topk, merge_topk_shards
            self.final = {}
            for mode in (2, 3):
                gr, gs = gather_topk(self.out[mode][1], self.out[mode][2])
                self.final[mode] = merge_topk_shards(gr, gs, self.k)
        else:
            self.final = self.out
        rec(7)
        if record:
            self.ev.append(e)

    def stage_ms(self):
        def mean(i, j):
            return float(np.mean([ev[i].elapsed_time(ev[j]) for ev in self.ev]))
        names = ["binary_sample", "binary_main", "binary_finish", "cosine_sample", "cosine_main", "cosine_finish"]
        d = {nm: mean(j, j + 1) for j, nm in enumerate(names)}
        d["collective"] = mean(6, 7)
        return d


def c5_candidates(P):
    """Candidates per query each MAIN pass hands its FINISH (the count next to the
    time): one SAMPLE + MAIN per mode after the timed region, on the pipeline's own workspace, then the
    per-(query, chunk) list lengths (vrq_gemm_topk_layout); an overflowed list counts as its capacity."""
    st = N.stream_handle(P.codes.device)
    nq, m = P.qf.shape[0], P.codes.shape[0]
    res = {}
    for mode, name in ((N.VRQ_GEMM_BINARY, "binary"), (N.VRQ_GEMM_INT8_COSINE, "int8_cosine")):
        plan, lay = np.zeros(8, np.int64), np.zeros(8, np.int64)
        N.check(P.lib.vrq_gemm_topk_plan(mode, m, 1024, nq, P.k, plan.ctypes.data), "plan")
        N.check(P.lib.vrq_gemm_topk_layout(mode, m, 1024, nq, P.k, lay.ctypes.data), "layout")
        nch, capc, off = int(plan[1]), int(plan[2]), int(lay[2])
        for stage in (N.VRQ_GEMM_STAGE_SAMPLE, N.VRQ_GEMM_STAGE_MAIN):
            P._call(mode, stage, st)
        torch.cuda.synchronize()
        cnt = P.ws[off:off + 4 * nq * nch].view(torch.int32).view(nq, nch)
        per_q = cnt.clamp(max=capc).sum(1).double()
        res[name] = {"mean": float(per_q.mean()), "max": int(per_q.max()), "min": int(per_q.min()),
                     "lists_overflowed": int((cnt > capc).sum()), "chunks": nch, "list_capacity": capc}
    return res


def cpu_baseline_c5(codes_h, x8_h, qf_h, k, n, nq_s=4, threads=16):
    """Reference arithmetic on the host (NumPy): Phase-II float64 GEMV over 2*unpackbits-1 and Phase-III
    float32 dot / float64 norm for every row, stable desc top-k -- on nq_s queries x the given leading
    rows, scaled to queries/s over the n-row corpus."""
    from oracle import oracle_np as O
    rs = codes_h.shape[0]
    t0 = time.perf_counter()
    for q in range(nq_s):
        for mode in ("binary", "int8_cosine"):
            S = np.concatenate([O.exhaustive_scores(mode, qf_h[q:q + 1], codes=codes_h[a:a + 65536],
                                                    x8=x8_h[a:a + 65536]) for a in range(0, rs, 65536)], 1)
            O.exhaustive_topk(S, k)
    t = time.perf_counter() - t0
    return {"value": nq_s / (t * n / rs), "unit": "queries/s", "kind": "port", **host_info(threads),
            "sample": f"{nq_s} queries x the first {rs} of {n} rows, both phases (NumPy float64 GEMV over "
                      f"2*unpackbits-1; float32 dot / float64 norm), {t:.1f} s, scaled by n/{rs}"}


def c5_identity(codes, x8, qf, out, k, threads, qsel=(5, 517), row0=0, world=1, rank=0):
    """Config-5 identity on the host: the oracle's reference scores (oracle_np.exhaustive_scores:
    CohereEnhancedVectorDB.py:283-293 / :302-318) of EVERY row for a few queries of the batch, their
    (score desc, row asc) top-k, against the GPU's rows and scores -- both phases.  Row blocks run
    on ``threads`` host threads (NumPy releases the GIL inside its kernels).  With N > 1 ranks each
    rank scores its own shard (global rows row0 + i) and keeps its top-k; rank 0 merges the shards'
    lists by (score desc, row asc) -- the union holds the global top-k -- and compares the merged GPU
    result (`out`); collective over the default group, None on the other ranks."""
    import concurrent.futures as cf
    from oracle import oracle_np as O
    t0 = time.perf_counter()
    qs = [q for q in qsel if q < qf.shape[0]]
    codes_h, x8_h, q_h = codes.cpu().numpy(), x8.cpu().numpy(), qf[qs].cpu().numpy()
    n = codes_h.shape[0]
    blk = 1 << 18
    part_top = {}
    with cf.ThreadPoolExecutor(max_workers=threads) as ex:
        for mode in ("binary", "int8_cosine"):
            S = np.empty((len(qs), n), np.float64)

            def part(a, mode=mode, S=S):
                b = min(n, a + blk)
                S[:, a:b] = O.exhaustive_scores(mode, q_h, codes=codes_h[a:b], x8=x8_h[a:b])
            list(ex.map(part, range(0, n, blk)))
            ref = O.exhaustive_topk(S, k)
            part_top[mode] = (ref + row0, np.take_along_axis(S, ref, 1))
    part_top["rows"] = n
    del codes_h, x8_h
    parts = [part_top]
    if world > 1:
        parts = [None] * world
        dist.all_gather_object(parts, part_top)
    if rank != 0:
        return None
    res = {}
    for mode in ("binary", "int8_cosine"):
        m = {"binary": 2, "int8_cosine": 3}[mode]
        rows = np.concatenate([p[mode][0] for p in parts], 1)
        sc = np.concatenate([p[mode][1] for p in parts], 1)
        ref_rows = np.empty((len(qs), k), np.int64)
        ref_sc = np.empty((len(qs), k), np.float64)
        for i in range(len(qs)):
            o = np.lexsort((rows[i], -sc[i]))[:k]
            ref_rows[i], ref_sc[i] = rows[i][o], sc[i][o]
        g_rows = out[m][1][qs].cpu().numpy()
        g_sc = out[m][2][qs].cpu().numpy()
        res[mode] = {"rows_identical": bool(np.array_equal(g_rows, ref_rows)),
                     "scores_identical": bool(np.array_equal(g_sc, ref_sc))}
    return {"queries": qs, "rows": sum(p["rows"] for p in parts), "k": k, "seconds": time.perf_counter() - t0,
            **res, "checker": "oracle_np.exhaustive_scores over every row on the host (test infrastructure)"
            + ("; each rank its shard, merged on rank 0 by (score desc, row asc)" if world > 1 else "")}


def c5_multi_gpu_fields(st, dev):
    """Config 5's N > 1 fields: process group, per-rank spread of the two main passes, the exchange time
    (the two gather_topk + merge_topk_shards).  Collective over the default group."""
    world = dist.get_world_size()
    mine = torch.tensor([st["binary_main"], st["cosine_main"], st["collective"]], dtype=torch.float64, device=dev)
    allr = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(allr, mine)
    allr = torch.stack(allr).cpu().numpy()
    return {"world_size_process_group": world, "backend": dist.get_backend(),
            "rank_binary_main_ms": {"min": float(allr[:, 0].min()), "max": float(allr[:, 0].max())},
            "rank_cosine_main_ms": {"min": float(allr[:, 1].min()), "max": float(allr[:, 1].max())},
            "gather_merge_ms_max_over_ranks": float(allr[:, 2].max()),
            "collective": "per phase one all_gather of the per-shard top-k (rows, scores) + merge_topk_shards"}


def timed_loop(P, a, world, dev):
    """W untimed warm-up steps, then EXACTLY K timed steps between barrier + synchronize (max over ranks).
    The timed steps carry no per-stage events: each timing event record costs ~4.8 us of GPU time on
    this stack (two consecutive records are that far apart), ~40 us per step at 8 records -- 7 % of a
    config-2 step.  The per-stage breakdown (stage_ms) comes from K further, instrumented steps run
    after the timed region."""
    for _ in range(a.warmup):
        P.step(False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        P.step(False)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    T = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([T], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        T = float(tt.item())
    for _ in range(a.steps):  # per-stage HIP events (not timed)
        P.step(True)
    torch.cuda.synchronize()
    return T


def run_c5(a, world, rank, dev):
    n = a.n or CONFIGS["c5"]["n"]
    nq = a.nq or CONFIGS["c5"]["nq"]
    t_setup = time.perf_counter()
    shard, qf, qb = make_data(n, nq, rank, world, dev)
    codes, x8, norms, row0 = shard["codes"], shard["x8"], shard["norms"], shard["row0"]
    torch.cuda.synchronize()
    log(f"[rank {rank}] c5 data ready in {time.perf_counter() - t_setup:.1f} s: shard rows {codes.shape[0]}")
    P = C5Pipeline(codes, x8, norms, row0, qf, a.k, world)
    T = timed_loop(P, a, world, dev)
    rec = None
    if not a.no_recall:
        rec = recall_at_10(P.final[3][1], qf, n, rank, world, dev, min(a.recall_sample, nq))
    st = P.stage_ms()
    multi = None
    if world > 1:
        multi = c5_multi_gpu_fields(st, dev)
        if not a.no_cpu_baseline:
            multi["sample_check"] = c5_identity(codes, x8, qf, P.final, a.k, cpu_threads(a), row0=row0,
                                                world=world, rank=rank)
    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return
    m = codes.shape[0]
    ops = 2.0 * nq * m * 1024  # algorithmic MACs x 2 per phase
    tag = f"c5_n{n}_nq{nq}_g{world}"
    pieces = P.lib.vrq_gemm_topk_pieces()
    roof = {"bound": "mfma", "achieved": ops / (st["cosine_main"] * 1e-3) / 1e12, "peak": I8_DENSE_PEAK_TOPS,
            "unit": "TOPS", "kernel": f"gemm_topk_kernel<INT8_COSINE> main pass (v_mfma_i32_32x32x32_i8, {pieces} "
            "int8 piece(s) per query)", "kernel_ms": st["cosine_main"], "algorithmic_ops_per_launch": ops,
            "peak_note": "i8 dense MFMA peak (1024 SIMDs x 2048 ops/clk x 2.4 GHz); vs the bf16 dense peak that "
                         "SURVEY.md 8(d) prices config 5 against (2516 TOPS) the fraction is 2x",
            "frac_vs_bf16_dense": ops / (st["cosine_main"] * 1e-3) / 1e12 / (I8_DENSE_PEAK_TOPS / 2),
            "mfma_issue_frac_i8": pieces * ops / (st["cosine_main"] * 1e-3) / 1e12 / I8_DENSE_PEAK_TOPS,
            "algorithmic_bytes_per_launch": m * 1024 + m * 8, "traffic": pmc_traffic(tag, "gemm_topk_kernel")}
    roof["frac"] = roof["achieved"] / roof["peak"]
    roof["rocprof"] = rocprof_field(tag, "gemm_topk_kernel<3, false, false>", ops, 1e12, I8_DENSE_PEAK_TOPS,
                                    st["cosine_main"])
    roof["clock"] = pmc_clock(tag, "gemm_topk_kernel", I8_DENSE_PEAK_TOPS, roof["achieved"])
    roof_bin = {"achieved": ops / (st["binary_main"] * 1e-3) / 1e12, "kernel_ms": st["binary_main"],
                "kernel": "gemm_topk_kernel<BINARY> main pass", "algorithmic_bytes_per_launch": m * 128}
    roof_bin["frac"] = roof_bin["achieved"] / roof["peak"]
    roof_bin["clock"] = pmc_clock(tag, "gemm_topk_kernel_binary", I8_DENSE_PEAK_TOPS, roof_bin["achieved"])
    out = {
        "metric": METRIC, "value": nq * a.steps / T, "unit": "queries/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": T / a.steps * 1e3, "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "i8 (int8-quantised f32 queries, proven error bound) + f64 exact rescoring",
        "data": "synthetic (SURVEY.md 8(d) clustered d=1024 generator; int8/ubinary from the gfx950 encoder)",
        "config": {"workload": f"{CONFIGS['c5']['name']}, {n} x 1024 corpus, nq={nq} queries per step, "
                               f"fused top-{a.k}",
                   "corpus_rows": n, "nq": nq, "k": a.k,
                   "parallelism": f"row-shard x{world} + RCCL all_gather" if world > 1 else "1 GPU"},
        "recall_at_10": rec, "phase_ms": st, "roofline": roof, "roofline_binary": roof_bin,
    }
    if multi is not None:
        out["multi_gpu"] = multi
    if world == 1 and not a.no_cpu_baseline:
        rs = min(m, 1_000_000)
        out["cpu_baseline"] = cpu_baseline_c5(codes[:rs].cpu().numpy(), x8[:rs].cpu().numpy(), qf.cpu().numpy(),
                                              a.k, m, threads=cpu_threads(a))
        out["cpu_gpu_identity"] = c5_identity(codes, x8, qf, P.final, a.k, cpu_threads(a))
    out["candidates_per_query"] = c5_candidates(P)  # (after every check of P's outputs: it reuses P's workspace)
    emit(out)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def make_data(n, nq, rank, world, dev):
    """This rank's rows of the synthetic corpus and the query batch (the same on every rank).  In a
    VRQ_BENCH_SHARED_GPU rehearsal the ranks take turns (their generation transients would not fit one
    GPU together) and return the cached blocks."""
    def gen():
        shard = synth.make_corpus(n, rank=rank, world=world, device=dev)
        qf, qb, _ = synth.make_queries(n, nq, device=dev)
        return shard, qf, qb
    return in_turns(gen, rank, world)


def in_turns(fn, rank, world):
    """fn() (no collective inside); in a VRQ_BENCH_SHARED_GPU rehearsal the ranks run it one after
    another and release their allocator caches in between, so that the transients of N ranks never
    meet on the one GPU."""
    if os.environ.get("VRQ_BENCH_SHARED_GPU") != "1" or world == 1:
        return fn()
    out = None
    for r in range(world):
        if r == rank:
            out = fn()
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
        dist.barrier()
    return out


def emit(rec):
    """Rank 0's one JSON line (a VRQ_BENCH_SHARED_GPU rehearsal says so in the line)."""
    if os.environ.get("VRQ_BENCH_SHARED_GPU") == "1":
        rec["rehearsal"] = (f"{rec.get('n_gpus')} ranks sharing cuda:0 over gloo: exercises the N > 1 code path, "
                            "not a measurement")
    print(json.dumps(rec), flush=True)


def visible_gpus(env=None, topology="/sys/class/kfd/kfd/topology/nodes") -> int:
    """GPUs this process may use, counted WITHOUT initialising HIP (the launcher parent stays GPU-free):
    the KFD topology's GPU nodes (simd_count > 0), narrowed by HIP_VISIBLE_DEVICES /
    ROCR_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES when set.  Falls back to torch.cuda.device_count()
    only where the topology is unreadable."""
    env = os.environ if env is None else env
    n = 0
    try:
        for node in os.listdir(topology):
            with open(os.path.join(topology, node, "properties")) as f:
                props = dict(line.split(None, 1) for line in f if line.strip())
            if int(props.get("simd_count", "0")) > 0:
                n += 1
    except OSError:
        return torch.cuda.device_count()
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = env.get(var)
        if v is not None:
            ids = [x for x in v.split(",") if x.strip() != ""]
            n = min(n, len(ids))
    return n


def launch_plan(gpus: int, env, device_count: int):
    """How this process runs ``--gpus N`` (decided before any GPU call).

    * ``("run", world, rank, local)``: this process is one rank -- either N = 1 without a
      launcher, or one of the N ranks a launcher (torch.distributed.run, or this script's own
      spawn) started with WORLD_SIZE = N.
    * ``("spawn", N)``: N > 1 and no launcher: start N ranks of this script as child processes
      (one per GPU) and exit with their status.
    * ``("refuse", message)``: the launch cannot produce an N-GPU record (WORLD_SIZE != N, fewer
      than N devices, a local rank without a device)."""
    if gpus < 1:
        return ("refuse", f"--gpus {gpus}: need at least 1")
    ws = env.get("WORLD_SIZE")
    if ws is None:
        if device_count < gpus:
            return ("refuse", f"--gpus {gpus} but only {device_count} GPU(s) are visible")
        if gpus == 1:
            return ("run", 1, 0, 0)
        return ("spawn", gpus)
    world = int(ws)
    if world != gpus:
        return ("refuse", f"WORLD_SIZE={world} (launcher) but --gpus {gpus}: refusing to print a mislabelled record")
    rank = int(env.get("RANK", "0"))
    local = int(env.get("LOCAL_RANK", str(rank)))
    if not (0 <= rank < world) or local < 0:
        return ("refuse", f"bad RANK={rank} / LOCAL_RANK={local} for WORLD_SIZE={world}")
    if local >= device_count:
        return ("refuse", f"LOCAL_RANK={local} but only {device_count} GPU(s) are visible")
    return ("run", world, rank, local)


def spawn_ranks(n: int, build: bool = True) -> int:
    """Start n ranks of this script (same argv) as child processes with the torch.distributed env
    (127.0.0.1 rendezvous); rank 0's stdout is this process's stdout.  The parent never touches the
    GPU (it counted the devices through the KFD topology, visible_gpus) and builds the library once before
    the ranks start, so they never compile it concurrently.  If a rank fails, the others are terminated.  Returns the exit status."""
    import signal
    import socket
    import subprocess
    if build:
        N._build.build()  # (no GPU call: hipcc only, when the library is stale)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, WORLD_SIZE=str(n), RANK=str(r), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c
                log(f"[launcher] rank {procs.index(p)} exited with {c}; stopping the other ranks")
                for q in live:
                    q.send_signal(signal.SIGTERM)
        time.sleep(0.2)
    return rc


def main():
    a = parse()
    # --launch-probe (CPU tests of the launcher): pretend N devices, rendezvous over gloo, no GPU work
    # VRQ_BENCH_SHARED_GPU=1 (rehearsal of the N > 1 path on a one-GPU box): every rank runs on cuda:0 and
    # the group is gloo (RCCL refuses two ranks on one device); the line is marked and is no measurement
    shared = os.environ.get("VRQ_BENCH_SHARED_GPU") == "1"
    plan = launch_plan(a.gpus, os.environ, a.gpus if (a.launch_probe or shared) else visible_gpus())
    if plan[0] == "refuse":
        log(f"bench.py: {plan[1]}")
        sys.exit(2)
    if plan[0] == "spawn":
        sys.exit(spawn_ranks(plan[1], build=not a.launch_probe))
    _, world, rank, local = plan
    if a.launch_probe:
        rec = {"launch_probe": True, "n_gpus": world}
        if world > 1:
            dist.init_process_group("gloo", rank=rank, world_size=world)
            t = torch.tensor([rank], dtype=torch.int64)
            dist.all_reduce(t)
            assert int(t) == world * (world - 1) // 2
            rec["multi_gpu"] = launch_probe_fields(world, rank)
            dist.destroy_process_group()
        if rank == 0:
            print(json.dumps(rec), flush=True)
        return
    if shared:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if shared:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        else:
            dist.init_process_group("nccl", device_id=dev)
    if a.config == "c5":
        return run_c5(a, world, rank, dev)
    if a.config == "c3":
        return run_c3(a, world, rank, dev)
    return run_3phase(a, world, rank, dev)


PHASE1_NQS = (1, 8, 64)  # nq in {1, 8, 64} per pass


def phase1_leg(dev, n, nqs, k, osb, steps, warmup, threads, cpu=True, scan="auto"):
    """BASELINE config 3, the north star's numeric target: Phase-I-only Hamming top-K (K = k * osb)
    over n uniform random 1024-bit codes (queries = corpus rows with 64-256 flipped
    bits), at each batch size of `nqs` (the first nq queries of one query set).  Per batch size:
    `warmup` untimed + `steps` timed passes, every stage bracketed by HIP events on the library's
    stream; the dominant kernel (K1r, hamming_mfma_rows_kernel) is priced against HBM with its
    algorithmic bytes n * 128 + nq * 128.  With `cpu`, the C restatement of FAISS hammings_knn_hc
    (oracle/hamming_knn.c, checker) runs the largest query set over the same corpus on the host:
    (dist, row) of the whole top-K and the top-10 ids must be identical at every nq."""
    codes = synth.random_codes(n, device=dev)
    qall, _ = synth.flip_queries(codes, max(nqs))
    x8 = torch.empty((1, 1024), dtype=torch.int8, device=dev)
    norms = torch.empty((1,), dtype=torch.float64, device=dev)
    points, outs = {}, {}
    for nq in nqs:
        qb = qall[:nq].contiguous()
        qf = torch.zeros((nq, 1024), dtype=torch.float32, device=dev)
        P = Pipeline(codes, x8, norms, 0, n, qf, qb, k, osb, 1, 1, phase1_only=True, scan=scan)
        for _ in range(warmup):
            P.step(False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            P.step(False)
        torch.cuda.synchronize()
        T = time.perf_counter() - t0
        for _ in range(steps):  # per-stage HIP events, after the timed region (see timed_loop)
            P.step(True)
        torch.cuda.synchronize()
        st = P.stage_ms()
        mb = n * 128 + nq * 128
        kern = K1R_MAIN if P.kind == N.VRQ_SCAN_KIND_MFMA and nq <= 128 else \
            ("hamming_mfma_kernel<0" if P.kind == N.VRQ_SCAN_KIND_MFMA else "hamming_scan_kernel")
        kms = st["matrix"] if P.kind == N.VRQ_SCAN_KIND_MFMA else st["scan"]
        ach = mb / (kms * 1e-3) / 1e9
        pt = {"nq": nq, "qps": nq * steps / T, "ms_per_step": T / steps * 1e3, "phase_ms": st,
              "kernel": _kname(kern), "kernel_ms": kms, "achieved": ach, "frac": ach / HBM_PEAK_GBS,
              "algorithmic_bytes_per_launch": mb, "timing": f"HIP events on the library's stream, {steps} passes "
                                                            f"after {warmup} warm-up and {steps} timed passes",
              "mfma": {"achieved": 2048.0 * nq * n / (kms * 1e-3) / 1e12, "peak": MFMA_FP4_PEAK_TOPS, "unit": "TOPS",
                       "frac": 2048.0 * nq * n / (kms * 1e-3) / 1e12 / MFMA_FP4_PEAK_TOPS}}
        tag = f"c3_n{n}_nq{nq}_g1"
        pt["rocprof"] = rocprof_field(tag, kern, mb, 1e9, HBM_PEAK_GBS, kms)
        pt["traffic"] = pmc_traffic(tag, "hamming_mfma_rows_kernel")
        pt["clock"] = pmc_clock(tag, "hamming_mfma_rows_kernel", MFMA_FP4_PEAK_TOPS, pt["mfma"]["achieved"])
        points[str(nq)] = pt
        outs[nq] = (P.dist.cpu().numpy(), P.rows.cpu().numpy())
        del P
    out = {"workload": f"BASELINE config 3: Phase-I-only Hamming top-{min(k * osb, n)} (k={k}), {n} x 1024 "
                       "uniform random codes, queries = corpus rows with 64-256 flipped bits",
           "bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "peak_note": "8 TB/s spec; MI355X_MICROARCH.md measures 6.0-6.3 TB/s for plain in-order reads and "
                        "6.5-6.8 TB/s chip-wide for non-temporal LDS-DMA streams (the load K1r uses)",
           "target": "north_star: >= 0.50 of the HBM-read roofline at 100M rows, top-10 ids identical to the CPU",
           "points": points}
    if cpu:
        lib = _oracle_lib()
        codes_h = codes.cpu().numpy()
        q_h = qall.cpu().numpy()
        K = min(k * osb, n)
        t0 = time.perf_counter()
        D, I = cpu_phase1(lib, codes_h, q_h, K, threads)
        t_all = time.perf_counter() - t0
        t0 = time.perf_counter()
        cpu_phase1(lib, codes_h, q_h[:1], K, 1)
        t_one = time.perf_counter() - t0
        ident = {}
        for nq, (gd, gr) in outs.items():
            ident[str(nq)] = {"topK_dist_rows_identical": bool(np.array_equal(D[:nq], gd) and np.array_equal(I[:nq], gr)),
                              "top10_ids_identical": float(np.mean([np.array_equal(a[:10], b[:10])
                                                                    for a, b in zip(I[:nq], gr)]))}
        out["cpu_gpu_identity"] = ident
        out["identical_all"] = all(v["topK_dist_rows_identical"] for v in ident.values())
        out["cpu_baseline"] = {"value": q_h.shape[0] / t_all, "unit": "queries/s", "kind": "port",
                               **host_info(threads),
                               "sample": f"{q_h.shape[0]} queries over the full {n}-row corpus in one call, C "
                                         f"restatement of FAISS hammings_knn_hc (OpenMP over queries, {threads} "
                                         f"threads, {t_all:.2f} s)",
                               "single_core": {"value": 1.0 / t_one, "unit": "queries/s", "cores": 1,
                                               "sample": "1 query (nq=1), 1 thread"}}
        del codes_h
    del codes, qall
    torch.cuda.empty_cache()
    return out


def run_c3(a, world, rank, dev):
    """--config c3: the Phase-I-only line at one batch size (--nq, default 8) on one GPU."""
    if world != 1:
        log("bench.py: --config c3 is the single-GPU HBM-roofline configuration (BASELINE config 3)")
        sys.exit(2)
    n = a.n or CONFIGS["c3"]["n"]
    nq = a.nq or CONFIGS["c3"]["nq"]
    N.load()
    t0 = time.perf_counter()
    leg = phase1_leg(dev, n, (nq,), a.k, a.binary_oversample, a.steps, a.warmup, cpu_threads(a),
                     cpu=not a.no_cpu_baseline, scan=a.scan)
    pt = leg["points"][str(nq)]
    log(f"[rank 0] c3 leg in {time.perf_counter() - t0:.1f} s")
    roof = {k: pt[k] for k in ("achieved", "frac", "kernel", "kernel_ms", "algorithmic_bytes_per_launch", "timing",
                               "mfma", "rocprof", "traffic")}
    roof.update(bound="hbm", peak=HBM_PEAK_GBS, unit="GB/s", rows=n)
    out = {"metric": METRIC, "value": pt["qps"], "unit": "queries/s", "n_gpus": 1, "steps": a.steps,
           "warmup": a.warmup, "ms_per_step": pt["ms_per_step"], "higher_is_better": True, "scaling": "strong",
           "vs_baseline": None, "dtype": "u8", "data": "synthetic (uniform random 1024-bit codes, bit-flipped-row queries)",
           "config": {"workload": f"{CONFIGS['c3']['name']}, {n} x 1024 corpus, nq={nq} queries per step",
                      "corpus_rows": n, "nq": nq, "k": a.k, "binary_oversample": a.binary_oversample,
                      "parallelism": "1 GPU"},
           "phase_ms": pt["phase_ms"], "roofline": roof, "peak_note": leg["peak_note"]}
    if "cpu_baseline" in leg:
        out["cpu_baseline"] = leg["cpu_baseline"]
        out["cpu_gpu_identity"] = leg["cpu_gpu_identity"][str(nq)]
    emit(out)


def cpu_shard_candidates(lib, codes_h, x8_of, row0, qf_h, qb_h, K, threads):
    """One rank's part of the whole-corpus CPU restatement: its shard's exact top-K by (dist, row)
    (hammings_knn_hc restatement) with global rows, and every candidate's Phase-II score (f64 dot with
    2*unpackbits-1, CohereEnhancedVectorDB.py:283-293) and Phase-III score (f32 dot / f64 norm,
    :302-318).  The union over shards holds the global top-K, so the merge below restates the
    single-index search exactly."""
    D, I = cpu_phase1(lib, codes_h, qb_h, K, threads)
    res = []
    for q in range(qb_h.shape[0]):
        ok = I[q] >= 0
        rows = I[q][ok]
        pm = 2 * np.unpackbits(codes_h[rows], axis=1).astype(np.int32) - 1
        s2 = pm.astype(np.float64) @ qf_h[q].astype(np.float64)
        s3 = []
        for r in rows:
            v = x8_of(int(r))
            nrm = np.linalg.norm(v)
            s3.append(-np.inf if nrm == 0 else float(qf_h[q].dot(v)) / nrm)
        res.append((D[q][ok], rows + row0, s2, np.array(s3, np.float64)))
    return res


def cpu_merge(parts, k, K, K3):
    """Single-index semantics over the shards' candidates (CohereEnhancedVectorDB.py:267-322): global
    top-K by (dist, row) -> stable sort by s2 desc -> first K3 -> stable sort by s3 desc -> first k."""
    d = np.concatenate([p[0] for p in parts])
    r = np.concatenate([p[1] for p in parts])
    s2 = np.concatenate([p[2] for p in parts])
    s3 = np.concatenate([p[3] for p in parts])
    o = np.lexsort((r, d))[:K]
    o2 = sorted(o.tolist(), key=lambda j: -s2[j])[:K3]
    o3 = sorted(o2, key=lambda j: -s3[j])[:k]
    return r[o3]


def shard_sample_check(gpu_rows, K, K3, k, codes_h, x8_of, row0, qf_h, qb_h, threads, world, rank):
    """Rank-0 check of the merged N-rank result on a query sample against the CPU restatement over the
    WHOLE corpus: every rank restates its shard's part on its host (cpu_shard_candidates), rank 0
    merges the parts (cpu_merge) and compares the final top-k rows with `gpu_rows` (rank 0's merged
    GPU result for the sample, i64[nq, k], -1 padded).  Collective over the default group."""
    lib = _oracle_lib()
    t0 = time.perf_counter()
    part = cpu_shard_candidates(lib, codes_h, x8_of, row0, qf_h, qb_h, K, threads)
    parts = [None] * world
    if world > 1:
        dist.all_gather_object(parts, part)
    else:
        parts = [part]
    if rank != 0:
        return None
    same = []
    for q in range(qf_h.shape[0]):
        ref = cpu_merge([p[q] for p in parts], k, K, K3)
        g = gpu_rows[q][gpu_rows[q] >= 0]
        same.append(bool(np.array_equal(ref, g)))
    return {"queries": int(qf_h.shape[0]), "top10_identical": float(np.mean(same)),
            "seconds": time.perf_counter() - t0,
            "checker": "C hammings_knn_hc restatement + NumPy Phases II/III over each rank's shard on its host, "
                       "merged on rank 0 with the single-index rule (test infrastructure)"}


def multi_gpu_fields(st, gather_bytes, dev):
    """The N > 1 line's view of the run from the process group: its size and backend, per-rank min / max
    of the stage times (shard imbalance) and the exchange (bytes, time).  Collective over the default
    group; every rank returns the same dict."""
    world = dist.get_world_size()
    mine = torch.tensor([st["matrix"], st["scan"], st["finish"], st["allgather"], st["collective"]],
                        dtype=torch.float64, device=dev)
    allr = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(allr, mine)
    allr = torch.stack(allr).cpu().numpy()
    return {"world_size_process_group": world, "backend": dist.get_backend(),
            "rank_matrix_ms": {"min": float(allr[:, 0].min()), "max": float(allr[:, 0].max())},
            "rank_scan_ms": {"min": float(allr[:, 1].min()), "max": float(allr[:, 1].max())},
            "rank_finish_ms": {"min": float(allr[:, 2].min()), "max": float(allr[:, 2].max())},
            "allgather": {"bytes_per_rank": gather_bytes, "bytes_total": gather_bytes * world,
                          "ms_max_over_ranks": float(allr[:, 3].max()),
                          "with_merge_ms_max_over_ranks": float(allr[:, 4].max()),
                          "collective": "one all_gather_into_tensor (RCCL over xGMI) + vrq_merge_shards"}}


def launch_probe_fields(world, rank):
    """--launch-probe (CPU, gloo): the N > 1 line's fields on synthetic stage times, and the sample check
    on a small corpus sharded like bench.py's, with rank 0's "GPU" rows taken from the single-index
    oracle over the whole corpus (oracle_np.three_phase_batch)."""
    from oracle import oracle_np as O
    st = {"matrix": 1.0 + rank, "scan": 2.0 + rank, "finish": 0.1, "allgather": 0.05 * (rank + 1),
          "collective": 0.2}
    fields = multi_gpu_fields(st, 1234, torch.device("cpu"))
    rng = np.random.default_rng(11)
    n, nq, k, osb, osi = 6400, 8, 10, 10, 3
    codes = rng.integers(0, 256, (n, 128), dtype=np.uint8)
    codes[3000:3200] = codes[5]                               # ties across the shard boundary
    x8 = rng.integers(-127, 128, (n, 1024), dtype=np.int8)
    qf = rng.standard_normal((nq, 1024)).astype(np.float32)
    qb = codes[rng.integers(0, n, nq)] ^ rng.integers(0, 2, (nq, 128), dtype=np.uint8)
    r0, r1 = synth.shard_range(n, rank, world)
    gpu = None
    if rank == 0:
        ref = O.three_phase_batch(codes, x8, np.arange(n), qf, qb, k, osb, osi)
        gpu = np.full((nq, k), -1, np.int64)
        for q in range(nq):
            gpu[q, :ref[q]["row"].shape[0]] = ref[q]["row"]
    fields["sample_check"] = shard_sample_check(gpu, k * osb, k * osi, k, np.ascontiguousarray(codes[r0:r1]),
                                                lambda r: x8[r0 + r], r0, qf, qb, 2, world, rank)
    return fields


def run_3phase(a, world, rank, dev):
    """Configs 4 (default) and 2: the three-phase search of an nq-query batch, row-sharded over the ranks."""
    cfg = CONFIGS[a.config]
    n = a.n or cfg["n"]
    nq = a.nq or cfg["nq"]
    N.load()
    t_setup = time.perf_counter()
    shard, qf, qb = make_data(n, nq, rank, world, dev)
    codes, x8, norms, row0 = shard["codes"], shard["x8"], shard["norms"], shard["row0"]
    torch.cuda.synchronize()
    log(f"[rank {rank}] data ready in {time.perf_counter() - t_setup:.1f} s: shard rows {codes.shape[0]}")

    P = Pipeline(codes, x8, norms, row0, n, qf, qb, a.k, a.binary_oversample, a.int8_oversample, world, False,
                 a.scan)
    T = timed_loop(P, a, world, dev)
    st = P.stage_ms()

    top_rows = P.final[1]
    rec = None
    if not a.no_recall:
        rec = recall_at_10(top_rows, qf, n, rank, world, dev, min(a.recall_sample, nq))
    multi = None
    if world > 1:
        multi = multi_gpu_fields(st, P.gather_bytes, dev)
        if not a.no_cpu_baseline:
            ns = min(16, nq)
            cache = {}

            def x8_of(r):
                if r not in cache:
                    cache[r] = x8[r].cpu().numpy()
                return cache[r]
            multi["sample_check"] = shard_sample_check(
                P.final[1][:ns].cpu().numpy(), P.K, P.K3, a.k, codes.cpu().numpy(), x8_of, row0,
                qf[:ns].cpu().numpy(), qb[:ns].cpu().numpy(), cpu_threads(a), world, rank)

    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    m = codes.shape[0]
    K = P.K
    tag = f"{a.config}_n{n}_nq{nq}_g{world}"
    # whole Phase-I scan against HBM: algorithmic bytes = corpus codes + queries + K keys/query
    scan_bytes = m * 128 + nq * 128 + nq * K * 12
    roof_scan_hbm = {"bound": "hbm", "achieved": scan_bytes / (st["scan"] * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": scan_bytes / (st["scan"] * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     "scope": "all Phase-I stages", "ms": st["scan"], "algorithmic_bytes": scan_bytes}
    roof_valu = None
    if P.kind == N.VRQ_SCAN_KIND_MFMA:
        # dominant kernel: hamming_mfma_kernel over rows [prefix, m): one 1024-bit AND-popcount
        # = 1024 MACs = 2048 ops per (query, row), real queries only (padding not counted)
        rows_m = m - P.prefix_rows
        ops = 2048.0 * nq * rows_m
        ach = ops / (st["matrix"] * 1e-3) / 1e12
        # large batches: K1s (hamming_mfma_swap_kernel, plan kind 2) or K1m (hamming_mfma_kernel), both
        # summarised under "hamming_mfma_kernel" in the committed PMC summaries (tools/summarize_profile.py)
        info = np.zeros(12, np.int64)
        N.check(N.load().vrq_scan_plan(m, 1024, nq, K, P.flags, info.ctypes.data), "plan")
        k1s = int(info[0]) == 2
        kern = K1R_MAIN if nq <= 128 else ("hamming_mfma_kernel<0", "hamming_mfma_swap_kernel<0")
        roof = {"bound": "mfma", "achieved": ach, "peak": MFMA_FP4_PEAK_TOPS, "unit": "TOPS",
                "frac": ach / MFMA_FP4_PEAK_TOPS, "traffic": pmc_traffic(tag, _kname(kern)),
                "kernel": f"{'hamming_mfma_swap_kernel (K1s)' if k1s else _kname(kern)} "
                          "(FP4 e2m1 MX MFMA 32x32x64, f32 accumulate)",
                "kernel_ms": st["matrix"], "timing": "HIP events on the library's stream, this run",
                "algorithmic_ops_per_launch": ops, "algorithmic_bytes_per_launch": rows_m * 128 + nq * 128,
                "rows": rows_m,
                "prefix_rows_exact_scan": P.prefix_rows}
        roof["rocprof"] = rocprof_field(tag, kern, ops, 1e12, MFMA_FP4_PEAK_TOPS, st["matrix"])
        roof["clock"] = pmc_clock(tag, _kname(kern), MFMA_FP4_PEAK_TOPS, ach)
        if nq <= 128:  # small batches (config-2 latency leg): K1r streams the codes, priced against HBM too
            mb = rows_m * 128 + nq * 128
            roof["hbm"] = {"achieved": mb / (st["matrix"] * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                           "frac": mb / (st["matrix"] * 1e-3) / 1e9 / HBM_PEAK_GBS}
    else:
        roof = dict(roof_scan_hbm, traffic=pmc_traffic(tag, "hamming_scan_kernel"),
                    kernel="hamming_scan_kernel (wavefront popcount)", kernel_ms=st["scan"])
        valu_ops = nq * m * 64  # 32 v_xor + 32 v_bcnt lane-ops per (query, 1024-bit row)
        roof_valu = {"bound": "valu", "achieved": valu_ops / (st["scan"] * 1e-3) / 1e12, "peak": VALU_PEAK_TOPS,
                     "unit": "T lane-ops/s", "frac": valu_ops / (st["scan"] * 1e-3) / 1e12 / VALU_PEAK_TOPS}
    out = {
        "metric": METRIC, "value": nq * a.steps / T, "unit": "queries/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": T / a.steps * 1e3, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "u8+f64",
        "data": "synthetic (SURVEY.md 8(d) clustered d=1024 generator; int8/ubinary from the gfx950 encoder)",
        "config": {"workload": f"{cfg['name']}, {n} x 1024 corpus, nq={nq} queries per step",
                   "corpus_rows": n, "rows_per_gpu": m, "nq": nq, "k": a.k, "binary_oversample": a.binary_oversample,
                   "int8_oversample": a.int8_oversample, "parallelism": f"row-shard x{world} + RCCL all_gather"
                   if world > 1 else "1 GPU"},
        "recall_at_10": rec,
        "phase_ms": st, "scan_kind": "mfma" if P.kind == N.VRQ_SCAN_KIND_MFMA else "valu",
        "roofline": roof, "roofline_scan_hbm": roof_scan_hbm, "roofline_valu": roof_valu,
    }
    if multi:
        out["multi_gpu"] = multi
    if not a.no_recall:
        out["recall_note"] = ("recall_at_10 is vs exact float32 IP over the synthetic generator's floats; its "
                              "top-10 beyond the query's source row is a near-tie among ~n/4096 cluster-mates, which "
                              "sign-bit codes cannot resolve (the CPU path agrees exactly). real_data is the same "
                              "GPU search on the reference's own persisted Cohere corpus.")
        out["real_data"] = real_data_recall(dev)
    threads = cpu_threads(a)
    if world == 1 and nq <= 16:
        out["latency"] = search_latency(codes, x8, norms, qf, qb, a, dev)
    if world == 1 and not a.no_cpu_baseline:
        sample = a.cpu_sample or min(nq, 1024 if n <= 2_000_000 else 64)
        x8_src = x8

        def fetch_x8(rows):
            return x8_src[torch.from_numpy(rows).to(dev)].cpu().numpy()
        t0 = time.perf_counter()
        codes_h = codes.cpu().numpy()
        log(f"[rank 0] codes to host in {time.perf_counter() - t0:.1f} s; CPU baseline on {threads} threads, "
            f"{sample} queries")
        cb, parity = cpu_baseline(codes_h, fetch_x8, qf.cpu().numpy(), qb.cpu().numpy(), a.k, a.binary_oversample,
                                  a.int8_oversample, threads, sample, top_rows.cpu().numpy(),
                                  single_sample=max(2, min(32, 400_000_000 // n)))
        out["cpu_baseline"] = cb
        out["cpu_gpu_top10_identical"] = parity
        del codes_h
    if world == 1 and not a.no_encode:
        out["roofline_encode"] = encode_roofline(dev)
    if world == 1 and a.config == "c4" and not a.no_phase1:
        # the north star's target (BASELINE config 3) measured in the same run: the config-4 corpus
        # stays resident (117 GB) beside the 12.8 GB Phase-I corpus
        t0 = time.perf_counter()
        out["roofline_phase1"] = phase1_leg(dev, CONFIGS["c3"]["n"], PHASE1_NQS, a.k, a.binary_oversample,
                                            a.steps, a.warmup, threads, cpu=not a.no_cpu_baseline)
        log(f"[rank 0] Phase-I leg in {time.perf_counter() - t0:.1f} s")
    emit(out)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def search_latency(codes, x8, norms, qf, qb, a, dev, calls=200):
    """Single-query latency through the Python drop-in surface (SURVEY.md 8(d) config 2's nq=1 leg; the
    reference's search() answers one query per call, CohereEnhancedVectorDB.py:227-322): host wall time
    of search3 on one host-resident query -- H2D of the f32 + ubinary query, the scan stages, the
    finish, D2H of the top-k -- median and p99 over `calls` calls after 10 warm-up calls."""
    from vectorragquantization_amd.enhanced import search3
    qf_h = qf[:1].cpu().pin_memory()
    qb_h = qb[:1].cpu().pin_memory()
    ts = []
    for i in range(calls + 10):
        t0 = time.perf_counter()
        c, r, d, s2, s3 = search3(codes, x8, norms, qf_h.to(dev, non_blocking=True), qb_h.to(dev, non_blocking=True),
                                  a.k, a.binary_oversample, a.int8_oversample)
        r.cpu()
        if i >= 10:
            ts.append(time.perf_counter() - t0)
    ts = np.array(ts) * 1e3
    return {"queries_per_call": 1, "calls": calls, "median_ms": float(np.median(ts)),
            "p99_ms": float(np.percentile(ts, 99)), "min_ms": float(ts.min()),
            "what": "host wall time of one enhanced.search3 call (H2D query, Phase I-III on the GPU, D2H top-k), "
                    "workspace allocated per call by the caching allocator"}


if __name__ == "__main__":
    main()
