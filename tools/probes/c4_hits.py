"""Hits of the Phase-I thresholded pass per query: list lengths after PREFIX + MATRIX (+ RECHECK) for the
config-4 generator (clustered) and for uniform codes, 100M x 1024 queries, K = 100 (timing aid)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from vectorragquantization_amd import _native as N  # noqa: E402
from vectorragquantization_amd import synth  # noqa: E402

dev = torch.device("cuda", 0)
lib = N.load()
n, nq, K = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000, 1024, 100
for kind in ("clustered", "uniform"):
    if kind == "clustered":
        sh = synth.make_corpus(n, device=dev)
        codes = sh["codes"]
        del sh
        _, qb, _ = synth.make_queries(n, nq, device=dev)
    else:
        codes = synth.random_codes(n, device=dev)
        qb, _ = synth.flip_queries(codes, nq)
    torch.cuda.empty_cache()
    flags = N.VRQ_SEARCH_PHASE1_ONLY | N.VRQ_SEARCH_SCAN_MFMA
    info = np.zeros(12, np.int64)
    N.check(lib.vrq_scan_plan(n, 1024, nq, K, flags, info.ctypes.data), "plan")
    ws = torch.zeros((int(info[11]),), dtype=torch.uint8, device=dev)
    st = N.stream_handle(dev)
    for stage in (N.VRQ_SCAN_STAGE_PREFIX, N.VRQ_SCAN_STAGE_MATRIX):
        N.check(lib.vrq_search3_scan(N.ptr(codes), n, 1024, N.ptr(qb), nq, K, flags | stage, N.ptr(ws), ws.numel(),
                                     st), "scan")
    torch.cuda.synchronize()
    nch, capc, off_cnt, off_tau, j = int(info[3]), int(info[4]), int(info[6]), int(info[7]), int(info[9])
    cnt = ws[off_cnt:off_cnt + 4 * nq * nch].view(torch.int32).view(nq, nch).cpu().numpy().astype(np.int64)
    tot = cnt.sum(1)
    print({"kind": kind, "n": n, "kernel": int(info[0]), "chunks": nch, "capc": capc, "j": j,
           "hits_per_query_mean": float(tot.mean()), "p50": float(np.percentile(tot, 50)),
           "p99": float(np.percentile(tot, 99)), "max": int(tot.max()),
           "lists_over_capc": int((cnt > capc).sum()), "max_list": int(cnt.max())}, flush=True)
    del codes, qb, ws
    torch.cuda.empty_cache()
