#!/usr/bin/env python
"""Micro-benchmark of the Phase-I scan kernel (K1) alone: HIP-event timing per (n, nq, K)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vectorragquantization_amd import _native as N  # noqa: E402
from vectorragquantization_amd import synth  # noqa: E402


def run(n, nq, K, reps, dev, flags=0):
    lib = N.load()
    codes = synth.random_codes(n, device=dev)
    qb, _ = synth.flip_queries(codes, nq)
    ws = torch.empty((lib.vrq_search3_workspace_size(n, 1024, nq, K),), dtype=torch.uint8, device=dev)
    st = N.stream_handle(dev)
    for _ in range(2):
        N.check(lib.vrq_search3_scan(N.ptr(codes), n, 1024, N.ptr(qb), nq, K, flags, N.ptr(ws), ws.numel(), st), "scan")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        N.check(lib.vrq_search3_scan(N.ptr(codes), n, 1024, N.ptr(qb), nq, K, flags, N.ptr(ws), ws.numel(), st), "scan")
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    gbs = (n * 128 + nq * 128) / (ms * 1e-3) / 1e9
    valu = nq * n * 64 / (ms * 1e-3) / 1e12
    del codes, ws
    torch.cuda.empty_cache()
    return {"n": n, "nq": nq, "K": K, "path": {0: "auto", N.VRQ_SEARCH_SCAN_VALU: "valu",
                                               N.VRQ_SEARCH_SCAN_MFMA: "mfma"}[flags], "ms": ms, "GB/s": gbs, "hbm_frac": gbs / 8000, "valu_Tops": valu,
            "valu_frac": valu / 39.3216}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="1000000:1024:100:valu,1000000:1024:100:mfma,1000000:256:100:mfma,10000000:1024:100:mfma,1000000:64:100,100000000:1:100,100000000:8:100,100000000:64:100")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    paths = {"auto": 0, "valu": N.VRQ_SEARCH_SCAN_VALU, "mfma": N.VRQ_SEARCH_SCAN_MFMA}
    for c in a.cases.split(","):
        f = c.split(":")
        n, nq, K = (int(x) for x in f[:3])
        print(json.dumps(run(n, nq, K, a.reps, dev, paths[f[3]] if len(f) > 3 else 0)), flush=True)
