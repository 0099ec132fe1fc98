#!/usr/bin/env python
"""A/B timing of the Phase-I matrix-core scan's stages: for each (n, nq) case, uniform random codes
(config-3 generator), one PREFIX stage, then the MATRIX stage timed with HIP events (reps launches,
interleaved across the given library builds, ABAB..., so clock drift hits every build alike).  Prints
one JSON line per (case, library): ms per MATRIX launch, its FP4-dense fraction and HBM fraction.

Usage: stage_bench.py --cases 100000000:128,100000000:1024 --libs a.so,b.so [--reps 10 --rounds 3]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vectorragquantization_amd import _native as N  # noqa: E402
from vectorragquantization_amd import synth  # noqa: E402

FP4_PEAK = 10066.3  # TOPS: 1024 SIMDs x 4096 ops/clk x 2.4 GHz


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="100000000:1024")
    ap.add_argument("--libs", default="")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--K", default="100", help="K, or a comma list alternated like the libraries")
    ap.add_argument("--stage", default="matrix", choices=["matrix", "prefix", "all"])
    ap.add_argument("--clustered", action="store_true", help="the config-4 generator instead of uniform codes")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    paths0 = [p for p in a.libs.split(",") if p] or [N.lib_path()]
    Ks = [int(k) for k in str(a.K).split(",")]
    runs = [(p, k) for p in paths0 for k in Ks]  # every (library, K) pair, alternated
    opened = {p: N._open(p, p) for p in paths0}
    paths = [p for p, _ in runs]
    libs = [opened[p] for p in paths]
    st = N.stream_handle(dev)
    cur_n, codes = None, None
    for c in a.cases.split(","):
        n, nq = (int(x) for x in c.split(":")[:2])
        if n != cur_n:
            codes = None
            torch.cuda.empty_cache()
            codes = synth.make_corpus(n, device=dev)["codes"] if a.clustered else synth.random_codes(n, device=dev)
            torch.cuda.empty_cache()
            cur_n = n
        qb = synth.make_queries(n, nq, device=dev)[1] if a.clustered else synth.flip_queries(codes, nq)[0]
        base = N.VRQ_SEARCH_PHASE1_ONLY
        wss = []
        for lib, (_, K) in zip(libs, runs):
            ws = torch.zeros((lib.vrq_search3_workspace_size(n, 1024, nq, K),), dtype=torch.uint8, device=dev)
            for stage in (N.VRQ_SCAN_STAGE_PREFIX, N.VRQ_SCAN_STAGE_MATRIX):
                N.check(lib.vrq_search3_scan(N.ptr(codes), n, 1024, N.ptr(qb), nq, K, base | stage, N.ptr(ws),
                                             ws.numel(), st), "warm")
            wss.append(ws)
        flag = {"matrix": N.VRQ_SCAN_STAGE_MATRIX, "prefix": N.VRQ_SCAN_STAGE_PREFIX, "all": 0}[a.stage]
        res = [[] for _ in libs]
        for _ in range(a.rounds):
            for i, lib in enumerate(libs):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    lib.vrq_search3_scan(N.ptr(codes), n, 1024, N.ptr(qb), nq, runs[i][1], base | flag, N.ptr(wss[i]),
                                         wss[i].numel(), st)
                e1.record()
                torch.cuda.synchronize()
                res[i].append(e0.elapsed_time(e1) / a.reps)
        for i, p in enumerate(paths):
            ms = min(res[i])
            ops = 2048.0 * nq * n
            print(json.dumps({"lib": os.path.basename(p), "K": runs[i][1], "n": n, "nq": nq, "stage": a.stage,
                              "ms": round(ms, 4),
                              "ms_rounds": [round(x, 4) for x in res[i]],
                              "fp4_frac": ops / (ms * 1e-3) / 1e12 / FP4_PEAK,
                              "hbm_frac": n * 128 / (ms * 1e-3) / 1e9 / 8000.0}), flush=True)
        del wss


if __name__ == "__main__":
    main()
