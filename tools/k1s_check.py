#!/usr/bin/env python
"""Exactness check of whichever Phase-I scan a library build plans, for A/B builds whose plan differs from
the release one (run under tools/with_lib.py): per case, every candidate list entry and every list against
the true distances (tests/test_gpu_lists.check_scan_lists), then the top-K (dist, row) of a query sample
against the C restatement of FAISS hammings_knn_hc.  Uniform codes, the config-4 clustered generator, and a
cluster-ordered corpus (lists may overflow there: those queries take the exact rescan, checked by the top-K).

Usage: python tools/with_lib.py tools/ab/lib_X.so tools/k1s_check.py [--cases 4200007:1024,...]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
from tests import test_gpu_lists as TL  # noqa: E402
from tests.conftest import oracle_knn  # noqa: E402
from vectorragquantization_amd import _native as N  # noqa: E402
from vectorragquantization_amd import synth  # noqa: E402
from vectorragquantization_amd.enhanced import search3  # noqa: E402


def oracle():
    import ctypes as C
    lib = C.CDLL(os.path.join(HERE, "oracle", "_build", "liboracle.so"))
    lib.oracle_hamming_knn.restype = C.c_int
    lib.oracle_hamming_knn.argtypes = [C.c_void_p, C.c_int64, C.c_int, C.c_void_p, C.c_int, C.c_int,
                                       C.c_void_p, C.c_void_p, C.c_int]
    return lib


def cluster_ordered(n, nq, dev, seed):
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    per = 1000
    ncl = (n + per - 1) // per
    cen = torch.randint(0, 256, (ncl, 128), generator=g, device=dev, dtype=torch.uint8)
    codes = cen.repeat_interleave(per, 0)[:n].clone()
    fl = torch.randint(0, 256, (n, 128), generator=g, device=dev, dtype=torch.uint8)
    for _ in range(3):
        fl &= torch.randint(0, 256, (n, 128), generator=g, device=dev, dtype=torch.uint8)
    codes ^= fl
    qb = cen[torch.randint(0, ncl, (nq,), generator=g, device=dev)].clone()
    qb ^= torch.randint(0, 256, (nq, 128), generator=g, device=dev, dtype=torch.uint8) & \
        torch.randint(0, 256, (nq, 128), generator=g, device=dev, dtype=torch.uint8) & \
        torch.randint(0, 256, (nq, 128), generator=g, device=dev, dtype=torch.uint8) & \
        torch.randint(0, 256, (nq, 128), generator=g, device=dev, dtype=torch.uint8)
    return codes, qb


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="4200007:1024:uniform,1000003:1024:uniform,4200007:1100:clustered,"
                                       "4200007:1024:ordered")
    ap.add_argument("--K", type=int, default=100)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.set_float32_matmul_precision("highest")
    olib = oracle()
    for c in a.cases.split(","):
        n, nq, kind = c.split(":")
        n, nq = int(n), int(nq)
        if kind == "uniform":
            codes, qb = TL._corpus(n, nq, dev, 7000 + nq)
        elif kind == "clustered":
            codes = synth.make_corpus(n, device=dev)["codes"]
            qb = synth.make_queries(n, nq, device=dev)[1]
        else:
            codes, qb = cluster_ordered(n, nq, dev, 99)
        info = TL.check_scan_lists(codes, qb, a.K, allow_overflow=kind != "uniform")
        x8 = torch.empty((1, 1024), dtype=torch.int8, device=dev)
        norms = torch.empty((1,), dtype=torch.float64, device=dev)
        qf = torch.zeros((nq, 1024), dtype=torch.float32, device=dev)
        cnt, rows, dist, _, _ = search3(codes, x8, norms, qf, qb, a.K, a.K, a.K, N.VRQ_SEARCH_PHASE1_ONLY)
        torch.cuda.synchronize()
        qsel = np.linspace(0, nq - 1, 64).round().astype(np.int64)
        D, I = oracle_knn(olib, codes.cpu().numpy(), qb.cpu().numpy()[qsel], a.K, threads=16)
        ok = bool(np.array_equal(D, dist.cpu().numpy()[qsel]) and np.array_equal(I, rows.cpu().numpy()[qsel]))
        print(json.dumps({"case": c, "lib": os.path.basename(N.lib_path()), "plan_kind": int(info[0]),
                          "mb": int(info[1]), "lists_exact": True, "topk_identical_64q": ok}), flush=True)
        if not ok:
            sys.exit(1)
        del codes, qb
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
