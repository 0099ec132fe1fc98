#!/usr/bin/env python
"""Sampled-threshold re-runs at the driver's N > 1 shard sizes (config 4: 100M rows over N ranks, nq = 1024):
for rank 0's shard of the N-way split (synth.make_corpus(n, rank=0, world=N) -- the rows bench.py gives that
rank), PREFIX + MATRIX + RECHECK with the library's own plan, then the number of queries the recheck sent to the
exact re-run (C < K: the sample under-represented their neighbourhood) and the list overflows.  A re-run costs a
whole matrix pass for every query block holding such a query.  One JSON line per N.

Usage: rank_rerun_census.py [--worlds 1,2,4,8] [--n 100000000] [--nq 1024]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests import test_gpu_lists as TL  # noqa: E402
from vectorragquantization_amd import _native as N  # noqa: E402
from vectorragquantization_amd import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--n", type=int, default=100_000_000)
    ap.add_argument("--nq", type=int, default=1024)
    ap.add_argument("--K", type=int, default=100)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    qb = synth.make_queries(a.n, a.nq, device=dev)[1]
    for world in (int(x) for x in a.worlds.split(",")):
        sh = synth.make_corpus(a.n, rank=0, world=world, device=dev)
        codes = sh["codes"]
        del sh
        torch.cuda.empty_cache()
        info, ws = TL._scan_stages(codes, qb, a.K, (N.VRQ_SCAN_STAGE_PREFIX, N.VRQ_SCAN_STAGE_MATRIX,
                                                    N.VRQ_SCAN_STAGE_RECHECK))
        nch, capc, off_cnt, off_tau = int(info[3]), int(info[4]), int(info[6]), int(info[7])
        nq = a.nq
        qa = (4 * nq + 255) // 256 * 256
        rerun = ws[off_tau + 2 * qa:off_tau + 2 * qa + 4 * nq].view(torch.int32)
        cnt = ws[off_cnt:off_cnt + 4 * nq * nch].view(torch.int32).view(nq, nch)
        print(json.dumps({"world": world, "shard_rows": int(codes.shape[0]), "plan_kind": int(info[0]), "mb": int(info[1]),
                          "queries_rerun": int((rerun != 0).sum()), "query_blocks_rerun":
                          int(((rerun != 0).view(-1, 512 if int(info[1]) == 4 else 256).any(1)).sum()) if nq % 512 == 0 else None,
                          "lists_overflowed": int((cnt > capc).sum()),
                          "candidates_per_query_mean": float(cnt.clamp(max=capc).sum(1).double().mean())}), flush=True)
        del codes, ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
