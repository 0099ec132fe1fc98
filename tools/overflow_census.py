#!/usr/bin/env python
"""Candidate-list overflow census of the large-batch Phase-I pass: on the config-4 clustered
generator and on uniform codes, run PREFIX + MATRIX + RECHECK with the library's own plan
and count the (query, chunk) lists past their capacity (each such query takes the exact rescan in the
suffix stage).  One JSON line per case: plan kind (2 = K1s, 0 = K1m), queries with an overflowed list,
lists overflowed, and the mean / max candidates per query.

Usage: overflow_census.py [--cases 1000000:1024:clustered,4000000:1024:clustered,...]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests import test_gpu_lists as TL  # noqa: E402
from vectorragquantization_amd import _native as N  # noqa: E402
from vectorragquantization_amd import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="1000000:1024:clustered,4000000:1024:clustered,12500000:1024:clustered,"
                                       "1000000:1024:uniform,4000000:1024:uniform")
    ap.add_argument("--K", type=int, default=100)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    for c in a.cases.split(","):
        n, nq, kind = c.split(":")
        n, nq = int(n), int(nq)
        if kind == "clustered":
            codes = synth.make_corpus(n, device=dev)["codes"]
            qb = synth.make_queries(n, nq, device=dev)[1]
        else:
            codes, qb = TL._corpus(n, nq, dev, 555)
        info, ws = TL._scan_stages(codes, qb, a.K, (N.VRQ_SCAN_STAGE_PREFIX, N.VRQ_SCAN_STAGE_MATRIX,
                                                    N.VRQ_SCAN_STAGE_RECHECK))
        nch, capc, off_cnt = int(info[3]), int(info[4]), int(info[6])
        cnt = ws[off_cnt:off_cnt + 4 * nq * nch].view(torch.int32).view(nq, nch).cpu().numpy()
        ovf = cnt > capc
        per_q = np.minimum(cnt, capc).sum(1)
        print(json.dumps({"case": c, "plan_kind": int(info[0]), "mb": int(info[1]), "chunks": nch, "capc": capc,
                          "queries_overflowed": int(ovf.any(1).sum()), "lists_overflowed": int(ovf.sum()),
                          "candidates_per_query_mean": float(per_q.mean()), "candidates_per_query_max": int(per_q.max())}),
              flush=True)
        del codes, qb, ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
