#!/usr/bin/env python
"""Config-5 candidate statistics: after the sample + main stages of vrq_gemm_topk, the per-(query,
chunk) list lengths in the workspace (offsets restated from gemm_plan in gemm_topk.hip for n = 10M,
nq = 1024, k = 10) -> candidates per query (mean / percentiles / max) for each mode."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vectorragquantization_amd import _native as N  # noqa: E402
from vectorragquantization_amd import synth  # noqa: E402


def al(x):
    return (x + 255) & ~255


n, nq, k = 10_000_000, 1024, 10
nchunks = 256
off_delta = al(nq * 1024)
off_alpha = off_delta + al(nq * 8)
off_beta = off_alpha + al(nq * 8)
off_qbf = off_beta + al(nq * 8)
off_thr = off_qbf + al(4 * 4)
off_flag = off_thr + al(nq * 4)
off_cnt = off_flag + al(nq * 4)
dev = torch.device("cuda", 0)
sh = synth.make_corpus(n, device=dev)
qf, _, _ = synth.make_queries(n, nq, device=dev)
lib, st = N.load(), N.stream_handle(dev)
for mode in (3, 2):
    ws = torch.empty((lib.vrq_gemm_topk_workspace_size(mode, n, 1024, nq, k),), dtype=torch.uint8, device=dev)
    cnt = torch.empty((nq,), dtype=torch.int32, device=dev)
    rows = torch.empty((nq, k), dtype=torch.int64, device=dev)
    sc = torch.empty((nq, k), dtype=torch.float64, device=dev)
    for stage in (16, 32):
        rc = lib.vrq_gemm_topk(mode, N.ptr(sh["codes"]), N.ptr(sh["x8"]), N.ptr(sh["norms"]), n, 1024, 0, N.ptr(qf), nq,
                               k, stage, N.ptr(cnt), N.ptr(rows), N.ptr(sc), N.ptr(ws), ws.numel(), st)
        assert rc == 0, rc
    torch.cuda.synchronize()
    cc = ws[off_cnt: off_cnt + nq * nchunks * 4].view(torch.int32).view(nq, nchunks).to(torch.int64)
    per_q = cc.clamp(max=512).sum(1).to(torch.float64)
    qs = torch.quantile(per_q, torch.tensor([0.5, 0.9, 0.99], dtype=torch.float64, device=dev)).tolist()
    print(json.dumps({"mode": mode, "mean": per_q.mean().item(), "p50": qs[0], "p90": qs[1], "p99": qs[2],
                      "max": per_q.max().item(), "total": per_q.sum().item(), "max_list": cc.max().item()}), flush=True)
