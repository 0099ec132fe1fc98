"""K1r debug: after the thresholded pass, every staged candidate (v, row) of every (query, chunk) list is
checked against the true Hamming distance (dist = v + tau_s - 1025); mismatches are printed with their
chunk / tile / n-block coordinates."""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, HERE)
from vectorragquantization_amd import _native as N  # noqa: E402
from vectorragquantization_amd import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=100_000_000)
ap.add_argument("--nq", type=int, default=64)
ap.add_argument("--reps", type=int, default=4)
a = ap.parse_args()
dev = torch.device("cuda", 0)
lib = N.load()
codes = synth.random_codes(a.n, device=dev)
qb, _ = synth.flip_queries(codes, a.nq)
K = 100
info = np.zeros(12, np.int64)
N.check(lib.vrq_scan_plan(a.n, 1024, a.nq, K, N.VRQ_SEARCH_PHASE1_ONLY, info.ctypes.data), "plan")
rows_k, mb, cr, nch, capc, off_cand, off_cnt, off_tau = (int(x) for x in info[:8])
print("plan rows", rows_k, "MB", mb, "chunk_rows", cr, "nchunks", nch, "capc", capc, flush=True)
ws = torch.zeros((int(info[11]),), dtype=torch.uint8, device=dev)
st = N.stream_handle(dev)
w8 = torch.tensor([128, 64, 32, 16, 8, 4, 2, 1], dtype=torch.uint8, device=dev)
for rep in range(a.reps):
    for stage in (N.VRQ_SCAN_STAGE_PREFIX, N.VRQ_SCAN_STAGE_MATRIX):
        N.check(lib.vrq_search3_scan(N.ptr(codes), a.n, 1024, N.ptr(qb), a.nq, K, N.VRQ_SEARCH_PHASE1_ONLY | stage,
                                     N.ptr(ws), ws.numel(), st), "scan")
    torch.cuda.synchronize()
    cnt = ws[off_cnt:off_cnt + 4 * a.nq * nch].view(torch.int32).view(a.nq, nch).clone()
    cand = ws[off_cand:off_cand + 8 * a.nq * nch * capc].view(torch.int64).view(a.nq, nch, capc).clone()
    tau_s = ws[off_tau:off_tau + 4 * a.nq].view(torch.int32).clone()
    bad = 0
    for q in range(a.nq):
        c = cnt[q].clamp(max=capc)
        idx = torch.arange(capc, device=dev)[None, :] < c[:, None]
        keys = cand[q][idx]
        rows = keys & ((1 << 40) - 1)
        v = (keys >> 40) & 0xFFFFFF
        d_gpu = v + int(tau_s[q]) - 1025
        x = codes[rows] ^ qb[q]
        d_true = sum(((x >> s) & 1).sum(1) for s in range(8))
        mism = torch.nonzero(d_gpu != d_true).flatten()
        if mism.numel():
            bad += mism.numel()
            pcr = lambda rr: int(sum(((codes[rr] >> s_) & 1).sum() for s_ in range(8)))
            for i in mism[:4].tolist():
                r = int(rows[i]); ch = r // cr; lr = r - ch * cr
                dl = int(d_gpu[i]) - int(d_true[i])
                x_all = codes[r][None, :] ^ qb
                d_all = sum(((x_all >> s_) & 1).sum(1) for s_ in range(8))
                pred = d_all - tau_s[:a.nq] + int(tau_s[q])
                cands = {"other_q": [int(qq) for qq in torch.nonzero(pred == int(d_gpu[i])).flatten().tolist()][:6],
                         "hits_of_row": [int(qq) for qq in torch.nonzero(d_all < tau_s[:a.nq]).flatten().tolist()][:6]}
                print(f"   delta {dl} q {q} " + " ".join(f"{k}={v}" for k, v in cands.items()) + f" tau_s {int(tau_s[q])}", flush=True)
                print(f"rep {rep} q {q} row {r} gpu {int(d_gpu[i])} true {int(d_true[i])} chunk {ch} "
                      f"local {lr} tile {lr // 64} nblk {(lr // 32) % 2} lane {lr % 32} tiles/chunk {cr // 64}", flush=True)
    print("rep", rep, "mismatches", bad, "lists", int(cnt.clamp(max=capc).sum()), flush=True)
