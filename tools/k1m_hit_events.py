#!/usr/bin/env python
"""How often K1m's hit-extraction branch runs (config 4): PREFIX + MATRIX + RECHECK on the config-4 clustered
corpus with the library's own plan, then from the candidate lists count, per wave (128 queries x one chunk):
the hits, the n-blocks (32 rows) holding at least one hit -- each is one taken extraction branch -- the
(n-block, M-block) pairs (each runs the fast path's compare/mask code once) and the pairs in which some lane
holds two hits (the 16-ballot fallback: one row, two queries of one register half).  Divided into a probe
build's saving, this gives the cost of one taken branch.  One JSON line.

Usage: k1m_hit_events.py [--n 100000000] [--nq 1024]"""
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

KEY_ROW_BITS = TL.KEY_ROW_BITS


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000_000)
    ap.add_argument("--nq", type=int, default=1024)
    ap.add_argument("--K", type=int, default=100)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    codes = synth.make_corpus(a.n, device=dev)["codes"]
    qb = synth.make_queries(a.n, a.nq, device=dev)[1]
    info, ws = TL._scan_stages(codes, qb, a.K, (N.VRQ_SCAN_STAGE_PREFIX, N.VRQ_SCAN_STAGE_MATRIX,
                                                N.VRQ_SCAN_STAGE_RECHECK))
    kind, mb, cr, nch, capc, off_cand, off_cnt = (int(info[i]) for i in (0, 1, 2, 3, 4, 5, 6))
    nq = a.nq
    cnt = ws[off_cnt:off_cnt + 4 * nq * nch].view(torch.int32).view(nq, nch)
    cand = ws[off_cand:off_cand + 8 * nq * nch * capc].view(torch.int64).view(nq, nch, capc)
    ovf = (cnt > capc)
    live = torch.arange(capc, device=dev)[None, None, :] < torch.clamp(cnt, max=capc)[:, :, None]
    qs = torch.arange(nq, device=dev)[:, None, None].expand(nq, nch, capc)[live]
    chs = torch.arange(nch, device=dev)[None, :, None].expand(nq, nch, capc)[live]
    rows = cand[live] & ((1 << KEY_ROW_BITS) - 1)
    qpw = 32 * mb  # queries per wave
    wave = (qs // qpw) * nch + chs
    nblk = (rows - chs * cr) // 32
    nw = (nq // qpw) * nch
    # one key per (wave, n-block): taken branches
    kb = torch.unique(wave * (cr // 32 + 2) + nblk)
    # (wave, n-block, M-block): fast-path compare/mask runs
    mblk = (qs % qpw) // 32
    km = torch.unique((wave * (cr // 32 + 2) + nblk) * mb + mblk)
    # lane (r, h) of an M-block's 32x32 accumulator holds row r of the n-block and the 16 queries whose bit 2 is
    # h (one register each): two hits in one lane -> the 16-ballot fallback
    h = ((qs % 32) >> 2) & 1
    kl, lc = torch.unique((((wave * (cr // 32 + 2) + nblk) * mb + mblk) * 32 + (rows - chs * cr) % 32) * 2 + h,
                          return_counts=True)
    multi = kl[lc > 1] // 64
    per_wave = torch.bincount(kb // (cr // 32 + 2), minlength=nw).float()
    nblocks_per_wave = (cr + 31) // 32
    print(json.dumps({
        "n": a.n, "nq": nq, "plan_kind": kind, "mb": mb, "chunks": nch, "chunk_rows": cr, "capc": capc,
        "lists_overflowed": int(ovf.sum()), "hits": int(rows.numel()), "hits_per_query": rows.numel() / nq,
        "waves": nw, "nblocks_per_wave": nblocks_per_wave,
        "taken_branches_per_wave_mean": float(per_wave.mean()), "taken_branches_per_wave_max": float(per_wave.max()),
        "taken_frac": float(per_wave.mean()) / nblocks_per_wave,
        "mblock_events_per_wave": km.numel() / nw,
        "fallback_mblock_events_per_wave": torch.unique(multi).numel() / nw,
    }), flush=True)


if __name__ == "__main__":
    main()
