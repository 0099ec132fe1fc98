"""K1m per-workgroup timeline (diagnostic build tools/probes/var/lib_k1m_stamps.so, -DVRQ_K1M_STAMPS): for
each (n, nq) the PREFIX stage once, then the MATRIX stage several times; per workgroup the s_memrealtime
(100 MHz) stamps of its start, of its main-loop start (after the prologue) and of its end, and its
XCC / HW_ID.  Prints the spread of starts, prologue lengths, loop lengths and ends (us)."""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from vectorragquantization_amd import _native as N  # noqa: E402
from vectorragquantization_amd import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--lib", default="tools/probes/var/lib_k1m_stamps.so")
ap.add_argument("--cases", default="1000000:1024,16000000:1024")
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()
dev = torch.device("cuda", 0)
lib = N._open(a.lib, a.lib)
st = N.stream_handle(dev)
for c in a.cases.split(","):
    n, nq = (int(x) for x in c.split(":"))
    codes = synth.random_codes(n, device=dev)
    qb, _ = synth.flip_queries(codes, nq)
    info = np.zeros(12, np.int64)
    N.check(lib.vrq_scan_plan(n, 1024, nq, 100, N.VRQ_SEARCH_PHASE1_ONLY, info.ctypes.data), "plan")
    nwg = int(info[3])
    ws = torch.zeros((int(info[11]),), dtype=torch.uint8, device=dev)
    f = N.VRQ_SEARCH_PHASE1_ONLY
    lib.vrq_search3_scan(N.ptr(codes), n, 1024, N.ptr(qb), nq, 100, f | N.VRQ_SCAN_STAGE_PREFIX, N.ptr(ws), ws.numel(), st)
    for r in range(a.reps):
        lib.vrq_search3_scan(N.ptr(codes), n, 1024, N.ptr(qb), nq, 100, f | N.VRQ_SCAN_STAGE_MATRIX, N.ptr(ws), ws.numel(), st)
        torch.cuda.synchronize()
    grid = int(info[3]) * ((nq + (512 if nq >= 512 else 256) - 1) // (512 if nq >= 512 else 256))
    s = ws[:grid * 32].view(torch.int64).view(grid, 4).cpu().numpy()
    t0 = s[:, 0].min()
    start, loop, end = (s[:, 0] - t0) / 100.0, (s[:, 1] - s[:, 0]) / 100.0, (s[:, 2] - t0) / 100.0
    body = (s[:, 2] - s[:, 1]) / 100.0
    xcc = (s[:, 3] >> 32) & 0xF
    q = lambda v: [round(float(np.percentile(v, p)), 1) for p in (0, 10, 50, 90, 100)]
    print(json.dumps({"n": n, "nq": nq, "workgroups": grid, "start_us_pct0_10_50_90_100": q(start),
                      "prologue_us": q(loop), "loop_us": q(body), "end_us": q(end),
                      "kernel_span_us": round(float(end.max()), 1),
                      "per_xcc_end_max_us": {int(x): round(float(end[xcc == x].max()), 1) for x in np.unique(xcc)},
                      "per_xcc_start_max_us": {int(x): round(float(start[xcc == x].max()), 1) for x in np.unique(xcc)}}),
          flush=True)
    del codes, ws
    torch.cuda.empty_cache()
