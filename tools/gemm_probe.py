#!/usr/bin/env python
"""Quick timing of vrq_gemm_topk stages (config-5 kernel iteration aid): synthetic corpus of --n rows,
nq queries; prints ms per stage per mode for each library given in VRQ_LIBS (comma-separated paths,
default: the in-tree libvrq.so) and each environment setting given by --env (repeatable,
"NAME=V,NAME2=V2"; the library reads its tuning knobs per call).  Results of every run are compared
with the first."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vectorragquantization_amd import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=2_000_000)
ap.add_argument("--nq", type=int, default=1024)
ap.add_argument("--k", type=int, default=10)
ap.add_argument("--iters", type=int, default=5)
ap.add_argument("--env", action="append", default=[])
ap.add_argument("--modes", default="2,3")
ap.add_argument("--stages", default="16,32,64", help="stage flags to time (64 = finish; bisect builds: skip it)")
a = ap.parse_args()
dev = torch.device("cuda", 0)
sh = synth.make_corpus(a.n, device=dev)
qf, _, _ = synth.make_queries(a.n, a.nq, device=dev)
libs = [p for p in os.environ.get("VRQ_LIBS", "").split(",") if p] or [None]
envs = a.env or [""]
modes = [int(m) for m in a.modes.split(",")]
stages = [int(x) for x in a.stages.split(",")]
ref = None
import ctypes as C  # noqa: E402
from vectorragquantization_amd import _native as N  # noqa: E402
for path in libs:
    if path:
        lib = C.CDLL(path)
        for name, (res, args) in N.SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
    else:
        lib = N.load()
    st = N.stream_handle(dev)
    for env in envs:
        kv = dict(x.split("=", 1) for x in env.split(",") if x)
        old = {k: os.environ.get(k) for k in kv}
        os.environ.update(kv)
        out, res = {}, {}
        for mode in modes:
            ws = torch.empty((lib.vrq_gemm_topk_workspace_size(mode, a.n, 1024, a.nq, a.k),), dtype=torch.uint8,
                             device=dev)
            cnt = torch.empty((a.nq,), dtype=torch.int32, device=dev)
            rows = torch.empty((a.nq, a.k), dtype=torch.int64, device=dev)
            sc = torch.empty((a.nq, a.k), dtype=torch.float64, device=dev)
            times = {st_: [] for st_ in stages}
            for it in range(a.iters + 1):
                for stage in stages:
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    rc = lib.vrq_gemm_topk(mode, N.ptr(sh["codes"]), N.ptr(sh["x8"]), N.ptr(sh["norms"]), a.n, 1024,
                                           0, N.ptr(qf), a.nq, a.k, stage, N.ptr(cnt), N.ptr(rows), N.ptr(sc),
                                           N.ptr(ws), ws.numel(), st)
                    assert rc == 0, rc
                    e1.record()
                    torch.cuda.synchronize()
                    if it:
                        times[stage].append(e0.elapsed_time(e1))
            out[mode] = {k: round(sorted(v)[len(v) // 2], 3) for k, v in times.items()}
            res[mode] = (rows.clone(), sc.clone())
            del ws
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        same = None
        if ref is None:
            ref = res
        else:
            same = all(torch.equal(ref[m][0], res[m][0]) and torch.equal(ref[m][1], res[m][1]) for m in modes)
        tot = round(sum(sum(v.values()) for v in out.values()), 3)
        print(json.dumps({"lib": path or "in-tree", "env": env, "ms": out, "total_ms": tot, "same_as_first": same}),
              flush=True)
