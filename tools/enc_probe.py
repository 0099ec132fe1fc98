#!/usr/bin/env python
"""Encoder (vrq_encode) throughput per mode for each library in VRQ_LIBS (comma-separated; default the
in-tree libvrq.so): 2^20 vectors of d = 1024 per launch, preallocated outputs, HIP events around
back-to-back launches; prints HBM fractions (algorithmic bytes as bench.py's roofline_encode)."""
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vectorragquantization_amd import _native as N  # noqa: E402

dev = torch.device("cuda", 0)
n, reps = 1 << 20, 10
g = torch.Generator(device=dev)
g.manual_seed(3)
X = torch.randn((n, 1024), generator=g, device=dev) * 0.05
X16 = (X * 3000).to(torch.int16)
qb = {"int8g": 1024, "int16g": 2048, "int4g": 512, "int8": 1024 + 16, "int4": 512 + 16, "bin16": 0, "cohere": 1024}
codes = torch.empty((n, 128), dtype=torch.uint8, device=dev)
q = torch.empty((n, 2048), dtype=torch.uint8, device=dev)
mm = torch.empty((n, 2), dtype=torch.float64, device=dev)
ref = None
for path in [p for p in os.environ.get("VRQ_LIBS", "").split(",") if p] or [None]:
    if path:
        lib = C.CDLL(path)
        for name, (res, args) in N.SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
    else:
        lib = N.load()
    st = N.stream_handle(dev)
    out, outs = {}, {}
    for mode, mi in N.ENC_MODES.items():
        inp = X16 if mode == "bin16" else X
        args = (mi, N.ptr(inp), n, 1024, 0.1, N.ptr(codes), N.ptr(q), N.ptr(mm), st)
        assert lib.vrq_encode(*args) == 0
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            lib.vrq_encode(*args)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        b = n * ((2048 if mode == "bin16" else 4096) + 128 + qb[mode])
        out[mode] = round(b / (ms * 1e-3) / 8e12, 3)
        outs[mode] = (codes[:4096].clone(), q[:4096].clone())
    same = None if ref is None else all(torch.equal(ref[m][0], outs[m][0]) and torch.equal(ref[m][1], outs[m][1])
                                        for m in outs)
    ref = ref or outs
    print(json.dumps({"lib": path or "in-tree", "hbm_frac": out, "same_as_first": same}), flush=True)
