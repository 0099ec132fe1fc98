"""Build libvrq.so (the gfx950 HIP kernels + C ABI) in-tree with hipcc.

``python -m vectorragquantization_amd._build`` or ``__graft_entry__.build()``.
The shared object lands next to this file so it travels with the repository
snapshot to the GPU box (it is git-ignored, not gpurun-ignored).
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libvrq.so")
# the probe build: the same sources with -DVRQ_TUNING_ENV, whose planners read the VRQ_* tuning
# overrides from the environment (tools/ sweeps and one test); the release libvrq.so never does
PROBE_LIB = os.path.join(PKG, "libvrq_probe.so")
OBJDIR = os.path.join(PKG, "_obj")
SOURCES = ["hamming_scan.hip", "hamming_mfma.hip", "select_rescore.hip", "encode.hip", "gemm_topk.hip", "dequant.hip"]
ARCH = os.environ.get("VRQ_OFFLOAD_ARCH", "gfx950")
CFLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", f"--offload-arch={ARCH}",
          "-Wall", "-Wno-unused-function", "-Wno-unused-variable"]
# per-source extras: the matrix-core scan keeps MFMA accumulators in VGPRs (the epilogue reads
# them there; the AGPR form costs 16 v_accvgpr moves per accumulator use)
EXTRA = {"hamming_mfma.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"],
         "gemm_topk.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"]}


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the vrq HIP library cannot be built")


def _deps() -> list:
    return [os.path.join(CSRC, f) for f in os.listdir(CSRC)] + [
        os.path.join(os.path.dirname(PKG), "include", "vrq.h")]


def up_to_date(lib: str = LIB) -> bool:
    if not os.path.exists(lib):
        return False
    t = os.path.getmtime(lib)
    return all(os.path.getmtime(d) <= t for d in _deps())


def build(force: bool = False, verbose: bool = False) -> str:
    """Build libvrq.so and libvrq_probe.so (whichever is stale); returns the release library path."""
    todo = [(lib, probe) for lib, probe in ((LIB, False), (PROBE_LIB, True)) if force or not up_to_date(lib)]
    if not todo:
        return LIB
    hipcc = _hipcc()

    def compile_one(job):
        src, probe = job
        odir = os.path.join(OBJDIR, "probe") if probe else OBJDIR
        os.makedirs(odir, exist_ok=True)
        obj = os.path.join(odir, os.path.splitext(src)[0] + ".o")
        cmd = [hipcc, *CFLAGS, *(["-DVRQ_TUNING_ENV"] if probe else []), *EXTRA.get(src, []), "-c",
               os.path.join(CSRC, src), "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
        if verbose and r.stderr:
            print(r.stderr, file=sys.stderr)
        return obj

    jobs = [(src, probe) for _, probe in todo for src in SOURCES]
    with cf.ThreadPoolExecutor(max_workers=8) as ex:
        objs = list(ex.map(compile_one, jobs))
    for i, (lib, _) in enumerate(todo):
        tmp = lib + ".tmp"
        r = subprocess.run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC",
                            *objs[i * len(SOURCES):(i + 1) * len(SOURCES)], "-o", tmp], capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link of {os.path.basename(lib)} failed:\n{r.stderr}")
        os.replace(tmp, lib)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
