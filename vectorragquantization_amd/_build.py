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


_TOOLCHAIN = None


def _toolchain_id() -> str:
    """`hipcc --version` plus the compile-flag environment hipcc reads: part of each object's stamp."""
    global _TOOLCHAIN
    if _TOOLCHAIN is None:
        r = subprocess.run([_hipcc(), "--version"], capture_output=True, text=True)
        env = [f"{k}={os.environ[k]}" for k in ("HIPCC_COMPILE_FLAGS_APPEND", "HIPCC_LINK_FLAGS_APPEND",
                                               "HIP_CLANG_PATH", "ROCM_PATH") if k in os.environ]
        _TOOLCHAIN = "\n".join([r.stdout.strip(), *env])
    return _TOOLCHAIN


def _deps() -> list:
    return [os.path.join(CSRC, f) for f in os.listdir(CSRC)] + [
        os.path.join(os.path.dirname(PKG), "include", "vrq.h")]


def up_to_date(lib: str = LIB) -> bool:
    if not os.path.exists(lib):
        return False
    t = os.path.getmtime(lib)
    return all(os.path.getmtime(d) <= t for d in _deps())


class _BuildLock:
    """Exclusive lock on the object directory: concurrent loaders (the ranks of one job, the two
    workers of a test) build one after another, and the later ones find the library up to date."""

    def __enter__(self):
        import fcntl
        os.makedirs(OBJDIR, exist_ok=True)
        self.f = open(os.path.join(OBJDIR, ".build.lock"), "w")
        fcntl.flock(self.f, fcntl.LOCK_EX)
        return self

    def __exit__(self, *exc):
        import fcntl
        fcntl.flock(self.f, fcntl.LOCK_UN)
        self.f.close()


def _build_one(lib: str, probe: bool, verbose: bool, force_all: bool = False) -> None:
    hipcc = _hipcc()
    odir = os.path.join(OBJDIR, "probe") if probe else OBJDIR
    os.makedirs(odir, exist_ok=True)

    headers = [d for d in _deps() if d.endswith(".h")]

    def compile_one(src):
        obj = os.path.join(odir, os.path.splitext(src)[0] + ".o")
        cmd = [hipcc, *CFLAGS, *(["-DVRQ_TUNING_ENV"] if probe else []), *EXTRA.get(src, []), "-c",
               os.path.join(CSRC, src), "-o", obj]
        # incremental: an object newer than its source and every header, built by the same command
        # (the stamp names the toolchain and the flag environment too, and is removed before hipcc runs,
        # so an interrupted compile or a toolchain change never leaves a stale object looking current)
        stamp = obj + ".cmd"
        stamp_text = "\n".join([" ".join(cmd), _toolchain_id()])
        if not force_all and os.path.exists(obj) and os.path.exists(stamp):
            t = os.path.getmtime(obj)
            with open(stamp) as f:
                same = f.read() == stamp_text
            if same and all(os.path.getmtime(d) <= t for d in [os.path.join(CSRC, src), *headers]):
                return obj
        if os.path.exists(stamp):
            os.remove(stamp)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
        if verbose and r.stderr:
            print(r.stderr, file=sys.stderr)
        with open(stamp, "w") as f:
            f.write(stamp_text)
        return obj

    with cf.ThreadPoolExecutor(max_workers=8) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    tmp = lib + ".tmp"
    r = subprocess.run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", tmp], capture_output=True,
                       text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link of {os.path.basename(lib)} failed:\n{r.stderr}")
    os.replace(tmp, lib)


def build(force: bool = False, verbose: bool = False, probe: bool = False) -> str:
    """Build libvrq.so (or, with ``probe``, libvrq_probe.so) if stale; returns its path.  The release
    library never depends on the probe build."""
    lib = PROBE_LIB if probe else LIB
    if not force and up_to_date(lib):
        return lib
    with _BuildLock():
        if force or not up_to_date(lib):  # (another process may have built it while we waited)
            _build_one(lib, probe, verbose, force_all=force)
    return lib


def build_all(force: bool = False, verbose: bool = False) -> str:
    """The release library first, then the probe build (tools/ sweeps and two tests load it)."""
    build(force, verbose)
    build(force, verbose, probe=True)
    return LIB


if __name__ == "__main__":
    print(build_all(force="--force" in sys.argv, verbose=True))
