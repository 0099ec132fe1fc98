"""The C ABI library loads and exports every symbol include/vrq.h declares; argument
validation paths that never touch a GPU.  CPU only."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from vectorragquantization_amd import _native as N

HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "vrq.h")


def declared():
    src = open(HDR).read()
    return sorted(set(re.findall(r"^\s*(?:[\w\s\*]+?)\b(vrq_\w+)\s*\(", src, re.M)))


def test_header_and_binding_agree():
    names = declared()
    assert len(names) >= 11
    assert sorted(N.SIGNATURES) == names


def test_library_exports_every_declared_symbol():
    lib = N.load()
    raw = C.CDLL(N.lib_path())
    for name in declared():
        assert hasattr(raw, name), name
    assert lib.vrq_abi_version() == 1
    assert lib.vrq_strerror(N.VRQ_EUNSUPPORTED) == b"unsupported shape"


def test_workspace_sizes():
    lib = N.load()
    # deterministic in the call shape; covers both Phase-I scans (chunk lists nq * nchunks * K * 8
    # for the wavefront scan; prefix lists + suffix list + candidate lists for the matrix-core scan)
    ws = lib.vrq_search3_workspace_size(1_000_000, 1024, 1024, 100)
    assert ws >= 1024 * 4096 * 8 and ws % 8 == 0
    assert lib.vrq_search3_workspace_size(1_000_000, 1024, 1024, 500) % (1024 * 500 * 8) == 0  # wavefront only
    assert ws == lib.vrq_hamming_topk_workspace_size(1_000_000, 128, 1024, 100)
    assert lib.vrq_search3_workspace_size(1000, 512, 1, 10) == 0      # dim unsupported
    assert lib.vrq_hamming_topk_workspace_size(10, 128, 1, 2000) == 0  # K > 1024
    # exhaustive matrix-core scorer: pure function of the shape, 0 for unsupported shapes
    g = lib.vrq_gemm_topk_workspace_size(3, 10_000_000, 1024, 1024, 10)
    assert g > 1024 * 2048 and g == lib.vrq_gemm_topk_workspace_size(2, 10_000_000, 1024, 1024, 10)
    assert lib.vrq_gemm_topk_workspace_size(3, 10_000_000, 1024, 1024, 10) < 4 << 30  # dense sample <= 2^21 cols
    assert lib.vrq_gemm_topk_workspace_size(1, 1000, 1024, 1, 10) == 0
    assert lib.vrq_gemm_topk_workspace_size(3, 1000, 1024, 1, 1025) == 0
    assert lib.vrq_gemm_topk_workspace_size(3, 1 << 32, 1024, 1, 10) == 0
    n = 100_000_000
    per_q = lib.vrq_hamming_topk_workspace_size(n, 128, 1, 100) // (100 * 8)
    assert 1 <= per_q <= 4096


def test_workspace_sizes_lane_extrema_samples():
    """The sample passes keep 32 lane extrema per (query, sample chunk), not one value per sample
    row: the workspace no longer scales with nq x S (round 1: nq x S u16 / f32 matrices), and very
    large batches or k still plan (>= 8 / >= 2k/32 sample chunks)."""
    lib = N.load()
    # config 4 shape: the scan workspace is the candidate lists plus a few MB, far below nq x S x 2 B
    ws4 = lib.vrq_search3_workspace_size(100_000_000, 1024, 1024, 100)
    assert 0 < ws4 < 1024 * (1 << 20) * 2
    # config 5 shape: f32 maxima (nq x nsc x 32) instead of nq x S floats (~800 MB at 10M rows)
    g5 = lib.vrq_gemm_topk_workspace_size(3, 10_000_000, 1024, 1024, 10)
    assert 0 < g5 < 700 << 20
    # huge batches / large k still produce a plan
    assert lib.vrq_search3_workspace_size(1_000_000, 1024, 65536, 100) > 0
    assert lib.vrq_gemm_topk_workspace_size(3, 1_000_000, 1024, 8192, 1000) > 0


@pytest.mark.parametrize("call,expect", [
    (lambda L: L.vrq_encode(99, None, 1, 1024, 0.3, None, None, None, None), N.VRQ_EINVAL),
    (lambda L: L.vrq_encode(0, None, -1, 1024, 0.3, None, None, None, None), N.VRQ_EINVAL),
    (lambda L: L.vrq_encode(0, None, 1, 1020, 0.3, None, None, None, None), N.VRQ_EINVAL),
    (lambda L: L.vrq_encode(0, None, 1, 1024, 0.0, None, None, None, None), N.VRQ_EINVAL),
    (lambda L: L.vrq_encode(0, None, 0, 1024, 0.3, None, None, None, None), N.VRQ_OK),
    (lambda L: L.vrq_search3(None, None, None, None, 10, 512, 0, None, None, 1, 1, 1, 1, 0,
                             C.c_void_p(8), C.c_void_p(8), C.c_void_p(8), C.c_void_p(8), C.c_void_p(8),
                             None, 0, None), N.VRQ_EUNSUPPORTED),
    (lambda L: L.vrq_search3(None, None, None, None, 10, 1024, 0, None, None, 1, 1, 2000, 1, 0,
                             C.c_void_p(8), C.c_void_p(8), C.c_void_p(8), C.c_void_p(8), C.c_void_p(8),
                             None, 0, None), N.VRQ_EUNSUPPORTED),
    (lambda L: L.vrq_hamming_topk(None, 10, 128, 0, None, 1, 1, None, None, None, 0, None), N.VRQ_EINVAL),
    (lambda L: L.vrq_rescore_binary(None, 1, 512, None, 1, None, 1, None, None), N.VRQ_EUNSUPPORTED),
    (lambda L: L.vrq_merge_shards(0, 1, 1, None, None, None, None, None, 1, 1, None, None, None, None, None,
                                  None, None), N.VRQ_EINVAL),
    (lambda L: L.vrq_int8_row_norms(None, -1, 1024, None, None), N.VRQ_EINVAL),
    (lambda L: L.vrq_gemm_topk(1, None, None, None, 10, 1024, 0, None, 1, 1, 0, None, None, None, None, 0, None),
     N.VRQ_EINVAL),
    (lambda L: L.vrq_gemm_topk(3, None, None, None, 10, 512, 0, None, 1, 1, 0, None, None, None, None, 0, None),
     N.VRQ_EUNSUPPORTED),
    (lambda L: L.vrq_gemm_topk(3, None, None, None, 10, 1024, 0, C.c_void_p(8), 1, 1, 0, C.c_void_p(8),
                               C.c_void_p(8), C.c_void_p(8), C.c_void_p(8), 0, None), N.VRQ_EINVAL),  # no x8
    (lambda L: L.vrq_gemm_topk(2, C.c_void_p(8), None, None, 10, 1024, 0, C.c_void_p(8), 1, 2000, 0,
                               C.c_void_p(8), C.c_void_p(8), C.c_void_p(8), C.c_void_p(8), 1 << 30, None),
     N.VRQ_EUNSUPPORTED),  # k > 1024
    (lambda L: L.vrq_gemm_topk(2, C.c_void_p(8), None, None, 100_000, 1024, 0, C.c_void_p(8), 64, 10, 0,
                               C.c_void_p(8), C.c_void_p(8), C.c_void_p(8), C.c_void_p(8), 16, None),
     N.VRQ_EWORKSPACE),
])
def test_argument_validation(call, expect):
    assert call(N.load()) == expect


def test_release_library_ignores_tuning_environment(monkeypatch):
    """The release libvrq.so plans from its defaults whatever the environment holds (it does not
    even import getenv); the probe build libvrq_probe.so reads the VRQ_* tuning overrides."""
    import subprocess
    lib, probe = N.load(), N.load_probe()
    nm = subprocess.run(["nm", "-D", N.lib_path()], capture_output=True, text=True).stdout
    assert "getenv" not in nm
    args = (3, 10_000_000, 1024, 1024, 10)
    base = lib.vrq_gemm_topk_workspace_size(*args)
    assert base == probe.vrq_gemm_topk_workspace_size(*args)
    s3 = lib.vrq_search3_workspace_size(1_000_000, 1024, 1024, 100)
    monkeypatch.setenv("VRQ_GEMM_CHUNK_MULT", "1")
    monkeypatch.setenv("VRQ_GEMM_SAMPLE_DIV", "2")
    monkeypatch.setenv("VRQ_SAMPLE_DIV", "4")
    monkeypatch.setenv("VRQ_MFMA_MB", "4")
    assert lib.vrq_gemm_topk_workspace_size(*args) == base
    assert lib.vrq_search3_workspace_size(1_000_000, 1024, 1024, 100) == s3
    assert probe.vrq_gemm_topk_workspace_size(*args) != base


def test_gemm_plan_chunk_rows_fit_the_hit_stage():
    """the thresholded pass stages a hit as (query-in-wave << 26 | chunk row), so
    every plan keeps chunk rows below 2^26 -- at large n with few chunks per query block (large nq)
    too -- and the workspace size equals the planned one."""
    import numpy as np
    lib = N.load()
    info = np.zeros(8, np.int64)
    for mode in (2, 3, 4):
        for n in (1000, 10_000_000, 300_000_000, (1 << 32) - 1):
            for nq in (1, 1024, 65536):
                assert lib.vrq_gemm_topk_plan(mode, n, 1024, nq, 10, info.ctypes.data) == N.VRQ_OK
                chunk_rows, nchunks = int(info[0]), int(info[1])
                assert 0 < chunk_rows < (1 << 26) and chunk_rows % 32 == 0
                assert nchunks == -(-n // chunk_rows) and nchunks <= 2048
                assert info[6] == lib.vrq_gemm_topk_workspace_size(mode, n, 1024, nq, 10)
    assert lib.vrq_gemm_topk_plan(3, 1 << 32, 1024, 1, 10, info.ctypes.data) == N.VRQ_EUNSUPPORTED
    assert lib.vrq_gemm_topk_plan(1, 1000, 1024, 1, 10, info.ctypes.data) == N.VRQ_EUNSUPPORTED


def test_no_dropped_kernel_stubs():
    """Every kernel the host code launches has its launch stub in the library: hipcc's host-side
    compile can drop a template kernel's stub without a diagnostic (a compound pointer expression
    in an LDS-DMA builtin did, round 4), which only shows as an unresolved symbol at load time."""
    import subprocess
    N.load()
    for lib in (N.lib_path(), N._build.PROBE_LIB):
        if not os.path.exists(lib):
            continue
        nm = subprocess.run(["nm", "-DC", lib], capture_output=True, text=True).stdout
        undefined = [ln for ln in nm.splitlines() if " U " in ln and "vrq::" in ln]
        assert not undefined, undefined[:3]


def test_no_copies_of_inflight_lds_reads(tmp_path):
    """No kernel copies (or overwrites) a register that an inline-asm LDS read has not yet filled:
    the register allocator may move such a value with a v_mov placed before the s_waitcnt that
    retires the read (round 4: K1r's next-n-block rows, ~1 in 10^4 candidates with a wrong distance
    on the GPU).  Checked on the disassembly of every built object along every static control-flow path
(tests/isa_check.py; its own unit tests: tests/test_isa_check.py)."""
    import glob
    import shutil
    import isa_check
    N.load()
    objs = sorted(glob.glob(os.path.join(N._build.OBJDIR, "*.o")))
    if not objs or not os.path.exists(os.path.join(isa_check.LLVM_BIN, "llvm-objdump")):
        pytest.skip("no built objects or no ROCm llvm tools")
    if not shutil.which("objcopy") and not os.path.exists(os.path.join(isa_check.LLVM_BIN, "llvm-objcopy")):
        pytest.skip("no objcopy")
    bad, kernels, loads = [], 0, 0
    for o in objs:
        v, st = isa_check.scan(isa_check.disassemble(o, str(tmp_path)))
        bad += v
        kernels += st["kernels"]
        loads += st["ds_loads"]
    assert kernels >= 50 and loads >= 1000, (kernels, loads)  # the disassembly was parsed, not skipped
    assert not bad, [f"{k}: {i} <- {ld}" for k, i, ld in bad[:4]]


@pytest.mark.parametrize("n,nq,kernel", [(1_000_000, 1024, 2), (4_194_304, 1024, 2), (4_194_305, 1024, 0),
                                         (1_000_000, 511, 0), (100_000_000, 1024, 0), (1_000_000, 64, 1)])
def test_scan_plan_picks_k1s_for_short_large_batch_passes(n, nq, kernel):
    """Batches of >= 512 queries run K1s (row sets resident, queries streamed; kind 2) while the pass has
    at most 2^32 (query, row) pairs and K1m's MB = 4 instance (kind 0) above; both in 512-query blocks."""
    lib = N.load()
    info = np.zeros(12, np.int64)
    N.check(lib.vrq_scan_plan(n, 1024, nq, 100, 0, info.ctypes.data), "plan")
    assert int(info[0]) == kernel
    if nq >= 512:
        assert int(info[1]) == 4


@pytest.mark.parametrize("nq,rows_kernel,mb", [(1, 1, 1), (32, 1, 1), (33, 1, 2), (64, 1, 2), (65, 1, 4),
                                               (128, 1, 4), (129, 0, 2), (1024, 0, 4)])
def test_scan_plan_picks_the_k1r_instance(nq, rows_kernel, mb):
    """vrq_scan_plan (host-only) reports the matrix-core scan a batch runs: K1r with 1 / 2 / 4 M-blocks
    per wave for <= 32 / 64 / 128 queries (the MB = 2 instance is the two-waves-per-SIMD lean kernel:
    twice the chunks of the one-wave MB = 4 instance), K1m above; the chunks cover every row once and
    the workspace holds the candidate lists, list lengths and thresholds it reports."""
    lib = N.load()
    n, K = 100_000_000, 100
    info = np.zeros(12, np.int64)
    N.check(lib.vrq_scan_plan(n, 1024, nq, K, 0, info.ctypes.data), "plan")
    assert (int(info[0]), int(info[1])) == (rows_kernel, mb)
    chunk_rows, nchunks, capc = int(info[2]), int(info[3]), int(info[4])
    assert chunk_rows % 64 == 0 and (nchunks - 1) * chunk_rows < n <= nchunks * chunk_rows
    if rows_kernel:  # one chunk per wave: 256 CUs x 4 waves x workgroups per CU
        assert nchunks == 256 * 4 * (2 if mb <= 2 else 1)
    off_cand, off_cnt, off_tau, ws = int(info[5]), int(info[6]), int(info[7]), int(info[11])
    assert off_cand + nq * nchunks * capc * 8 <= off_cnt <= off_tau < ws
