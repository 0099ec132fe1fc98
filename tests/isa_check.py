"""ISA checks of the built gfx950 code objects (test helper, CPU only).

copies_of_inflight_lds_reads: the kernels read LDS through inline asm (`ds_read_b128` whose
completion the compiler does not track) and retire the reads with an explicit `s_waitcnt lgkmcnt`
that names the destination registers.  Nothing stops the register allocator from moving such a
value to another register with a v_mov *before* that wait, which then copies whatever the register
held before the load landed (round 4: ~1 in 10^4 K1r candidates with a wrong distance).  This scan
walks each kernel's disassembly in program order and reports any instruction that reads or writes
the destination registers of a DS load that no lgkmcnt wait has retired yet.  Straight-line
approximation: branches are ignored (a wait on one path is taken to cover the others), which is
exact for the unrolled main loops this guards."""
import os
import re
import shutil
import subprocess

LLVM_BIN = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"


def _regs(tok):
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m[1]), int(m[2]) + 1))
    m = re.fullmatch(r"v(\d+)", tok)
    return {int(m[1])} if m else set()


def disassemble(obj, workdir):
    """Device code of a hipcc -c object (its .hip_fatbin bundle) -> llvm-objdump text."""
    objcopy = shutil.which("objcopy") or os.path.join(LLVM_BIN, "llvm-objcopy")
    fb = os.path.join(workdir, os.path.basename(obj) + ".fatbin")
    co = os.path.join(workdir, os.path.basename(obj) + ".co")
    subprocess.run([objcopy, "-O", "binary", "--only-section=.hip_fatbin", obj, fb], check=True)
    subprocess.run([os.path.join(LLVM_BIN, "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={fb}",
                    f"--targets={TARGET}", f"--output={co}"], check=True)
    r = subprocess.run([os.path.join(LLVM_BIN, "llvm-objdump"), "-d", "--no-show-raw-insn", co],
                       capture_output=True, text=True, check=True)
    return r.stdout


def copies_of_inflight_lds_reads(dis):
    """[(kernel, instruction, load)] for every touch of an in-flight DS load destination."""
    out, func, pending = [], None, []
    for ln in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", ln)
        if m:
            func, pending = m[1], []
            continue
        s = ln.split("//")[0].strip()
        if not s or func is None or s.endswith(":"):
            continue
        op = s.split()[0]
        toks = [t for t in re.split(r"[,\s]+", s)[1:] if t]
        if op == "s_waitcnt" and "lgkmcnt" in s:
            keep = int(re.search(r"lgkmcnt\((\d+)\)", s)[1])
            pending = pending[len(pending) - keep:] if keep else []
            continue
        if op.startswith("ds_") or op.startswith("s_load") or op.startswith("s_buffer_load"):
            loads = op.startswith(("ds_read", "ds_load")) or (op.startswith("ds_") and "_rtn" in op)
            srcs = set().union(*[_regs(t) for t in toks[1:]]) if loads else \
                set().union(*[_regs(t) for t in toks]) if op.startswith("ds_") else set()
            for (ld, dr) in pending:
                if dr & srcs:
                    out.append((func, s, ld))
            pending.append((s, _regs(toks[0]) if loads and toks else set()))
            continue
        if op.startswith("s_"):
            continue
        used = set().union(*[_regs(t) for t in toks]) if toks else set()
        for (ld, dr) in pending:
            if dr & used:
                out.append((func, s, ld))
    return out
