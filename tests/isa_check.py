"""ISA checks of the built gfx950 code objects (test helper, CPU only).

copies_of_inflight_lds_reads: the kernels read LDS through inline asm (`ds_read_b128` whose
completion the compiler does not track) and retire the reads with an explicit `s_waitcnt lgkmcnt`
that names the destination registers.  Nothing stops the register allocator from moving such a
value to another register with a v_mov *before* that wait, which then copies whatever the register
held before the load landed (round 4: ~1 in 10^4 K1r candidates with a wrong distance).

The check is a may-analysis over each kernel's control-flow graph (basic blocks from the s_branch
/ s_cbranch_* targets): for every DS load with a destination the state holds the minimum, over the
paths reaching the instruction, of the number of DS operations issued after it (its age).  DS
operations complete in order, so `s_waitcnt lgkmcnt(k)` retires a load exactly on the paths where
its age is >= k: the load may still be in flight iff its minimum age is < k, and states join by
taking the minimum (scalar-memory loads, which complete out of order, are not counted: the worst
case for the DS loads).  Any VGPR/AGPR touch of a destination of a DS load that may still be in
flight on SOME path is reported -- a wait inside a rarely taken branch does not cover the paths
that skip it.  Ages saturate at 15, the hardware's outstanding-LGKM limit."""
import os
import re
import shutil
import subprocess

LLVM_BIN = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
MAX_LGKM = 15

# DS operations that write a destination register
_DS_RET = ("ds_read", "ds_load", "ds_bpermute", "ds_permute", "ds_swizzle", "ds_append", "ds_consume")


def _regs(tok):
    """Vector registers a disassembly operand names: {('v', i)} / {('a', i)}."""
    m = re.fullmatch(r"([va])\[(\d+):(\d+)\]", tok)
    if m:
        return {(m[1], i) for i in range(int(m[2]), int(m[3]) + 1)}
    m = re.fullmatch(r"([va])(\d+)", tok)
    return {(m[1], int(m[2]))} if m else set()


def _regset(toks):
    out = set()
    for t in toks:
        out |= _regs(t)
    return out


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


def parse(dis):
    """{kernel: [(addr, op, toks, text, target)]} from llvm-objdump text.  `addr` is the instruction's
    address (the `// ADDR:` comment; its index when absent), `target` the absolute branch target."""
    funcs, cur, start = {}, None, 0
    for ln in dis.splitlines():
        m = re.match(r"^([0-9a-f]+) <(\S+)>:", ln)
        if m:
            start, cur = int(m[1], 16), m[2]
            funcs[cur] = []
            continue
        if cur is None:
            continue
        code, _, comment = ln.partition("//")
        s = code.strip()
        if not s or s.endswith(":"):
            continue
        op = s.split()[0]
        toks = [t for t in re.split(r"[,\s]+", s)[1:] if t]
        am = re.match(r"\s*([0-9A-Fa-f]+):", comment)
        addr = int(am[1], 16) if am else len(funcs[cur])
        target = None
        if op.startswith(("s_branch", "s_cbranch")):
            tm = re.search(r"<\S+\+0x([0-9a-f]+)>", comment)
            if tm:
                target = start + int(tm[1], 16)
            elif am and toks:  # simm16 word offset from the next instruction
                off = int(toks[0], 0)
                off = off - 65536 if off >= 32768 else off
                target = addr + 4 + 4 * off
        funcs[cur].append((addr, op, toks, s, target))
    return funcs


def _blocks(ins):
    """Basic blocks: (list of instruction indices, successor block ids)."""
    idx = {a: i for i, (a, *_r) in enumerate(ins)}
    leaders = {0}
    for i, (_a, op, _t, _s, tgt) in enumerate(ins):
        if op.startswith(("s_branch", "s_cbranch", "s_endpgm", "s_setpc")):
            if i + 1 < len(ins):
                leaders.add(i + 1)
            if tgt is not None and tgt in idx:
                leaders.add(idx[tgt])
    starts = sorted(leaders)
    bid = {s: b for b, s in enumerate(starts)}
    blocks = []
    for b, s in enumerate(starts):
        e = starts[b + 1] if b + 1 < len(starts) else len(ins)
        last = ins[e - 1]
        op, tgt = last[1], last[4]
        succ = []
        if op.startswith("s_endpgm") or op.startswith("s_setpc"):
            pass
        elif op.startswith("s_branch"):
            if tgt in idx:
                succ.append(bid[idx[tgt]])
        else:
            if op.startswith("s_cbranch") and tgt in idx:
                succ.append(bid[idx[tgt]])
            if e < len(ins):
                succ.append(bid[e])
        blocks.append((list(range(s, e)), succ))
    return blocks


def _step(st, ins, i, out, func):
    """Transfer of instruction i on a state {load index: min age}; reports touches into `out`."""
    _a, op, toks, text, _t = ins[i]
    if op == "s_waitcnt" and "lgkmcnt" in text:
        keep = int(re.search(r"lgkmcnt\((\d+)\)", text)[1])
        return {ld: age for ld, age in st.items() if age < keep}
    if op.startswith("ds_"):
        ret = op.startswith(_DS_RET) or "_rtn" in op
        srcs = _regset(toks[1:]) if ret else _regset(toks)
        for ld in st:
            if _regset(ins[ld][2][:1]) & srcs:
                out.add((func, text, ins[ld][3]))
        st = {ld: min(age + 1, MAX_LGKM) for ld, age in st.items()}
        if ret and toks:
            st[i] = 0
        return st
    if op.startswith("s_"):
        return st
    used = _regset(toks)
    for ld in st:
        if _regset(ins[ld][2][:1]) & used:
            out.add((func, text, ins[ld][3]))
    return st


def scan(dis):
    """(violations [(kernel, instruction, load)], stats {kernels, ds_loads}) over every kernel."""
    out = set()
    stats = {"kernels": 0, "ds_loads": 0}
    for func, ins in parse(dis).items():
        if not ins:
            continue
        stats["kernels"] += 1
        stats["ds_loads"] += sum(1 for x in ins if x[1].startswith(_DS_RET) or "_rtn" in x[1])
        blocks = _blocks(ins)
        state_in = [None] * len(blocks)
        state_in[0] = {}
        work = [0]
        while work:
            b = work.pop()
            st = dict(state_in[b])
            for i in blocks[b][0]:
                st = _step(st, ins, i, out, func)
            for s in blocks[b][1]:
                cur = state_in[s]
                if cur is None:
                    state_in[s] = dict(st)
                    work.append(s)
                    continue
                new = dict(cur)
                for ld, age in st.items():
                    if ld not in new or age < new[ld]:
                        new[ld] = age
                if new != cur:
                    state_in[s] = new
                    work.append(s)
    return sorted(out), stats


def copies_of_inflight_lds_reads(dis):
    """[(kernel, instruction, load)] for every touch of a DS load destination that may be in flight."""
    return scan(dis)[0]
