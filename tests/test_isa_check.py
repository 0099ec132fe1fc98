"""Unit tests of tests/isa_check.py on hand-written gfx950 disassembly (CPU only): the in-flight LDS
read check must follow every static path -- a wait inside a branch covers only the paths through it."""
import isa_check


def _dis(lines, name="k"):
    """llvm-objdump-style text: one 4-byte instruction per line from 0x1000, labels 'L:' resolved to
    <name+0xOFF> branch comments."""
    labels, out, pc = {}, [], 0
    for ln in lines:
        if ln.endswith(":"):
            labels[ln[:-1]] = pc
        else:
            pc += 4
    out.append(f"0000000000001000 <{name}>:")
    pc = 0
    for ln in lines:
        if ln.endswith(":"):
            continue
        op = ln.split()[0]
        cmt = f"// {0x1000 + pc:012X}: 00000000"
        if op.startswith(("s_branch", "s_cbranch")):
            tgt = ln.split()[1]
            ln = f"{op} 0"
            cmt += f" <{name}+0x{labels[tgt]:x}>"
        out.append(f"\t{ln:<58}{cmt}")
        pc += 4
    return "\n".join(out) + "\n"


def _bad(lines):
    v, st = isa_check.scan(_dis(lines))
    assert st["kernels"] == 1
    return [i for _k, i, _ld in v]


def test_straight_line():
    assert _bad(["ds_read_b128 v[0:3], v10", "v_mov_b32_e32 v4, v1", "s_endpgm"]) == ["v_mov_b32_e32 v4, v1"]
    assert _bad(["ds_read_b128 v[0:3], v10", "s_waitcnt lgkmcnt(0)", "v_mov_b32_e32 v4, v1", "s_endpgm"]) == []


def test_counted_wait_retires_the_oldest():
    prog = ["ds_read_b128 v[0:3], v10", "ds_read_b128 v[4:7], v11", "s_waitcnt lgkmcnt(1)",
            "v_mov_b32_e32 v8, v0", "v_mov_b32_e32 v9, v4", "s_endpgm"]
    assert _bad(prog) == ["v_mov_b32_e32 v9, v4"]


def test_wait_inside_a_branch_does_not_cover_the_other_path():
    prog = ["ds_read_b128 v[0:3], v10", "s_cbranch_scc1 J", "s_waitcnt lgkmcnt(0)", "J:",
            "v_mov_b32_e32 v4, v0", "s_endpgm"]
    assert _bad(prog) == ["v_mov_b32_e32 v4, v0"]
    both = ["ds_read_b128 v[0:3], v10", "s_cbranch_scc1 L", "s_waitcnt lgkmcnt(0)", "s_branch J", "L:",
            "s_waitcnt lgkmcnt(0)", "J:", "v_mov_b32_e32 v4, v0", "s_endpgm"]
    assert _bad(both) == []


def test_copy_after_a_branch_local_wait():
    """The round-4 ADVICE case: reads in flight across `if (any) { ...; s_waitcnt lgkmcnt(0) }`, and a
    copy after the join but before the retiring wait -- wrong on the no-hit path."""
    prog = ["ds_read_b128 v[0:3], v10", "s_cbranch_vccz J", "v_add_u32_e32 v20, v21, v22",
            "s_waitcnt lgkmcnt(0)", "ds_write_b32 v23, v20", "J:", "v_mov_b32_e32 v30, v2",
            "s_waitcnt lgkmcnt(0)", "s_endpgm"]
    assert _bad(prog) == ["v_mov_b32_e32 v30, v2"]


def test_loop_back_edge():
    prog = ["L:", "v_mov_b32_e32 v4, v0", "ds_read_b128 v[0:3], v10", "s_cbranch_scc1 L",
            "s_waitcnt lgkmcnt(0)", "s_endpgm"]
    assert _bad(prog) == ["v_mov_b32_e32 v4, v0"]


def test_scalar_loads_do_not_retire_ds_reads():
    prog = ["ds_read_b128 v[0:3], v10", "s_load_dword s0, s[2:3], 0x0", "s_waitcnt lgkmcnt(1)",
            "v_mov_b32_e32 v4, v0", "s_endpgm"]
    assert _bad(prog) == ["v_mov_b32_e32 v4, v0"]


def test_agpr_destinations_and_ds_address_reuse():
    prog = ["ds_read_b128 a[0:3], v10", "v_accvgpr_read_b32 v4, a2", "s_endpgm"]
    assert _bad(prog) == ["v_accvgpr_read_b32 v4, a2"]
    prog = ["ds_read_b128 v[0:3], v10", "ds_read_b128 v[4:7], v1", "s_waitcnt lgkmcnt(0)", "s_endpgm"]
    assert _bad(prog) == ["ds_read_b128 v[4:7], v1"]


def test_stats_count_kernels_and_loads():
    v, st = isa_check.scan(_dis(["ds_read_b32 v0, v1", "ds_add_rtn_u32 v2, v3, v4", "ds_write_b32 v5, v6",
                                 "s_waitcnt lgkmcnt(0)", "s_endpgm"]))
    assert v == [] and st == {"kernels": 1, "ds_loads": 2}
