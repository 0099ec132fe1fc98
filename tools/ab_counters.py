#!/usr/bin/env python
"""Condense tools/ab_counters.sh output: one JSON line per (library, kernel) for the kernels that take
>= 50 us per launch, with the per-dispatch mean duration (kernel-trace pass, first launch dropped), the
mean of every counter over that kernel's dispatches, and the derived fractions:
  eff_clock_ghz   = GRBM_GUI_ACTIVE / 8 XCDs / duration
  mfma_busy       = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x those cycles)
  wait_any / wait_inst / active = SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES
  wait_inst_lds   = SQ_WAIT_INST_LDS over SQ_WAVE_CYCLES (pass 'lds'; its own SQ_WAVE_CYCLES is not in
                    that pass, so the 'sq' pass's is used)
  lds_conflict    = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  lds_active_per_busy = SQ_LDS_IDX_ACTIVE / SQ_BUSY_CYCLES (relative LDS-array load; compare builds)
Usage: ab_counters.py gpurun_out/<TAG>"""
import collections
import csv
import glob
import json
import os
import statistics
import sys


def kname(full):
    return full.split("(")[0].replace("void ", "")


def counters(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "vrq::" in r["Kernel_Name"]:
                agg[kname(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: statistics.mean(v) for c, v in cs.items()} for k, cs in agg.items()}


def durations(d):
    by = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
        for r in rows:
            if "vrq::" in r["Kernel_Name"]:
                by[kname(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return {k: (statistics.mean(v[1:]) if len(v) > 1 else v[0], len(v)) for k, v in by.items()}


def main(src):
    for libdir in sorted(glob.glob(os.path.join(src, "lib*"))):
        lib = open(os.path.join(libdir, "lib.txt")).read().strip()
        dur = durations(os.path.join(libdir, "trace"))
        cs = {p: counters(os.path.join(libdir, p)) for p in ("clk", "sq", "lds")}
        for k, (us, n) in sorted(dur.items(), key=lambda kv: -kv[1][0]):
            if us < 50:
                continue
            clk, sq, lds = cs["clk"].get(k, {}), cs["sq"].get(k, {}), cs["lds"].get(k, {})
            line = {"lib": os.path.basename(lib), "kernel": k, "launches": n, "us": round(us, 2)}
            cyc = clk.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
            if cyc > 0:
                line["eff_clock_ghz"] = round(cyc / (us * 1e3), 3)
                line["mfma_busy"] = round(clk.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (1024.0 * cyc), 3)
            wc = sq.get("SQ_WAVE_CYCLES", 0.0)
            if wc > 0:
                for key, c in (("wait_any", "SQ_WAIT_ANY"), ("wait_inst", "SQ_WAIT_INST_ANY"),
                               ("active", "SQ_ACTIVE_INST_ANY")):
                    line[key] = round(sq.get(c, 0.0) / wc, 3)
                if "SQ_WAIT_INST_LDS" in lds:
                    line["wait_inst_lds"] = round(lds["SQ_WAIT_INST_LDS"] / wc, 3)
            if lds.get("SQ_LDS_IDX_ACTIVE", 0.0) > 0:
                line["lds_conflict"] = round(lds.get("SQ_LDS_BANK_CONFLICT", 0.0) / lds["SQ_LDS_IDX_ACTIVE"], 4)
                if lds.get("SQ_BUSY_CYCLES", 0.0) > 0:
                    line["lds_active_per_busy"] = round(lds["SQ_LDS_IDX_ACTIVE"] / lds["SQ_BUSY_CYCLES"], 3)
            line["counters"] = {p: cs[p].get(k, {}) for p in cs}
            print(json.dumps(line))


if __name__ == "__main__":
    main(sys.argv[1])
