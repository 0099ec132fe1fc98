#!/usr/bin/env python
"""Condense rocprofv3 outputs (kernel-trace stats CSV + separate --pmc passes) into the JSON
summaries committed under profiles/ (per round), incl. per-launch HBM traffic of the scan
kernel corrected as MI355X_MICROARCH.md prescribes (gfx950 FETCH_SIZE reads 1/2 of the bytes
of 16-B-per-lane streams -> x2; WRITE_SIZE exact for 16-B stores; both in KiB)."""
import collections
import csv
import glob
import json
import os
import sys


def short(name):
    if "hamming_mfma_rows" in name:  # K1r (and its lean MB = 2 form), template MODE as below
        mode = name.split("_kernel<", 1)[-1][:1]
        return {"1": "hamming_mfma_rows_kernel_sample", "2": "hamming_mfma_rows_kernel_rerun"}.get(
            mode, "hamming_mfma_rows_kernel")
    if "hamming_mfma_swap" in name:  # K1s, the large-batch thresholded pass (MODE 0) and its re-run (2)
        mode = name.split("_swap_kernel<", 1)[-1][:1]
        return "hamming_mfma_kernel_rerun" if mode == "2" else "hamming_mfma_kernel"
    if "hamming_mfma" in name:  # template MODE: 0 thresholded pass, 1 dense sample pass, 2 re-run
        return {"1": "hamming_mfma_kernel_sample", "2": "hamming_mfma_kernel_rerun"}.get(
            name.split("hamming_mfma_kernel<", 1)[-1][:1], "hamming_mfma_kernel")
    if "gemm_topk_kernel" in name:  # <PH, DENSE>: PH 3 = int8 cosine, 2 = binary
        t = name.split("gemm_topk_kernel<", 1)[-1]
        base = "gemm_topk_kernel" if t.startswith("3") else "gemm_topk_kernel_binary"
        targs = [x.strip() for x in t.split(">")[0].split(",")]  # PH, DENSE[, RETRY]
        if len(targs) > 2 and targs[2] == "true":
            return base + "_retry"
        return base + ("_sample" if targs[1:2] == ["true"] else "")
    for nm in ("gemm_select_kernel", "gemm_finish_kernel", "gemm_fallback_kernel", "gemm_prep_kernel"):
        if nm in name:
            return nm + ("_binary" if "<2>" in name else "")
    if "sample_select" in name:
        return "sample_select_kernel"
    if "sample_check" in name:
        return "sample_check_kernel"
    if "prefix_tau" in name:
        return "prefix_tau_kernel"
    if "suffix_topk" in name:
        return "suffix_topk_kernel"
    if "hamming_scan" in name:
        return "hamming_scan_kernel"
    if "select_rescore" in name:
        return "select_rescore_kernel"
    if "merge_shards" in name:
        return "merge_shards_kernel"
    if "encode_kernel" in name:
        return "encode_kernel"
    return name[:60]


def pmc(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} | {"dispatches": len(next(iter(d.values())))}
            for k, d in agg.items()}


def main(src, dst, tag):
    out = {"tag": tag, "source": src}
    stats = glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        out["kernel_stats"] = [r for r in csv.DictReader(open(stats[0]))]
    for name in ("pmc_sq", "pmc_mfma", "pmc_v", "pmc_fetch", "pmc_write", "pmc_clk"):
        f = glob.glob(os.path.join(src, name, "**", "*counter_collection.csv"), recursive=True)
        if f:
            out[name] = pmc(f[0])
    # per-launch HBM bytes of every kernel seen by both traffic passes
    out["bytes_per_launch"] = {}
    for k in out.get("pmc_fetch", {}):
        try:
            fetch = out["pmc_fetch"][k]["FETCH_SIZE"] * 1024 * 2
            write = out["pmc_write"][k]["WRITE_SIZE"] * 1024
        except KeyError:
            continue
        out["bytes_per_launch"][k] = fetch + write
    # effective shader clock under load (GRBM_GUI_ACTIVE is the sum over the 8 XCDs) and the
    # matrix-core busy fraction (SQ_VALU_MFMA_BUSY_CYCLES sums MFMA cycles over all 1024 SIMDs).  The
    # duration is the per-dispatch mean after the warm-up steps (dispatch.json of the same run:
    # tools/trace_dispatches.py) -- not the --stats average, which includes cold launches -- and a clock
    # is reported only for kernels of >= 50 us and at most the 2.4 GHz maximum sclk (+5 %): shorter
    # launches and their counter start/stop overheads give meaningless ratios.
    dur_ns = {}
    disp = os.path.join(src, "dispatch.json")
    if os.path.exists(disp):
        for name, v in json.load(open(disp)).get("kernels", {}).items():
            dur_ns.setdefault(short(name), float(v["mean_after_warmup_ms"]) * 1e6)
    out["clock"] = {}
    for k, c in out.get("pmc_clk", {}).items():
        cyc = c.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        if cyc <= 0:
            continue
        d = {"cycles_per_xcd": cyc, "mfma_busy_frac": c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (1024.0 * cyc)}
        ns = dur_ns.get(k)
        if ns and ns >= 50e3:
            clk = cyc / ns
            if clk <= 2.4 * 1.05:
                d["eff_clock_ghz"] = clk
                d["duration_ns"] = ns
            else:
                d["eff_clock_invalid"] = clk
        out["clock"][k] = d
    if "hamming_scan_kernel" in out["bytes_per_launch"]:
        out["scan_bytes_per_launch"] = out["bytes_per_launch"]["hamming_scan_kernel"]
    json.dump(out, open(dst, "w"), indent=1)
    print("wrote", dst)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3])
