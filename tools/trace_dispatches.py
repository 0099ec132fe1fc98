#!/usr/bin/env python
"""Condense a rocprofv3 --kernel-trace per-dispatch CSV into the per-kernel JSON summary bench.py reads
(profiles/r<round>_<tag>_dispatch.json): for every vrq kernel, its launch count and the mean duration of
the launches after the bench's `warmup` untimed steps -- the launches its HIP events time -- beside the
mean of all launches, the median, the minimum and the first (cold) launch.

Usage: trace_dispatches.py <rocprofv3 output dir> <out.json> --warmup W [--per-step P]
  P = launches of each kernel per bench step (default 1): the first W * P launches are skipped."""
import argparse
import csv
import glob
import json
import statistics
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("dst")
    ap.add_argument("--warmup", type=int, required=True)
    ap.add_argument("--per-step", type=int, default=1)
    ap.add_argument("--command", default="")
    a = ap.parse_args()
    files = glob.glob(f"{a.src}/**/*kernel_trace.csv", recursive=True)
    if not files:
        sys.exit(f"no kernel_trace.csv under {a.src}")
    rows = []
    for f in files:
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if "vrq::" in name:
                rows.append((int(r["Start_Timestamp"]), name.split("(")[0],
                             int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    rows.sort()
    by = {}
    for _, k, d in rows:
        by.setdefault(k, []).append(d / 1e6)
    skip = a.warmup * a.per_step
    out = {"source": "rocprofv3 --kernel-trace per-dispatch durations", "command": a.command, "warmup": a.warmup,
           "per_step": a.per_step, "kernels": {}}
    for k, v in by.items():
        tail = v[skip:] or v
        out["kernels"][k] = {"n": len(v), "n_after_warmup": len(tail), "mean_after_warmup_ms": statistics.mean(tail),
                             "mean_all_ms": statistics.mean(v), "median_ms": statistics.median(tail),
                             "min_ms": min(tail), "first_ms": v[0]}
        print(f"{k[:70]:70s} n={len(v):4d} mean_after_warmup={statistics.mean(tail):.4f} ms "
              f"mean_all={statistics.mean(v):.4f} first={v[0]:.4f}")
    json.dump(out, open(a.dst, "w"), indent=1)


if __name__ == "__main__":
    main()
