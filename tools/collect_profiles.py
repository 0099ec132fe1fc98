#!/usr/bin/env python
"""Copy the rocprofv3 results of a tools/prof_r3.sh run (gpurun_out/<TAG>/<config>_nq<nq>/) into the
committed profiles/ directory under the names bench.py looks up:
  profiles/<round>_<config>_n<rows>_nq<nq>_g1_kernel_stats.csv   (kernel-trace --stats summary)
  profiles/<round>_<config>_n<rows>_nq<nq>_g1_pmc.json           (tools/summarize_profile.py summary)
  profiles/<round>_<config>_n<rows>_nq<nq>_g1_dispatch.json      (tools/trace_dispatches.py summary)
Usage: collect_profiles.py <round, e.g. r3> <gpurun_out/TAG> [--n config=rows ...]"""
import glob
import os
import shutil
import sys

ROWS = {"c2": 1_000_000, "c3": 100_000_000, "c4": 100_000_000, "c5": 10_000_000}


def main(rnd, src, overrides):
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    rows = dict(ROWS, **{k: int(v) for k, v in (o.split("=") for o in overrides)})
    for d in sorted(glob.glob(os.path.join(src, "c*_nq*"))):
        cfg, nq = os.path.basename(d).split("_nq")
        tag = f"{rnd}_{cfg}_n{rows[cfg]}_nq{nq}_g1"
        stats = glob.glob(os.path.join(d, "kernel_stats.csv")) or \
            glob.glob(os.path.join(d, "trace", "**", "*kernel_stats.csv"), recursive=True)
        if stats:
            shutil.copy(stats[0], os.path.join(here, "profiles", f"{tag}_kernel_stats.csv"))
        disp = os.path.join(d, "dispatch.json")
        if os.path.exists(disp):
            shutil.copy(disp, os.path.join(here, "profiles", f"{tag}_dispatch.json"))
        summ = os.path.join(d, "summary.json")
        if os.path.exists(summ):
            shutil.copy(summ, os.path.join(here, "profiles", f"{tag}_pmc.json"))
        print(tag, "stats" if stats else "-", "summary" if os.path.exists(summ) else "-")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3:])
