#!/bin/bash
# SQ counters of hamming_mfma_kernel alone (mfma_bisect_0) at two thresholds: no hits (440) and
# the 1M-row hit rate (465).  Run on the GPU box; writes gpurun_out/pmc_bisect/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_bisect
mkdir -p $OUT
for tau in 440 465; do
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $OUT/a_$tau -o run --output-format csv -- ./tools/probes/mfma_bisect_0 1000000 1024 $tau > $OUT/a_$tau.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES -d $OUT/b_$tau -o run --output-format csv -- ./tools/probes/mfma_bisect_0 1000000 1024 $tau > $OUT/b_$tau.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob, collections
for tau in (440, 465):
    agg = collections.defaultdict(float); cnt = collections.defaultdict(int)
    for f in glob.glob(f"gpurun_out/pmc_bisect/*_{tau}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "hamming_mfma" in r["Kernel_Name"]:
                agg[r["Counter_Name"]] += float(r["Counter_Value"]); cnt[r["Counter_Name"]] += 1
    print(tau, {k: round(v / cnt[k]) for k, v in sorted(agg.items())})
PY
