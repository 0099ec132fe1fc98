#!/bin/bash
# SQ / GRBM counter passes of a short bench run (run on the GPU box via gpurun), one rocprofv3
# --pmc pass per counter group (hardware limits: <= 8 SQ, <= 2 GRBM per pass), each
# time-limited; the chain stops at the first failure.  tools/summarize_profile.py condenses them.
#   CFG=c4  TAG=name  BARGS="extra bench args"
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
CFG=${CFG:-c4}
OUT=gpurun_out/${TAG:-pmc_$CFG}
mkdir -p $OUT
B="--config $CFG --no-cpu-baseline --no-recall --no-encode --steps 2 --warmup 1 ${BARGS:-}"
[ -f $OUT/counters.txt ] || timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" ${EXTRA_PASSES:+"$EXTRA_PASSES"}; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $OUT/pmc_p$i -o run --output-format csv -- python3 bench.py $B > $OUT/pmc_p$i.log 2>&1 || { echo PMC_FAIL $i; tail -5 $OUT/pmc_p$i.log; exit 1; }
done
python3 - <<PY
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("$OUT/pmc_p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "hamming_mfma_kernel<0>" in n or "gemm_topk_kernel" in n or "hamming_scan" in n:
            key = n.split("(")[0][-40:]
            agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
            if r.get("Start_Timestamp") and r.get("End_Timestamp"):
                agg[key]["dur_ns"].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
for k, d in agg.items():
    print(k, {c: round(sum(v) / len(v)) for c, v in sorted(d.items())})
PY
echo done
