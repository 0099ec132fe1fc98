#!/bin/bash
# PMC + kernel-trace passes of the config-5 bench (run on the GPU box via gpurun)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-prof_c5}
mkdir -p $OUT
B="python3 bench.py --config c5 --steps ${STEPS:-1} --warmup 1 --no-cpu-baseline --no-recall ${BENCH_ARGS:-}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $B > $OUT/trace.log 2>&1 || { echo TRACE_FAIL; tail $OUT/trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d $OUT/pmc_sq -o run --output-format csv -- $B > $OUT/pmc_sq.log 2>&1 || { echo PMC_FAIL; tail $OUT/pmc_sq.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE -d $OUT/pmc_v -o run --output-format csv -- $B > $OUT/pmc_v.log 2>&1 || { echo PMC_FAIL; tail $OUT/pmc_v.log; exit 1; }
if [ -n "$TRAFFIC" ]; then
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- $B > $OUT/pmc_fetch.log 2>&1 || { echo PMC_FAIL; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- $B > $OUT/pmc_write.log 2>&1 || { echo PMC_FAIL; exit 1; }
fi
python3 - <<PY
import csv, glob, collections
f = glob.glob("$OUT/trace/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "vrq" in r["Name"]:
        print(f'{r["Name"].split("(")[0][:70]:70s} calls {r["Calls"]:>4s} avg_us {float(r["AverageNs"])/1e3:10.2f}')
for d in ("pmc_sq", "pmc_v"):
    g = glob.glob(f"$OUT/{d}/**/*counter_collection.csv", recursive=True)
    if not g: continue
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.defaultdict(set)
    for r in csv.DictReader(open(g[0])):
        if "gemm_topk_kernel" in r["Kernel_Name"]:
            k = r["Kernel_Name"].split("(")[0][-40:]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[k].add(r["Dispatch_Id"])
    for k, v in agg.items():
        print(d, k, len(cnt[k]), {c: f"{x/len(cnt[k]):.4g}" for c, x in v.items()})
PY
if [ -n "$TRAFFIC" ]; then python3 - <<PY
import csv, glob, collections
for d in ("pmc_fetch", "pmc_write"):
    g = glob.glob(f"$OUT/{d}/**/*counter_collection.csv", recursive=True)
    agg = collections.defaultdict(float); ids = collections.defaultdict(set)
    for r in csv.DictReader(open(g[0])):
        if "gemm" in r["Kernel_Name"]:
            k = r["Kernel_Name"].split("(")[0][-40:]
            agg[k] += float(r["Counter_Value"]); ids[k].add(r["Dispatch_Id"])
    for k in agg: print(d, k, f"{agg[k] / len(ids[k]) * 1024 / 1e9:.3f} GB per launch (raw KiB counter x1024)")
PY
fi
