#!/bin/bash
# Round-2 profiling pass (run on the GPU box via gpurun): rocprofv3 kernel-trace stats of a short
# bench run of one --config, then separate FETCH_SIZE / WRITE_SIZE PMC passes (MI355X_MICROARCH.md:
# one counter block per pass), condensed by tools/summarize_profile.py.  Each GPU step is
# time-limited and the chain stops at the first failure.
#   CFG=c4|c2|c3|c5  TAG=name  BARGS="extra bench args"  PMC=1|0
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
CFG=${CFG:-c4}
OUT=gpurun_out/${TAG:-prof_$CFG}
mkdir -p $OUT
B="--config $CFG --no-cpu-baseline --no-recall --no-encode ${BARGS:-}"
timeout -k 10 ${PT:-400} rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 5 --warmup 1 $B > $OUT/bench_trace.json 2> $OUT/bench_trace.err || { echo TRACE_FAIL; tail -20 $OUT/bench_trace.err; exit 1; }
if [ "${PMC:-1}" = "1" ]; then
  timeout -k 10 ${PT:-400} rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 $B > $OUT/pmc_fetch.log 2>&1 || { echo FETCH_FAIL; tail -20 $OUT/pmc_fetch.log; exit 1; }
  timeout -k 10 ${PT:-400} rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 $B > $OUT/pmc_write.log 2>&1 || { echo WRITE_FAIL; tail -20 $OUT/pmc_write.log; exit 1; }
fi
python3 tools/summarize_profile.py $OUT $OUT/summary.json ${TAG:-prof_$CFG} > /dev/null
python3 - <<PY
import json
d = json.load(open("$OUT/summary.json"))
for r in d.get("kernel_stats", []):
    n = r["Name"]
    if float(r["Percentage"]) > 0.2:
        print(f'{n.split("(")[0][:70]:70s} calls {r["Calls"]:>5s} avg_us {float(r["AverageNs"])/1e3:10.2f} tot% {float(r["Percentage"]):.1f}')
print({k: round(v / 1e6, 1) for k, v in d.get("bytes_per_launch", {}).items()}, "MB/launch")
PY
echo done
