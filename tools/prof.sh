#!/bin/bash
# Profiling pass (run on the GPU box via gpurun): for each "config:nq" in RUNS, a rocprofv3
# --kernel-trace --stats run of the bench line (the same command and step counts as the event-timed
# line), condensed into kernel_stats.csv (every launch) and dispatch.json (tools/trace_dispatches.py:
# the launches after the warm-up steps); then (PMC=1) separate FETCH_SIZE and WRITE_SIZE passes (one
# counter block per pass, MI355X_MICROARCH.md), condensed by tools/summarize_profile.py into
# gpurun_out/$TAG/<config>_nq<nq>/summary.json.  tools/collect_profiles.py copies them into profiles/.
# Each GPU step is time-limited; the chain stops at the first failure.
#   RUNS="c3:1 c3:8 c3:64 c2:1024 c4:1024 c5:1024"  TAG=name  PMC=1|0  SQ=0|1  CLK=0|1  STEPS=20 WARMUP=3
#   BARGS="extra bench args"
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
S=${STEPS:-20}; W=${WARMUP:-3}
for run in ${RUNS:-c3:8}; do
  CFG=${run%%:*}; NQ=${run#*:}
  OUT=gpurun_out/${TAG:-prof}/${CFG}_nq${NQ}
  mkdir -p $OUT
  B="--config $CFG --nq $NQ --no-cpu-baseline --no-recall --no-encode --no-phase1 ${BARGS:-}"
  timeout -k 10 ${PT:-400} rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps $S --warmup $W $B > $OUT/bench_trace.json 2> $OUT/bench_trace.err || { echo TRACE_FAIL $run; tail -20 $OUT/bench_trace.err; exit 1; }
  python3 tools/trace_dispatches.py $OUT/trace $OUT/dispatch.json --warmup $W --command "python3 bench.py --steps $S --warmup $W $B" > $OUT/dispatch.txt
  if [ "${PMC:-1}" = "1" ]; then
    timeout -k 10 ${PT:-400} rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 $B > $OUT/pmc_fetch.log 2>&1 || { echo FETCH_FAIL $run; tail -20 $OUT/pmc_fetch.log; exit 1; }
    timeout -k 10 ${PT:-400} rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 $B > $OUT/pmc_write.log 2>&1 || { echo WRITE_FAIL $run; tail -20 $OUT/pmc_write.log; exit 1; }
  fi
  if [ "${SQ:-0}" = "1" ]; then  # one SQ pass (<= 8 SQ counters): wait / busy / MFMA-busy fractions
    timeout -k 10 ${PT:-400} rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA -d $OUT/pmc_sq -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 $B > $OUT/pmc_sq.log 2>&1 || { echo SQ_FAIL $run; tail -20 $OUT/pmc_sq.log; exit 1; }
  fi
  if [ "${CLK:-0}" = "1" ]; then  # effective clock and matrix-core busy fraction (MI355X_MICROARCH.md DVFS notes)
    timeout -k 10 ${PT:-400} rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES -d $OUT/pmc_clk -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 $B > $OUT/pmc_clk.log 2>&1 || { echo CLK_FAIL $run; tail -20 $OUT/pmc_clk.log; exit 1; }
  fi
  python3 tools/summarize_profile.py $OUT $OUT/summary.json ${CFG}_nq${NQ} > /dev/null
  # keep the condensed results only (the raw per-dispatch CSVs of a 100M-row run exceed gpurun's 64 MiB)
  cp "$(find $OUT/trace -name '*kernel_stats.csv' | head -1)" $OUT/kernel_stats.csv
  rm -rf $OUT/trace $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_sq $OUT/pmc_clk
  echo "== $run"; cat $OUT/dispatch.txt
  python3 -c "import json; print('   events', json.load(open('$OUT/bench_trace.json'))['phase_ms'])"
done
echo done
