#!/bin/bash
# Profiling pass for round 1 (run on the GPU box via gpurun). Each GPU step is time-limited.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${PROF_TAG:-prof_r1}
mkdir -p $OUT
BARGS="${BENCH_ARGS:-}"
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -k 10 300 python tools/scan_bench.py > $OUT/scan_bench.jsonl 2> $OUT/scan_bench.err || exit 1
timeout -k 10 60 ./tools/probes/mfma_rate_probe > $OUT/mfma_rate.jsonl 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-recall $BARGS > $OUT/bench_trace.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS -d $OUT/pmc_sq -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-recall $BARGS > $OUT/bench_pmc_sq.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F6F4 SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $OUT/pmc_mfma -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-recall $BARGS > $OUT/bench_pmc_mfma.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-recall $BARGS > $OUT/bench_pmc_fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-recall $BARGS > $OUT/bench_pmc_write.log 2>&1 || exit 1
echo done
