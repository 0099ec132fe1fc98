#!/bin/bash
# GPU pass for the config-2 bench (run on the GPU box via gpurun): parity tests, the bench line
# with the CPU baseline, one kernel-trace --stats run and the separate --pmc passes that
# tools/summarize_profile.py condenses into profiles/.  Each GPU step is time-limited.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${PROF_TAG:-prof_c2}
mkdir -p $OUT
BARGS="${BENCH_ARGS:-}"
PB="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-recall $BARGS"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
fi
timeout -k 10 400 python3 bench.py $BARGS > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAIL; tail -20 $OUT/bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-recall $BARGS > $OUT/bench_trace.log 2>&1 || { echo TRACE_FAIL; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS -d $OUT/pmc_sq -o run --output-format csv -- $PB > $OUT/bench_pmc_sq.log 2>&1 || { echo PMC_FAIL; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F6F4 SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $OUT/pmc_mfma -o run --output-format csv -- $PB > $OUT/bench_pmc_mfma.log 2>&1 || { echo PMC_FAIL; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- $PB > $OUT/bench_pmc_fetch.log 2>&1 || { echo PMC_FAIL; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- $PB > $OUT/bench_pmc_write.log 2>&1 || { echo PMC_FAIL; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('QPS',round(d['value']),{k:round(v,4) for k,v in d['phase_ms'].items()},d['roofline']['frac'],d.get('cpu_baseline'))"
echo done
