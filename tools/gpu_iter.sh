#!/bin/bash
# One GPU iteration: parity tests, matrix-kernel bisect probe, bench. Each step time-limited.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-iter}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for b in ${BISECT:-0 1 2 4}; do
  for tau in 440 465; do
    timeout -k 10 60 ./tools/probes/mfma_bisect_$b 10000000 1024 $tau >> $OUT/bisect.jsonl 2>&1 || { echo BISECT_FAIL; cat $OUT/bisect.jsonl; exit 1; }
  done
done
cat $OUT/bisect.jsonl
timeout -k 10 300 python bench.py ${BENCH_ARGS:---no-cpu-baseline} > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAIL; tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print('QPS',d['value'],d['phase_ms'],d['roofline']['frac'])"
