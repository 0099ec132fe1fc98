#!/bin/bash
# Round-2 GPU pass (run via gpurun): optional -m gpu tests, then the default bench line
# (config 4, 100M rows) and optional extra bench configs.  Each GPU step is time-limited and
# the chain stops at the first failure.
#   TAG=name  TESTS=1|0  TEST_ARGS="..."  BENCHES="c4 c2 c3 c5"  BENCH_EXTRA="..."
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r2}
mkdir -p $OUT
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${TEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -60 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
for c in ${BENCHES:-c4}; do
  timeout -k 10 ${BENCH_T:-600} python -u bench.py --config $c ${BENCH_EXTRA:-} > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { echo BENCH_FAIL $c; tail -30 $OUT/bench_$c.err; exit 1; }
  python -c "
import json;d=json.load(open('$OUT/bench_$c.json'))
print('$c', 'QPS', round(d['value']), 'ms/step', round(d['ms_per_step'],3), {k:round(v,4) for k,v in d['phase_ms'].items()}, 'frac', round(d['roofline']['frac'],3), 'recall', d.get('recall_at_10'))
for key in ('cpu_baseline','cpu_gpu_top10_identical','cpu_gpu_identity','real_data'):
    if key in d: print(key, json.dumps(d[key])[:600])
if 'roofline_encode' in d: print({m:round(v['frac'],3) for m,v in d['roofline_encode']['modes'].items()})
"
done
echo done
