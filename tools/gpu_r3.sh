#!/bin/bash
# Round-3 GPU pass (run via gpurun): optional -m gpu tests + smoke, bench lines, optional K5 probe
# variants (tools/probes/g5/lib_*.so via tools/gemm_probe.py).  Each GPU step has its own time limit
# and the chain stops at the first failure.
#   TAG=name TESTS=1|0 TEST_K="pytest -k expression" BENCHES="c4 c2 c3 c5" BENCH_EXTRA="..." G5LIBS="a,b" G5ARGS="..."
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r3}
mkdir -p $OUT
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 720 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${TEST_K:+-k "$TEST_K"} > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -60 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
if [ -n "${G5LIBS:-}" ]; then
  VRQ_LIBS=$G5LIBS timeout -k 10 400 python -u tools/gemm_probe.py ${G5ARGS:---n 10000000 --stages 16,32} > $OUT/g5_probe.jsonl 2> $OUT/g5_probe.err || { echo G5_FAIL; tail -20 $OUT/g5_probe.err; exit 1; }
  cat $OUT/g5_probe.jsonl
fi
if [ -n "${ENCLIBS:-}" ]; then
  VRQ_LIBS=$ENCLIBS timeout -k 10 300 python -u tools/enc_probe.py > $OUT/enc_probe.jsonl 2> $OUT/enc_probe.err || { echo ENC_FAIL; tail -20 $OUT/enc_probe.err; exit 1; }
  cat $OUT/enc_probe.jsonl
fi
for c in ${BENCHES:-}; do
  timeout -k 10 ${BENCH_T:-600} python -u bench.py --config $c ${BENCH_EXTRA:-} > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { echo BENCH_FAIL $c; tail -30 $OUT/bench_$c.err; exit 1; }
  python -c "
import json;d=json.load(open('$OUT/bench_$c.json'))
print('$c', 'QPS', round(d['value']), 'ms/step', round(d['ms_per_step'],3), {k:round(v,4) for k,v in d['phase_ms'].items()}, 'frac', round(d['roofline']['frac'],3), 'recall', d.get('recall_at_10'))
for key in ('cpu_baseline','cpu_gpu_top10_identical','cpu_gpu_identity','real_data'):
    if key in d: print(key, json.dumps(d[key])[:600])
if 'roofline_encode' in d: print({m:round(v['frac'],3) for m,v in d['roofline_encode']['modes'].items()})
"
done
# VARIANTS="name=lib.so:config ...": the same bench line on another build of the library (VRQ_LIB)
for spec in ${VARIANTS:-}; do
  nm=${spec%%=*}; rest=${spec#*=}; lib=${rest%%:*}; c=${rest#*:}
  VRQ_LIB=$lib timeout -k 10 ${BENCH_T:-600} python -u bench.py --config $c --no-cpu-baseline --no-recall --no-encode ${BENCH_EXTRA:-} > $OUT/var_${nm}_$c.json 2> $OUT/var_${nm}_$c.err || { echo VAR_FAIL $nm; tail -30 $OUT/var_${nm}_$c.err; exit 1; }
  python -c "
import json;d=json.load(open('$OUT/var_${nm}_$c.json'))
print('variant $nm $c', 'QPS', round(d['value']), 'ms/step', round(d['ms_per_step'],3), {k:round(v,4) for k,v in d['phase_ms'].items()})
"
done
echo done
