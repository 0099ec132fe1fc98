#!/bin/bash
# Full GPU pass (run via gpurun): every -m gpu test, smoke(), the config-2 bench line (default
# workload, with the CPU baseline) and the config-5 bench line.  Each GPU step is time-limited.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-full}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { echo BENCH2_FAIL; tail -20 $OUT/bench_c2.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_c2.json'));print('c2 QPS',round(d['value']),{k:round(v,4) for k,v in d['phase_ms'].items()},round(d['roofline']['frac'],3),d['recall_at_10'],d['cpu_baseline']['value'],d['cpu_gpu_top10_agreement'])"
if [ -z "$NO_C5" ]; then
timeout -k 10 500 python bench.py --config c5 --steps 5 --warmup 1 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { echo BENCH5_FAIL; tail -20 $OUT/bench_c5.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_c5.json'));print('c5 QPS',round(d['value']),{k:round(v,3) for k,v in d['phase_ms'].items()},round(d['roofline']['frac'],3),d['recall_at_10'],d['cpu_baseline']['value'])"
fi
