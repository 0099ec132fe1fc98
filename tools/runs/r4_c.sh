#!/bin/bash
# K1r change check: the matrix-core scan tests, then config-3 lines at nq 1 / 8 / 32 / 64 / 128.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r4c}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for nq in ${NQS:-1 8 32 64 128}; do
  timeout -k 10 300 python -u bench.py --config c3 --nq $nq --steps 20 --warmup 3 --no-cpu-baseline > $O/c3_nq$nq.json 2> $O/c3_nq$nq.err || { echo BENCH_FAIL $nq; tail -20 $O/c3_nq$nq.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/c3_nq$nq.json')); r=d['roofline']; print('nq $nq', 'matrix', round(r['kernel_ms'],4), 'frac', round(r['frac'],3), 'mfma', round(r['mfma']['frac'],3), 'step', round(d['ms_per_step'],3))"
done
