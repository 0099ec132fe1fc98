#!/bin/bash
# K1m pin change: new full-shape tests (c2 1M x 1024, K5 flood), the matrix-core and fullsize tests, c4 and c2 lines.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4f; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_mfma.py tests/test_gpu_gemm.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u bench.py --no-phase1 --no-cpu-baseline > $O/c4.json 2> $O/c4.err || { echo C4_FAIL; tail -20 $O/c4.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/c4.json')); r=d['roofline']; print('c4', round(d['value']), 'QPS', round(d['ms_per_step'],3), 'ms matrix', round(r['kernel_ms'],3), 'frac', round(r['frac'],3))"
timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline > $O/c2.json 2> $O/c2.err || { echo C2_FAIL; tail -20 $O/c2.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/c2.json')); r=d['roofline']; print('c2', round(d['value']), 'QPS', round(d['ms_per_step'],4), 'ms matrix', round(r['kernel_ms'],4), 'frac', round(r['frac'],3), d.get('phase_ms'))"
