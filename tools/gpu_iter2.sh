#!/bin/bash
# Iteration pass (run on the GPU box via gpurun): selected -m gpu test files, then tools/gpu_sweep.sh.
#   TESTS="tests/a.py tests/b.py"  (+ gpu_sweep.sh variables)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-iter}
mkdir -p $OUT
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_T:-400} python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest.log; exit 1; }
  tail -1 $OUT/pytest.log
fi
bash tools/gpu_sweep.sh
