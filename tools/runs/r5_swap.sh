#!/bin/bash
# K1s (role-swapped large-batch pass): list/instance tests, then the matrix-stage A/B against K1m.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r5swap}
mkdir -p $OUT
timeout -k 10 ${T1:-500} python -u -m pytest tests/test_gpu_lists.py tests/test_gpu_mfma.py -m gpu -x -v --timeout 300 \
  --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 ${T2:-400} python -u tools/stage_bench.py --cases ${CASES:-100000000:1024,1000000:1024,4000000:1024,100000000:512} \
  --libs vectorragquantization_amd/libvrq.so,${BASE:-tools/probes/var/lib_k1m_r5.so}${EXTRA:-} --reps 5 --rounds 4 > $OUT/ab.jsonl 2>&1 || { tail -20 $OUT/ab.jsonl; exit 1; }
cat $OUT/ab.jsonl
