#!/bin/bash
# Round 6: K1s<4,4> (one wave per SIMD, spread row-set switch) and the per-block stage flush.
# 1) GPU tests of the release build (the K1s<2,8> flush changed); 2) exactness of the A/B builds;
# 3) MATRIX-stage A/B: 100M x 1024 clustered (K1m vs K1s<4,4> spread / unspread), 1M / 4M x 1024 (K1s<2,8> vs <4,4>)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r6k1s}
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 ${T1:-600} python -u -m pytest ${TESTS:-tests/test_gpu_lists.py tests/test_gpu_mfma.py tests/test_gpu_k1m_edges.py} \
  tests/test_gpu_fullsize.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 \
  || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
fi
for v in ${CHECK:-L S}; do
  timeout -k 10 300 python -u tools/with_lib.py tools/ab/lib_$v.so tools/k1s_check.py > $OUT/check_$v.jsonl 2>&1 \
    || { tail -20 $OUT/check_$v.jsonl; exit 1; }
  cat $OUT/check_$v.jsonl
done
timeout -k 10 ${T2:-500} python -u tools/stage_bench.py --clustered --cases ${BIG:-100000000:1024} \
  --libs vectorragquantization_amd/libvrq.so${BIGLIBS:-,tools/ab/lib_L.so,tools/ab/lib_LN.so} --reps 5 --rounds 4 \
  > $OUT/ab_big.jsonl 2>&1 || { tail -20 $OUT/ab_big.jsonl; exit 1; }
cat $OUT/ab_big.jsonl
timeout -k 10 ${T3:-300} python -u tools/stage_bench.py --cases ${SMALL:-1000000:1024,4000000:1024,12500000:1024} \
  --libs vectorragquantization_amd/libvrq.so${SMALLLIBS:-,tools/ab/lib_S.so,tools/ab/lib_L.so} --reps 5 --rounds 4 \
  > $OUT/ab_small.jsonl 2>&1 || { tail -20 $OUT/ab_small.jsonl; exit 1; }
cat $OUT/ab_small.jsonl
