#!/bin/bash
# Lean K1r (MB <= 2, two waves per SIMD): candidate lists vs true distances, the matrix-core tests,
# then c3 matrix-pass times of the lean and the previous K1r (variant lib) at nq 1 / 8 / 32 / 64.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4h; mkdir -p $O
for nq in 8 64; do
  timeout -k 10 300 python -u tools/probes/k1r_lists.py --nq $nq --reps 2 > $O/lists_$nq.log 2>&1 || { echo LISTS_FAIL $nq; tail -20 $O/lists_$nq.log; exit 1; }
  echo "nq $nq" $(grep "mismatches" $O/lists_$nq.log | tr '\n' ' ')
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for lib in default old; do
  for nq in ${NQS:-8 64}; do
    if [ $lib = default ]; then P=""; else P="tools/with_lib.py tools/probes/var/lib_old.so"; fi
    timeout -k 10 300 python -u $P bench.py --config c3 --nq $nq --steps 20 --warmup 3 --no-cpu-baseline > $O/c3_${lib}_$nq.json 2> $O/c3_${lib}_$nq.err || { echo BENCH_FAIL $lib $nq; tail -20 $O/c3_${lib}_$nq.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/c3_${lib}_$nq.json')); r=d['roofline']; print('$lib nq $nq', 'matrix', round(r['kernel_ms'],4), 'frac', round(r['frac'],3), 'step', round(d['ms_per_step'],3))"
  done
done
RUNS="c3:64 c4:1024" TAG=r4h_prof PMC=1 CLK=1 SQ=1 bash tools/prof.sh
