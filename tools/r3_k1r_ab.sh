#!/bin/bash
# K1r A/B (config 3 at nq 1 / 8 / 64): bench lines on the library variants in tools/probes/k1r/, then
# the -m gpu K1r tests on the in-tree library.  Each step time-limited; stops at the first failure.
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/${TAG:-r3q}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "mfma or fullsize or scale or parity" > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for lib in ${LIBS:-head occ1 occ2}; do for nq in 1 8 64; do
  VRQ_LIB=tools/probes/k1r/lib_$lib.so timeout -k 10 300 python -u bench.py --config c3 --nq $nq --steps 20 --warmup 3 \
    --no-cpu-baseline --no-recall --no-encode > $OUT/c3_${lib}_nq$nq.json 2> $OUT/c3_${lib}_nq$nq.err || { echo FAIL $lib $nq; tail -5 $OUT/c3_${lib}_nq$nq.err; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/c3_${lib}_nq$nq.json')); print('$lib nq $nq', round(d['ms_per_step'],3), 'matrix', round(d['phase_ms']['matrix'],3), 'prefix', round(d['phase_ms']['prefix'],3), 'frac', round(d['roofline']['frac'],3))"
done; done
