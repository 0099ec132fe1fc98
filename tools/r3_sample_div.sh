#!/bin/bash
# Config-4 shard sizes (12.5M = 100M over 8 ranks, 25M, 100M) with the probe library's K1m sample
# fraction VRQ_SAMPLE_DIV (n / div rows, clamped to [131072, 1M]): per-step stage times.  Each run
# time-limited; the chain stops at the first failure.
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/${TAG:-r3m}; mkdir -p $OUT
for n in ${NS:-12500000 25000000 100000000}; do for div in ${DIVS:-16 32 64 128}; do
  VRQ_LIB=vectorragquantization_amd/libvrq_probe.so VRQ_SAMPLE_DIV=$div timeout -k 10 300 python -u bench.py --n $n \
    --steps 10 --warmup 2 --no-cpu-baseline --no-recall --no-encode > $OUT/c4_n${n}_d${div}.json 2> $OUT/c4_n${n}_d${div}.err \
    || { echo FAIL $n $div; tail -5 $OUT/c4_n${n}_d${div}.err; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/c4_n${n}_d${div}.json')); print('n $n div $div', round(d['ms_per_step'],3), {k: round(v,3) for k, v in d['phase_ms'].items()})"
done; done
