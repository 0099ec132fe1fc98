#!/bin/bash
# bench.py at several exact-prefix fractions (VRQ_SAMPLE_DIV), one GPU call
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/sweep
for d in ${DIVS:-16 32 64}; do
  VRQ_SAMPLE_DIV=$d timeout -k 10 200 python bench.py --no-cpu-baseline --no-recall > gpurun_out/sweep/b_$d.json 2> gpurun_out/sweep/b_$d.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/sweep/b_$d.json'));print($d,'QPS',round(d['value']),{k:round(v,3) for k,v in d['phase_ms'].items()})"
done
