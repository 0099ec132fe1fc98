#!/bin/bash
# Round 4: config-3 timer reconciliation on the current build: for nq in 1 8 64, an event-timed bench line,
# then the same command under rocprofv3 --kernel-trace (per-dispatch durations reduced by trace_dispatches.py).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r4a}
mkdir -p $O
for nq in ${NQS:-1 8 64}; do
  timeout -k 10 300 python3 bench.py --config c3 --nq $nq --steps 20 --warmup 3 --no-cpu-baseline > $O/c3_nq$nq.json 2> $O/c3_nq$nq.err || { echo BENCH_FAIL $nq; tail -20 $O/c3_nq$nq.err; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr$nq -o run -- python3 bench.py --config c3 --nq $nq --steps 20 --warmup 3 --no-cpu-baseline > $O/c3p_nq$nq.json 2> $O/c3p_nq$nq.err || { echo PROF_FAIL $nq; tail -20 $O/c3p_nq$nq.err; exit 1; }
  python3 tools/trace_dispatches.py $O/tr$nq $O/disp_nq$nq.csv --skip 3 > $O/disp_nq$nq.txt && rm -rf $O/tr$nq
  echo "== nq $nq"; cat $O/disp_nq$nq.txt
  python3 -c "import json;d=json.load(open('$O/c3_nq$nq.json'));p=json.load(open('$O/c3p_nq$nq.json'));print('events', d['phase_ms'], '\nevents-under-prof', p['phase_ms'])"
done
echo done
