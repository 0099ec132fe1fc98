#!/bin/bash
# Round 6: GPU suite, then config-2 ABAB against a baseline library (VAR) and config-3 plain lines.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r6chk}; mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
if [ -n "$VAR" ]; then TAG=${TAG:-r6chk}_c2 VAR=$VAR bash tools/runs/r5_c2ab.sh || exit 1; fi
for nq in ${C3NQS:-}; do
  timeout -k 10 300 python3 bench.py --config c3 --nq $nq --steps 20 --warmup 3 --no-cpu-baseline --no-recall \
    --no-encode --no-phase1 > $O/c3_nq$nq.json 2> $O/c3_nq$nq.err || { tail -20 $O/c3_nq$nq.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c3_nq$nq.json').read().strip().splitlines()[-1]); print('c3 nq=$nq', round(d['ms_per_step'],4), 'ms/step', {k: round(v,4) for k,v in d['phase_ms'].items()})"
done
