#!/bin/bash
# K1r race fix check: candidate lists vs true distances (nq 8 / 64 / 128), then tests and c3 lines.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4e; mkdir -p $O
for nq in 8 64 128; do
  timeout -k 10 300 python -u tools/probes/k1r_lists.py --nq $nq --reps 3 > $O/lists_$nq.log 2>&1 || { echo LISTS_FAIL $nq; tail -20 $O/lists_$nq.log; exit 1; }
  echo "nq $nq" $(grep -c "^rep .* mismatches 0 " $O/lists_$nq.log) "clean reps of 3;" $(grep "mismatches" $O/lists_$nq.log | tr '\n' ' ')
done
TAG=r4e bash tools/runs/r4_c.sh
