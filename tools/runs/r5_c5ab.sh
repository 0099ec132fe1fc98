#!/bin/bash
# K5 A/B: config-5 bench steps with the in-tree library and a variant, alternated (ABAB).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r5c5}
mkdir -p $OUT
B="--config c5 --no-cpu-baseline --no-recall --no-encode --no-phase1 --steps ${STEPS:-10} --warmup 3"
for i in 1 2; do
  timeout -k 10 300 python bench.py $B > $OUT/new_$i.json 2> $OUT/new_$i.err || exit 1
  timeout -k 10 300 python tools/with_lib.py ${VAR:-tools/probes/var/lib_g5r4.so} bench.py $B > $OUT/old_$i.json 2> $OUT/old_$i.err || exit 1
done
