#!/bin/bash
# Config-4 bench at per-rank corpus sizes of the multi-GPU runs (100M / N rows on one GPU, nq = 1024,
# sustained steps): the in-tree build against a variant, alternated.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r5rank}
mkdir -p $OUT
B="--no-cpu-baseline --no-recall --no-encode --no-phase1 --steps ${STEPS:-20} --warmup 5"
for n in ${NS:-12500000 25000000 50000000}; do
  timeout -k 10 240 python bench.py --n $n $B > $OUT/new_$n.json 2> $OUT/new_$n.err || exit 1
  timeout -k 10 240 python tools/with_lib.py ${VAR:-tools/probes/var/lib_k1s_all.so} bench.py --n $n $B > $OUT/var_$n.json 2> $OUT/var_$n.err || exit 1
  timeout -k 10 240 python bench.py --n $n $B > $OUT/new2_$n.json 2> $OUT/new2_$n.err || exit 1
  timeout -k 10 240 python tools/with_lib.py ${VAR:-tools/probes/var/lib_k1s_all.so} bench.py --n $n $B > $OUT/var2_$n.json 2> $OUT/var2_$n.err || exit 1
done
python3 - <<'PY'
import json, glob, os
out = os.environ.get("TAG", "r5rank")
for f in sorted(glob.glob(f"gpurun_out/{out}/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(os.path.basename(f), round(d.get("value"), 1), round(d.get("ms_per_step"), 4), round(d["phase_ms"]["matrix"], 4))
PY
