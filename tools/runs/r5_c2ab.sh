#!/bin/bash
# Config-2 bench steps with the in-tree library and a variant, alternated (ABAB).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r5c2}
mkdir -p $OUT
B="--config ${CFG:-c2} --no-cpu-baseline --no-recall --no-encode --no-phase1 --steps ${STEPS:-30} --warmup 5"
for i in 1 2; do
  timeout -k 10 ${T:-300} python bench.py $B > $OUT/new_$i.json 2> $OUT/new_$i.err || exit 1
  timeout -k 10 ${T:-300} python tools/with_lib.py ${VAR:-tools/probes/var/lib_k1m_r5.so} bench.py $B > $OUT/old_$i.json 2> $OUT/old_$i.err || exit 1
done
python3 - <<'PY'
import json, glob, os
out = os.environ.get("TAG", "r5c2")
for f in sorted(glob.glob(f"gpurun_out/{out}/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(os.path.basename(f), d.get("value"), d.get("ms_per_step"), json.dumps(d.get("phase_ms")))
PY
