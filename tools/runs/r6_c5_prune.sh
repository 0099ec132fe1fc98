#!/bin/bash
# Round 6: K5 candidate-level prune -- the K5 / flat / full-shape tests, then config-5 bench ABAB against a
# baseline library (VAR, default tools/ab/lib_base.so)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r6prune}; mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 700 python -u -m pytest ${TESTS:-tests/test_gpu_gemm.py tests/test_gpu_flat.py tests/test_gpu_fullsize.py} \
    -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
B="--config c5 --no-cpu-baseline --no-recall --no-encode --no-phase1 --steps ${STEPS:-10} --warmup 3"
for i in 1 2; do
  timeout -k 10 300 python bench.py $B > $O/new_$i.json 2> $O/new_$i.err || { tail -20 $O/new_$i.err; exit 1; }
  timeout -k 10 300 python tools/with_lib.py ${VAR:-tools/ab/lib_base.so} bench.py $B > $O/old_$i.json 2> $O/old_$i.err || { tail -20 $O/old_$i.err; exit 1; }
done
python3 - <<PY
import json
for f in ("new_1", "old_1", "new_2", "old_2"):
    d = json.loads(open("$O/%s.json" % f).read().strip().splitlines()[-1])
    print(f, round(d["value"], 1), round(d["ms_per_step"], 4), {k: round(v, 4) for k, v in d["phase_ms"].items()})
PY
