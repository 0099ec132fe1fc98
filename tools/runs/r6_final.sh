#!/bin/bash
# Round-6 closing records: every GPU test, smoke, the list-overflow census, the bench lines of configs 4
# (default line, with the config-3 leg), 2, 5 and 3, then the config-5 profile passes (RUNS to override).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r6final}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u tools/overflow_census.py > $O/overflow_census.jsonl 2> $O/overflow_census.err || { tail -20 $O/overflow_census.err; exit 1; }
cat $O/overflow_census.jsonl
timeout -k 10 600 python3 bench.py > $O/c4.json 2> $O/c4.err || { tail -20 $O/c4.err; exit 1; }
for c in c2 c5 c3; do
  timeout -k 10 400 python3 bench.py --config $c > $O/$c.json 2> $O/$c.err || { tail -20 $O/$c.err; exit 1; }
done
python3 - <<'PY'
import json, os
O = "gpurun_out/" + os.environ.get("TAG", "r6final")
for c in ("c4", "c2", "c5", "c3"):
    d = json.loads(open(f"{O}/{c}.json").read().strip().splitlines()[-1])
    print(c, round(d["value"], 1), d["unit"], round(d["ms_per_step"], 4), "ms/step", "roofline frac", round(d["roofline"]["frac"], 4))
PY
if [ -n "${RUNS-c5:1024}" ]; then RUNS="${RUNS-c5:1024}" TAG=${TAG:-r6final}_prof PMC=1 CLK=1 SQ=1 bash tools/prof.sh || exit 1; fi
