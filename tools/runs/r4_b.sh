#!/bin/bash
# Round 4 check: GPU tests, the default bench line (config 4 + the config-3 Phase-I leg), the config-2
# nq = 1 latency line, and the config-3 profiles (kernel trace + PMC) of the current build.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r4b}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u bench.py > $O/c4.json 2> $O/c4.err || { echo C4_FAIL; tail -30 $O/c4.err; exit 1; }
timeout -k 10 300 python -u bench.py --config c2 --nq 1 > $O/c2_nq1.json 2> $O/c2_nq1.err || { echo C2_FAIL; tail -30 $O/c2_nq1.err; exit 1; }
python3 - <<PY
import json
d = json.load(open("$O/c4.json"))
print("c4", round(d["value"]), "QPS", round(d["ms_per_step"], 3), "ms", "frac", round(d["roofline"]["frac"], 3))
p = d.get("roofline_phase1", {})
for k, v in p.get("points", {}).items():
    print(" c3 nq", k, "ms", round(v["kernel_ms"], 4), "frac", round(v["frac"], 3), "rocprof", v.get("rocprof"))
print(" identity", p.get("cpu_gpu_identity"), p.get("cpu_baseline", {}).get("value"))
e = json.load(open("$O/c2_nq1.json"))
print("c2 nq1", round(e["value"]), "QPS", round(e["ms_per_step"], 4), "ms", e.get("latency"), e.get("cpu_baseline", {}).get("single_core"))
PY
RUNS="c3:1 c3:8 c3:64" TAG=${TAG:-r4b}/prof PMC=1 bash tools/prof.sh
