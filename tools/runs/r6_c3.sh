#!/bin/bash
# Config-3 timer reconciliation: in ONE lease, per nq, (a) the plain bench line (HIP
# events, no profiler), (b) the same bench command under rocprofv3 --kernel-trace (its own event line
# plus the per-dispatch durations of the same launches), then the FETCH/WRITE and clock passes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r6c3}; mkdir -p $O
S=${STEPS:-20}; W=${WARMUP:-3}
for nq in ${NQS:-1 8 64}; do
  timeout -k 10 300 python3 bench.py --config c3 --nq $nq --steps $S --warmup $W --no-cpu-baseline --no-recall \
    --no-encode --no-phase1 > $O/plain_nq$nq.json 2> $O/plain_nq$nq.err || { tail -20 $O/plain_nq$nq.err; exit 1; }
done
RUNS="$(for nq in ${NQS:-1 8 64}; do printf 'c3:%s ' $nq; done)" TAG=${TAG:-r6c3}_prof PMC=${PMC:-1} CLK=${CLK:-1} \
  STEPS=$S WARMUP=$W bash tools/prof.sh || exit 1
python3 - <<'PY'
import json, os
O = os.environ.get("TAG", "r6c3")
for nq in os.environ.get("NQS", "1 8 64").split():
    plain = json.loads(open(f"gpurun_out/{O}/plain_nq{nq}.json").read().strip().splitlines()[-1])
    d = f"gpurun_out/{O}_prof/c3_nq{nq}"
    prof = json.loads(open(f"{d}/bench_trace.json").read().strip().splitlines()[-1])
    disp = json.load(open(f"{d}/dispatch.json"))["kernels"]
    k = [v for n, v in disp.items() if "rows" in n and "<0," in n]
    print(json.dumps({"nq": int(nq), "events_plain_ms": plain["roofline"]["kernel_ms"],
                      "events_under_rocprof_ms": prof["roofline"]["kernel_ms"],
                      "rocprof_mean_after_warmup_ms": k[0]["mean_after_warmup_ms"] if k else None,
                      "rocprof_first_ms": k[0]["first_ms"] if k else None}))
PY
