#!/bin/bash
# Round 6: K1m change check -- the list / edge / MFMA tests, then MATRIX-stage ABAB (config-4 corpus)
# against a baseline library (BASE, default tools/ab/lib_base.so)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r6k1m}; mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_lists.py tests/test_gpu_k1m_edges.py tests/test_gpu_mfma.py} \
    -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
timeout -k 10 400 python -u tools/stage_bench.py --clustered --cases ${CASES:-100000000:1024} --rounds ${ROUNDS:-4} \
  --libs ${BASE:-tools/ab/lib_base.so},vectorragquantization_amd/libvrq.so > $O/ab.jsonl 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
python3 -c "
import json
for l in open('$O/ab.jsonl'):
    d = json.loads(l); print(d['lib'].split('/')[-1], d['n'], d['nq'], round(d['ms'], 4), [round(x, 3) for x in d['ms_rounds']])"
