#!/bin/bash
# Round-end profiling of every bench config (run on the GPU box via gpurun): tools/prof_r2.sh
# (rocprofv3 kernel-trace stats + separate FETCH_SIZE / WRITE_SIZE passes) per config, each step
# time-limited inside prof_r2.sh; the chain stops at the first failure.   CFGS="c4 c2 c3 c5"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for c in ${CFGS:-c4 c2 c3 c5}; do
  CFG=$c TAG=${PREFIX:-final}_$c PT=${PT:-300} bash tools/prof_r2.sh || { echo PROF_FAIL $c; exit 1; }
done
echo all_done
