#!/bin/bash
# Round 6: K1r lean (config 3, nq = 64) with and without the row unpack (timing-only NOUNPACK probe):
# MATRIX-stage ABAB, then the clock / SQ / LDS counter passes of both
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r6k1r}; mkdir -p $O
timeout -k 10 300 python -u tools/stage_bench.py --cases 100000000:64 --rounds 4 \
  --libs vectorragquantization_amd/libvrq.so,tools/ab/lib_NOUNPACK.so > $O/ab.jsonl 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab.jsonl
TAG=${TAG:-r6k1r}_ctr LIBS="vectorragquantization_amd/libvrq.so tools/ab/lib_NOUNPACK.so" \
  CMD="python3 tools/stage_bench.py --libs {lib} --cases 100000000:64 --reps 5 --rounds 1" bash tools/ab_counters.sh
