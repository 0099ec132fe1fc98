#!/bin/bash
# Round-5 bench lines of the final build: the driver's default line (c4 + the config-3 Phase-I leg),
# config 2 (nq 1024 and the nq = 1 latency leg) and config 5.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5bench; mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/c4.json 2> $O/c4.err || { echo C4_FAIL; tail -20 $O/c4.err; exit 1; }
echo c4 ok
timeout -k 10 300 python -u bench.py --config c2 > $O/c2.json 2> $O/c2.err || { echo C2_FAIL; tail -20 $O/c2.err; exit 1; }
echo c2 ok
timeout -k 10 300 python -u bench.py --config c2 --nq 1 > $O/c2_nq1.json 2> $O/c2_nq1.err || { echo C2N1_FAIL; tail -20 $O/c2_nq1.err; exit 1; }
echo c2 nq1 ok
timeout -k 10 400 python -u bench.py --config c5 > $O/c5.json 2> $O/c5.err || { echo C5_FAIL; tail -20 $O/c5.err; exit 1; }
echo c5 ok
