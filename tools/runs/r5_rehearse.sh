#!/bin/bash
# Rehearsal of the driver's N > 1 bench runs on a one-GPU box: torch.distributed.run with 2 ranks,
# both on cuda:0 over gloo (VRQ_BENCH_SHARED_GPU=1; the line is marked "rehearsal"): config 4 (default),
# config 2 and config 5.  Exercises the sharded pipeline, the all-gather + merge, the max-over-ranks
# timing, the N > 1 line's fields and the whole-corpus sample check with the real kernels.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r5rehearse}
mkdir -p $OUT
export VRQ_BENCH_SHARED_GPU=1
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
timeout -k 10 ${T4:-700} $R --master-port 29511 bench.py --gpus 2 --steps ${STEPS:-3} --warmup 1 > $OUT/c4.json 2> $OUT/c4.err || { tail -30 $OUT/c4.err; exit 1; }
tail -c 3000 $OUT/c4.json
timeout -k 10 300 $R --master-port 29512 bench.py --gpus 2 --config c2 --steps 10 --warmup 2 > $OUT/c2.json 2> $OUT/c2.err || { tail -30 $OUT/c2.err; exit 1; }
timeout -k 10 300 $R --master-port 29513 bench.py --gpus 2 --config c5 --steps 3 --warmup 1 > $OUT/c5.json 2> $OUT/c5.err || { tail -30 $OUT/c5.err; exit 1; }
echo REHEARSAL_OK
