#!/bin/bash
# Rehearsal of the driver's N = 4 and N = 8 config-4 runs on a one-GPU box (all ranks on cuda:0 over
# gloo, VRQ_BENCH_SHARED_GPU=1; the lines are marked "rehearsal" and are not measurements).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r5rehearse}
mkdir -p $OUT
export VRQ_BENCH_SHARED_GPU=1
for n in ${NS:-4 8}; do
  timeout -k 10 ${T4:-500} python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29520 + n)) bench.py --gpus $n --steps 3 --warmup 1 > $OUT/c4_n$n.json 2> $OUT/c4_n$n.err || { tail -30 $OUT/c4_n$n.err; exit 1; }
done
echo REHEARSAL_OK
