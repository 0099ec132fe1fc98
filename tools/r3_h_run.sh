#!/bin/bash
# GPU pass: K5 finish-kernel variants (candidate ids prefetched per batch) + tests + c5 bench
export TAG=${TAG:-r3h} BENCHES=${BENCHES-"c5"}
export TEST_K=${TEST_K-"gemm_topk or fullsize or flat or encoders or vectordb"}
export G5LIBS=${G5LIBS-tools/probes/g5/lib_prevfin.so,tools/probes/g5/lib_cur.so,tools/probes/g5/lib_sb3.so,tools/probes/g5/lib_sb4.so}
export G5ARGS="--n 10000000 --stages 16,32,64"
export ENCLIBS=vectorragquantization_amd/libvrq.so VARIANTS=""
exec bash tools/gpu_r3.sh
