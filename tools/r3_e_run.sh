#!/bin/bash
# GPU pass: encoder + K5 correctness tests, K5 hit-recording variants, encoder throughput
export TAG=${TAG:-r3f} BENCHES="c5"
export TEST_K=${TEST_K-"gemm_topk or fullsize or flat"}
export G5LIBS=${G5LIBS:-tools/probes/g5/lib_stg.so,tools/probes/g5/lib_stg0.so,tools/probes/g5/lib_w8stg.so,tools/probes/g5/lib_b16.so}
export G5ARGS="--n 10000000 --stages 16,32"
export ENCLIBS=""
export VARIANTS=""
exec bash tools/gpu_r3.sh
