#!/bin/bash
# one-off GPU pass for round-3 kernel iteration (see tools/gpu_r3.sh for the knobs)
export TAG=${TAG:-r3c} BENCHES=${BENCHES:-"c5 c2"} BENCH_T=${BENCH_T:-400}
export G5LIBS=${G5LIBS:-tools/probes/g5/lib_base.so,tools/probes/g5/lib_rs.so,tools/probes/g5/lib_np2.so,tools/probes/g5/lib_w8.so,tools/probes/g5/lib_w8np2.so,tools/probes/g5/lib_b1.so,tools/probes/g5/lib_rsb1.so}
export VARIANTS=${VARIANTS-"hitslow=tools/probes/g5/lib_hitslow.so:c2"}
export TEST_K=${TEST_K-"gemm_topk or encoders or hamming or search3"}
exec bash tools/gpu_r3.sh
