#!/bin/bash
# K5 sample-size sweep: stage times (sample 16 / main 32 / finish 64) at 10M x 1024, nq = 1024, for
# the sample fraction VRQ_GEMM_SAMPLE_DIV (probe builds read it), on the library layout and the
# 8-wave Phase-III variant
export TAG=${TAG:-r3d} TESTS=0 BENCHES=""
export G5LIBS=${G5LIBS:-vectorragquantization_amd/libvrq_probe.so,tools/probes/g5/lib_w8np2.so}
export G5ARGS="--n 10000000 --stages 16,32,64 --env VRQ_NONE=0 --env VRQ_GEMM_SAMPLE_DIV=16 --env VRQ_GEMM_SAMPLE_DIV=8 --env VRQ_GEMM_SAMPLE_DIV=4"
export VARIANTS=""
export ENCLIBS=${ENCLIBS:-vectorragquantization_amd/libvrq.so,tools/probes/g5/lib_encold.so,tools/probes/g5/lib_enc6.so,tools/probes/g5/lib_enc8.so,tools/probes/g5/lib_enc0.so}
exec bash tools/gpu_r3.sh
