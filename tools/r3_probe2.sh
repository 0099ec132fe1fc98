#!/bin/bash
# GPU pass: config-5 sample-size sweep (probe library, VRQ_GEMM_SAMPLE_DIV), K1m bisect at the
# config-2 size, encoder NT variants.  Each step time-limited; the chain stops at the first failure.
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/${TAG:-r3e}; mkdir -p $OUT
VRQ_LIBS=vectorragquantization_amd/libvrq_probe.so timeout -k 10 400 python -u tools/gemm_probe.py --n 10000000 \
  --stages 16,32,64 --modes 3,2 --env "" --env VRQ_GEMM_SAMPLE_DIV=20 --env VRQ_GEMM_SAMPLE_DIV=10 \
  --env VRQ_GEMM_SAMPLE_DIV=5 > $OUT/g5_sample.jsonl 2> $OUT/g5_sample.err || { echo G5_FAIL; tail -20 $OUT/g5_sample.err; exit 1; }
cat $OUT/g5_sample.jsonl
TAG=${TAG:-r3e} BITS="0 1 2 4" bash tools/probes/c2_bisect.sh > /dev/null || { echo C2B_FAIL; exit 1; }
cat $OUT/r.jsonl
VRQ_LIBS=tools/probes/enc/lib_cur.so,tools/probes/enc/lib_ntg.so,tools/probes/enc/lib_cur.so,tools/probes/enc/lib_ntg.so \
  timeout -k 10 300 python -u tools/enc_probe.py > $OUT/enc.jsonl 2> $OUT/enc.err || { echo ENC_FAIL; tail -20 $OUT/enc.err; exit 1; }
cat $OUT/enc.jsonl
