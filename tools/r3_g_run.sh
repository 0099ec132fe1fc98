#!/bin/bash
# GPU pass: full -m gpu suite + smoke, K5 variants, c5 and c2 bench lines
export TAG=${TAG:-r3g} BENCHES=${BENCHES-"c5 c2"}
export TEST_K=${TEST_K-""}
export G5LIBS=${G5LIBS-tools/probes/g5/lib_cur.so,tools/probes/g5/lib_noseed.so,tools/probes/g5/lib_w4.so}
export G5ARGS="--n 10000000 --stages 16,32,64"
export ENCLIBS=${ENCLIBS-""}
export VARIANTS=${VARIANTS-""}
exec bash tools/gpu_r3.sh
