#!/bin/bash
# Builds tools/probes/mfma_bisect_<bits>[_a<ahead>] (see mfma_bisect.hip): VRQ_BISECT bit sets
# from $BITS (default "0 1 2 4") at B-fragment prefetch distance 3, plus $AHEAD variants of bisect 0.
set -e
cd "$(dirname "$0")"
F="-O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form=1"
SRC="mfma_bisect.hip ../../vectorragquantization_amd/csrc/hamming_scan.hip"
for b in ${BITS:-0 1 2 4}; do
  /opt/rocm/bin/hipcc $F -DVRQ_BISECT=$b $SRC -o mfma_bisect_$b &
done
for a in ${AHEAD:-}; do
  /opt/rocm/bin/hipcc $F -DVRQ_BISECT=0 -DVRQ_BAHEAD=$a $SRC -o mfma_bisect_0_a$a &
done
wait
