#!/bin/bash
# Builds tools/probes/mfma_bisect_{0,1,2,4,7} (see mfma_bisect.hip).
set -e
cd "$(dirname "$0")"
for b in 0 1 2 3 4 7; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -DVRQ_BISECT=$b -mllvm -amdgpu-mfma-vgpr-form=1 \
    mfma_bisect.hip ../../vectorragquantization_amd/csrc/hamming_scan.hip -o mfma_bisect_$b &
done
wait
