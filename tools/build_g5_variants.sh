#!/bin/bash
# Build libvrq variants differing only in gemm_topk.hip compile flags (timing probes for the
# config-5 matrix pass, run by tools/gemm_probe.py with VRQ_LIBS=...).  Usage: NAME=FLAGS ...
set -e
cd "$(dirname "$0")/.."
python -m vectorragquantization_amd._build >/dev/null 2>&1 || true
OBJ=vectorragquantization_amd/_obj
mkdir -p tools/probes/g5
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form=1 -DVRQ_TUNING_ENV \
    $flags -c vectorragquantization_amd/csrc/gemm_topk.hip -o tools/probes/g5/gemm_$name.o &
done
wait
for spec in "$@"; do
  name=${spec%%=*}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $(ls $OBJ/*.o | grep -v gemm_topk.o) \
    tools/probes/g5/gemm_$name.o -o tools/probes/g5/lib_$name.so
  echo tools/probes/g5/lib_$name.so
done
