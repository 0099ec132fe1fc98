#!/bin/bash
# Build libvrq variants that differ in ONE source file's compile flags (timing probes).
# Usage: tools/build_variants.sh NAME=SOURCE.hip:FLAGS ...  -> tools/ab/lib_NAME.so
set -e
cd "$(dirname "$0")/.."
python -m vectorragquantization_amd._build >/dev/null 2>&1 || true
OBJ=vectorragquantization_amd/_obj
mkdir -p tools/ab
for spec in "$@"; do
  name=${spec%%=*}; rest=${spec#*=}; src=${rest%%:*}; flags=${rest#*:}
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form=1 \
    $flags -c vectorragquantization_amd/csrc/$src -o tools/ab/${name}_${src%.hip}.o &
done
wait
for spec in "$@"; do
  name=${spec%%=*}; rest=${spec#*=}; src=${rest%%:*}
  objs=""
  for s in hamming_scan hamming_mfma select_rescore encode gemm_topk dequant; do
    if [ "$s.hip" = "$src" ]; then objs="$objs tools/ab/${name}_$s.o"; else objs="$objs $OBJ/$s.o"; fi
  done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs -o tools/ab/lib_$name.so
  echo tools/ab/lib_$name.so
done
