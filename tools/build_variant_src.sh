#!/bin/bash
# Build a libvrq variant in which ONE source file is replaced by another (A/B of a previous version).
# Usage: tools/build_variant_src.sh NAME ORIGINAL.hip ALTERNATIVE_PATH [extra hipcc flags]
#   -> tools/ab/lib_NAME.so (the other objects from the in-tree build)
set -e
cd "$(dirname "$0")/.."
name=$1; src=$2; alt=$3; shift 3
python -m vectorragquantization_amd._build >/dev/null 2>&1 || true
OBJ=vectorragquantization_amd/_obj
mkdir -p tools/ab
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form=1 \
  -I vectorragquantization_amd/csrc "$@" -c "$alt" -o tools/ab/${name}_${src%.hip}.o
objs=""
for s in hamming_scan hamming_mfma select_rescore encode gemm_topk dequant; do
  if [ "$s.hip" = "$src" ]; then objs="$objs tools/ab/${name}_$s.o"; else objs="$objs $OBJ/$s.o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs -o tools/ab/lib_$name.so
echo tools/ab/lib_$name.so
