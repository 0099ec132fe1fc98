#!/bin/bash
# full library variant with extra flags on every source: buildfull.sh NAME FLAGS...
set -e
cd /root/repo
name=$1; shift
mkdir -p tools/ab/full_$name
objs=""
for s in hamming_scan hamming_mfma select_rescore encode gemm_topk dequant; do
  extra=""; [ $s = hamming_mfma -o $s = gemm_topk ] && extra="-mllvm -amdgpu-mfma-vgpr-form=1"
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 $extra "$@" -c vectorragquantization_amd/csrc/$s.hip -o tools/ab/full_$name/$s.o &
  objs="$objs tools/ab/full_$name/$s.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs -o tools/ab/lib_$name.so
rm -rf tools/ab/full_$name
echo tools/ab/lib_$name.so
