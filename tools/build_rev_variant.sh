#!/bin/bash
# full library from a git revision's csrc (A/B baselines): build_rev_variant.sh REV NAME -> tools/ab/lib_NAME.so
set -e
cd /root/repo
rev=$1; name=$2
d=$(mktemp -d)
mkdir -p $d/pkg/csrc $d/include tools/ab
for f in $(git ls-tree --name-only $rev vectorragquantization_amd/csrc/); do git show $rev:$f > $d/pkg/csrc/$(basename $f); done
git show $rev:include/vrq.h > $d/include/vrq.h
objs=""
for s in hamming_scan hamming_mfma select_rescore encode gemm_topk dequant; do
  extra=""; [ $s = hamming_mfma -o $s = gemm_topk ] && extra="-mllvm -amdgpu-mfma-vgpr-form=1"
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 $extra -c $d/pkg/csrc/$s.hip -o $d/$s.o &
  objs="$objs $d/$s.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs -o tools/ab/lib_$name.so
rm -rf $d
echo tools/ab/lib_$name.so
