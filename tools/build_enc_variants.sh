#!/bin/bash
# Build libvrq variants differing only in encode.hip compile flags (encoder timing probes, run by
# tools/enc_probe.py with VRQ_LIBS=...).  Usage: NAME=FLAGS ...
set -e
cd "$(dirname "$0")/.."
python -m vectorragquantization_amd._build >/dev/null 2>&1 || true
OBJ=vectorragquantization_amd/_obj
mkdir -p tools/probes/enc
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form=1 \
    $flags -c vectorragquantization_amd/csrc/encode.hip -o tools/probes/enc/encode_$name.o &
done
wait
for spec in "$@"; do
  name=${spec%%=*}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $(ls $OBJ/*.o | grep -v '/encode.o') \
    tools/probes/enc/encode_$name.o -o tools/probes/enc/lib_$name.so
  echo tools/probes/enc/lib_$name.so
done
