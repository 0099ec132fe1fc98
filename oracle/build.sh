#!/bin/sh
# Build the C restatement of FAISS hammings_knn_hc (TEST INFRASTRUCTURE ONLY) into
# oracle/_build/liboracle.so.  Pure gcc, no reference sources involved.
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
mkdir -p "$HERE/_build"
gcc -O3 -march=x86-64-v3 -mpopcnt -fopenmp -fPIC -shared -o "$HERE/_build/liboracle.so.tmp" "$HERE/hamming_knn.c"
mv "$HERE/_build/liboracle.so.tmp" "$HERE/_build/liboracle.so"
