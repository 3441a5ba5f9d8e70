#!/bin/bash
# Build the device library of git revision $1 into build/variants/librtmi355x_$2.so (A/B baseline)
set -e
REV=${1:-HEAD}; NAME=${2:-prev}
TMP=$(mktemp -d)
git archive "$REV" surely-raytracing_amd/csrc include | tar -x -C "$TMP"
mkdir -p build/variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-function \
  -I"$TMP/include" -I"$TMP/surely-raytracing_amd/csrc" -shared \
  "$TMP/surely-raytracing_amd/csrc/rt_device.hip" "$TMP/surely-raytracing_amd/csrc/rt_flatten.cpp" \
  -o "build/variants/librtmi355x_$NAME.so"
rm -rf "$TMP"
