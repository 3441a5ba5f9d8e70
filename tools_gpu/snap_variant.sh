#!/bin/bash
# Build the CURRENT working tree's device library into build/variants/librtmi355x_$1.so (extra
# compiler flags after the name), for A/B against later edits.
set -e
NAME=$1; shift
TMP=$(mktemp -d)
mkdir -p "$TMP/surely-raytracing_amd"
cp -r include "$TMP/" && cp -r surely-raytracing_amd/csrc "$TMP/surely-raytracing_amd/"
mkdir -p build/variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-function "$@" \
  -shared "$TMP/surely-raytracing_amd/csrc/rt_device.hip" "$TMP/surely-raytracing_amd/csrc/rt_flatten.cpp" \
  -o "build/variants/librtmi355x_$NAME.so"
rm -rf "$TMP"
