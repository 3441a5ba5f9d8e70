#!/bin/bash
# Build the CURRENT working tree's device library into build/variants/librtmi355x_$1.so with
# extra compiler flags (e.g. -DRT_ABL_FRESH2), for A/B against the default build.
set -e
NAME=$1; shift
TMP=$(mktemp -d)
cp -r Makefile include "$TMP/"
mkdir -p "$TMP/surely-raytracing_amd" && cp -r surely-raytracing_amd/csrc "$TMP/surely-raytracing_amd/"
HF="--offload-arch=gfx950 -Iinclude -Ibuild -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function $*"
make -C "$TMP" device HIPFLAGS="$HF" > "$TMP/make.log" 2>&1 || { tail -20 "$TMP/make.log"; exit 1; }
mkdir -p build/variants
cp "$TMP/build/librtmi355x.so" "build/variants/librtmi355x_$NAME.so"
rm -rf "$TMP"
