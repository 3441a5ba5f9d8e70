#!/bin/bash
# Build the device library of git revision $1 into build/variants/librtmi355x_$2.so (A/B baseline
# for tools_gpu/ab_variants.py), with the revision's own Makefile.
set -e
REV=${1:-HEAD}; NAME=${2:-prev}
TMP=$(mktemp -d)
git archive "$REV" Makefile include surely-raytracing_amd/csrc | tar -x -C "$TMP"
make -C "$TMP" device > "$TMP/make.log" 2>&1 || { tail -20 "$TMP/make.log"; exit 1; }
mkdir -p build/variants
cp "$TMP/build/librtmi355x.so" "build/variants/librtmi355x_$NAME.so"
rm -rf "$TMP"
