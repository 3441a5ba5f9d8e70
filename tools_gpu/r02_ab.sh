#!/bin/bash
# A/B: default build vs build/variants/*.so, interleaved in one process (torch imported first)
set -o pipefail
mkdir -p gpurun_out
AB_ENVS="$AB_ENVS" timeout -k 10 500 python -u tools_gpu/ab_variants.py ${1:-800} ${2:-1000} ${3:-3} ${4:-cornell_box} > gpurun_out/r02_ab_${4:-cornell_box}.log 2>&1
rc=$?; cat gpurun_out/r02_ab_${4:-cornell_box}.log | tail -8; exit $rc
