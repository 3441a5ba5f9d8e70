#!/bin/bash
# C4 (final_scene) section split and ordered-BVH walk statistics of the profiling build
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python3 tools_gpu/prof_sections.py final_scene 400 100 > gpurun_out/r02c_sec_c4.log 2>&1 || exit $?
cat gpurun_out/r02c_sec_c4.log
timeout -k 10 300 python3 tools_gpu/prof_obvh.py final_scene 400 100 > gpurun_out/r02c_obvh_c4.log 2>&1 || exit $?
cat gpurun_out/r02c_obvh_c4.log
timeout -k 10 300 python3 tools_gpu/prof_sections.py cornell_smoke 800 100 > gpurun_out/r02c_sec_c3.log 2>&1 || exit $?
cat gpurun_out/r02c_sec_c3.log
