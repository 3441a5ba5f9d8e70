#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools_gpu/prof_sections.py cornell_box 800 100 > gpurun_out/sec_c2.log 2>&1 || exit $?
timeout -k 10 300 python -u tools_gpu/prof_sections.py cornell_smoke 800 100 > gpurun_out/sec_c3.log 2>&1 || exit $?
