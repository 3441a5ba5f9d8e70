#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python tools_gpu/prof_sections.py cornell_box 800 1000 > gpurun_out/prof_sections.log 2>&1 || exit $?
timeout -k 10 300 python tools_gpu/prof_sections.py cornell_box 800 100 >> gpurun_out/prof_sections.log 2>&1 || exit $?
timeout -k 10 300 bash tools_gpu/prof_pmc.sh gpurun_out/pmc3 cornell_box 800 1000
