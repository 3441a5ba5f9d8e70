#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python tools_gpu/prof_sections.py cornell_box 800 100 > gpurun_out/prof_sections.log 2>&1 || exit $?
timeout -k 10 300 python tools_gpu/prof_sections.py final_scene 400 64 >> gpurun_out/prof_sections.log 2>&1 || exit $?
timeout -k 10 300 python tools_gpu/prof_sections.py cornell_smoke 400 64 >> gpurun_out/prof_sections.log 2>&1
