#!/bin/bash
# Diagnostics of the opt-in scene-specialised BVH kernel: section split of final_scene (profiling
# build, interpreter), then one small render with RT_JIT_BVH=1 at a 256-thread block.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools_gpu/prof_sections.py final_scene 400 100 > gpurun_out/prof_sections_c4.log 2>&1 || exit $?
RT_JIT_BVH=1 RT_JIT_BVH_BLOCK=256 timeout -k 10 120 python -u tools_gpu/one_render.py final_scene 200 16 2 > gpurun_out/bvhjit_256.log 2>&1
