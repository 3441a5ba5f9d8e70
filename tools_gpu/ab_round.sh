#!/bin/bash
# Interleaved A/B of kernel-source variants (tools_gpu/ab_src.py) on the three one-GPU configs.
# Usage: bash tools_gpu/ab_round.sh TAG VARIANT_DIR...   (dirs relative to the repo root)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=$1; shift
V=""; for d in "$@"; do V="$V $GRAFT_REPO_ROOT/$d"; done
for sc in "cornell_box 800 961 5" "cornell_smoke 800 961 5" "final_scene 800 400 4"; do
  timeout -k 10 300 python -u tools_gpu/ab_src.py $sc $V >> gpurun_out/$TAG.log 2>&1 || { tail -20 gpurun_out/$TAG.log; exit 1; }
done
grep -E "kernel ms|jit" gpurun_out/$TAG.log
