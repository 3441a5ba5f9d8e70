#!/bin/bash
# One-GPU scaling probe of C2 under different tail sizes (RT_TAIL_PAIRS; default = resident waves)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for T in default 2048 8192 16384; do
  if [ $T = default ]; then unset RT_TAIL_PAIRS; else export RT_TAIL_PAIRS=$T; fi
  echo "RT_TAIL_PAIRS=$T" >> gpurun_out/r02c_tail.log
  timeout -k 10 300 python -u tools_gpu/scaling_probe.py >> gpurun_out/r02c_tail.log 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/r02c_tail.log
