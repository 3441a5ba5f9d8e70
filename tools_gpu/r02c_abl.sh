#!/bin/bash
# ablation A/B on C2 and C3 (build/variants vs build/)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for spec in "800 1000 3 cornell_box" "800 1000 2 cornell_smoke"; do
  set -- $spec
  timeout -k 10 400 python -u tools_gpu/ab_variants.py $spec > gpurun_out/r02c_abl_$4.log 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/r02c_abl_$4.log
done
