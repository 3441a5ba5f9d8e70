#!/bin/bash
# ordered BVH: GPU parity suite (BVH scenes first), then A/B vs the reference-order walk at C4
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "final_scene or bvh or C4 or random_balls or chunked" > gpurun_out/r02_obvh_pytest.log 2>&1
rc=$?; tail -4 gpurun_out/r02_obvh_pytest.log; [ $rc -eq 0 ] || exit $rc
AB_ENVS="FLAGS=0x10" timeout -k 10 600 python -u tools_gpu/ab_variants.py 800 400 2 final_scene > gpurun_out/r02_ab_obvh.log 2>&1
rc=$?; tail -3 gpurun_out/r02_ab_obvh.log; exit $rc
