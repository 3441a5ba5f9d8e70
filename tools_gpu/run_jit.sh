#!/bin/bash
# GPU parity tests, then the scene-specialised vs interpreter A/B on C2 and C3.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_all.log 2>&1 || exit $?
timeout -k 10 300 python -u tools_gpu/ab_jit.py cornell_box 800 1000 3 > gpurun_out/ab_jit.log 2>&1 || exit $?
timeout -k 10 300 python -u tools_gpu/ab_jit.py cornell_smoke 800 1000 2 >> gpurun_out/ab_jit.log 2>&1 || exit $?
