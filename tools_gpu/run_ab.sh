#!/bin/bash
# GPU parity tests, then interleaved A/B of build/librtmi355x.so against $VARDIR/*.so on C2 and C4.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export VARDIR=${VARDIR:-build/variants_ab}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -u tools_gpu/ab_variants.py 800 1000 3 cornell_box > gpurun_out/ab_c2.log 2>&1 || exit $?
timeout -k 10 300 python -u tools_gpu/ab_variants.py 800 400 2 final_scene > gpurun_out/ab_c4.log 2>&1 || exit $?
timeout -k 10 300 python -u tools_gpu/ab_variants.py 800 400 2 cornell_smoke > gpurun_out/ab_c3.log 2>&1 || exit $?
