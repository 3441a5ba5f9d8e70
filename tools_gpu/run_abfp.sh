#!/bin/bash
# GPU tests of the default build, then A/B of the contraction variant on C2 and C3.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_all.log 2>&1 || exit $?
VARDIR=build/variants_fp timeout -k 10 300 python -u tools_gpu/ab_variants.py 800 1000 3 cornell_box > gpurun_out/abfp_c2.log 2>&1 || exit $?
VARDIR=build/variants_fp timeout -k 10 300 python -u tools_gpu/ab_variants.py 800 1000 3 cornell_smoke > gpurun_out/abfp_c3.log 2>&1
