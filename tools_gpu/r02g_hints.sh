#!/bin/bash
# GPU suite, then interleaved A/B of the CBVH stack entry hints (default) against
# RT_NO_CBVH_HINTS=1 on C4 (final_scene 800x800, 400 spp)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread \
  > gpurun_out/r02g_hints_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r02g_hints_pytest.log; [ $rc -eq 0 ] || exit $rc
AB_ENVS="RT_NO_CBVH_HINTS=1" timeout -k 10 400 python -u tools_gpu/ab_variants.py 800 400 3 final_scene \
  > gpurun_out/r02g_ab_hints_c4.log 2>&1 || exit $?
tail -4 gpurun_out/r02g_ab_hints_c4.log
