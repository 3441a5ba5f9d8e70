#!/bin/bash
# packed-fma slab times: interleaved A/B against the previous head, the GPU suite, then the
# round's profiles at this head (kept only if the A/B wins)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 bash tools_gpu/r03_prev.sh > gpurun_out/r03_ab_fma.log 2>&1 || exit $?
grep -v "^#" gpurun_out/r03_ab_fma.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
  > gpurun_out/r03_fma_pytest.log 2>&1 || { tail -20 gpurun_out/r03_fma_pytest.log; exit 1; }
tail -1 gpurun_out/r03_fma_pytest.log
bash tools_gpu/r03_profiles.sh r03h
