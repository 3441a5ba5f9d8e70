#!/bin/bash
# packed-fma slab times in the LDS BVH walk: GPU suite, then interleaved A/B against the previous head
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 bash tools_gpu/r03_prev.sh > gpurun_out/r03_ab_fma.log 2>&1 || exit $?
cat gpurun_out/r03_ab_fma.log | grep -v "^#"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
  > gpurun_out/r03_fma_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r03_fma_pytest.log; exit $rc
