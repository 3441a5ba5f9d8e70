#!/bin/bash
# The -m gpu suite on the box, one pytest process, output under gpurun_out/.
# Usage: bash tools_gpu/gpu_tests.sh TAG [test paths / pytest args...]   (default: tests/, the
# whole gpu suite)
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-gpu}; shift
[ $# -eq 0 ] && set -- tests
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest -m gpu -x -v -s --timeout 900 --timeout-method thread "$@" \
  > gpurun_out/${TAG}.log 2>&1
rc=$?
grep -E "^(C[0-9]|tests/)|passed|failed|error" gpurun_out/${TAG}.log | tail -60
exit $rc
