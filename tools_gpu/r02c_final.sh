#!/bin/bash
# Round-end rehearsal: the GPU suite, smoke() and the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread \
  > gpurun_out/r02c_final_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r02c_final_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02c_final_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r02c_final_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/r02c_final_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r02c_final_bench.log | cut -c1-400
