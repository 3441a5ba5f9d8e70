#!/bin/bash
# Round-end rehearsal: the whole GPU suite, smoke() and the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=${1:-r03}
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -s \
  > gpurun_out/${R}_pytest.log 2>&1
rc=$?; grep -E "max \|d\||C5 share|rt_multi|black pixels" gpurun_out/${R}_pytest.log; tail -3 gpurun_out/${R}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/${R}_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/${R}_bench.log 2>&1 || exit $?
tail -1 gpurun_out/${R}_bench.log | cut -c1-300
