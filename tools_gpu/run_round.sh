#!/bin/bash
# GPU parity tests, then the round profile (rocprof stats + PMC traffic + bench)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
R=${1:-r01}
timeout -k 10 900 python -m pytest tests -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" > gpurun_out/rc.txt
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools_gpu/profile_round.sh $R
