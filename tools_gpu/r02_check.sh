#!/bin/bash
# round 2: GPU parity suite, then C2 and C4 bench lines (no CPU baseline)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r02_pytest.log 2>&1
rc=$?
tail -5 gpurun_out/r02_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r02_c2.log 2>&1 || exit $?
tail -1 gpurun_out/r02_c2.log
timeout -k 10 300 python -u bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r02_c4.log 2>&1 || exit $?
tail -1 gpurun_out/r02_c4.log
