#!/bin/bash
# GPU parity suite, A/B of C4 against the head variant, then the one-GPU scaling probe of C2 and
# the C5 bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread \
  > gpurun_out/r02c_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r02c_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools_gpu/ab_variants.py 800 400 2 final_scene > gpurun_out/r02c_ab_final_scene.log 2>&1 || exit $?
tail -3 gpurun_out/r02c_ab_final_scene.log
timeout -k 10 300 python -u tools_gpu/scaling_probe.py > gpurun_out/r02c_scaling_probe.log 2>&1 || exit $?
tail -6 gpurun_out/r02c_scaling_probe.log
timeout -k 10 400 python -u bench.py --config c5 --steps 1 --warmup 1 --no-count --no-cpu-baseline > gpurun_out/r02c_c5_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r02c_c5_bench.log
