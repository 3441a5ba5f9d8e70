#!/bin/bash
# GPU parity suite, then interleaved A/B of build/ vs build/variants for C2, C3, C4
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread \
  > gpurun_out/r02c_pytest.log 2>&1
rc=$?; tail -4 gpurun_out/r02c_pytest.log; [ $rc -eq 0 ] || exit $rc
for spec in "800 1000 3 cornell_box" "800 1000 2 cornell_smoke" "800 400 2 final_scene"; do
  set -- $spec
  timeout -k 10 400 python -u tools_gpu/ab_variants.py $spec > gpurun_out/r02c_ab_$4.log 2>&1 || exit $?
  tail -3 gpurun_out/r02c_ab_$4.log
done
