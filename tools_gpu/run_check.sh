#!/bin/bash
# GPU tests, then bench lines for the given configs (scene-specialised, and RT_JIT=0 for A/B).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_all.log 2>&1 || exit $?
for c in "$@"; do
  timeout -k 10 300 python -u bench.py --config $c --steps 2 --no-cpu-baseline --no-count > gpurun_out/bench_$c.log 2>&1 || exit $?
  RT_JIT=0 timeout -k 10 300 python -u bench.py --config $c --steps 2 --no-cpu-baseline --no-count > gpurun_out/bench_${c}_interp.log 2>&1 || exit $?
done
