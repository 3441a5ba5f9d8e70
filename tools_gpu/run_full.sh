#!/bin/bash
# The round-end checks as the driver runs them: every GPU test, smoke(), then the default bench.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_all.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
