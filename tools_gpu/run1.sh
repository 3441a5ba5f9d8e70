#!/bin/bash
# first GPU round: parity tests -> smoke -> bench
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
echo "nproc=$(nproc)" > gpurun_out/env.txt
rocm-smi --showproductname >> gpurun_out/env.txt 2>&1
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/env.txt
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench.log 2>&1
