#!/bin/bash
# C5 bench line (no op-count pass: 83 G samples) and the single-GPU strong-scaling probe of C2.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools_gpu/scaling_probe.py > gpurun_out/scaling_probe.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --config c5 --steps 1 --warmup 1 --no-count --no-cpu-baseline > gpurun_out/bench_c5.log 2>&1
