#!/bin/bash
# What the driver runs at round end: smoke(), then the default bench line
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02c_smoke.log 2>&1 || { tail -5 gpurun_out/r02c_smoke.log; exit 1; }
tail -1 gpurun_out/r02c_smoke.log
SECONDS=0; timeout -k 10 600 python -u bench.py > gpurun_out/r02c_bench_default.log 2> gpurun_out/r02c_bench_default.err || { tail -5 gpurun_out/r02c_bench_default.err; exit 1; }
tail -1 gpurun_out/r02c_bench_default.log
echo "bench wall s: $SECONDS"
