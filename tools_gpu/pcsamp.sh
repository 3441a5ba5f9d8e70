#!/bin/bash
# PC sampling of one C2 render (instruction-level hotspots of rt_trace)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pcs
timeout -s KILL 120 rocprofv3 -L > gpurun_out/pcs/list.txt 2>&1
timeout -k 10 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1 --kernel-trace -d gpurun_out/pcs/run -o pcs --output-format csv -- python3 tools_gpu/one_render.py ${1:-cornell_box} 800 ${2:-100} > gpurun_out/pcs/run.log 2>&1
echo "rc=$?" >> gpurun_out/pcs/run.log
