#!/bin/bash
# PMC instruction mix of the current library vs the round-2 head variant (C2), then the
# section-cycle split of the profiling build
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools_gpu/pmc_ab.sh build/variants/librtmi355x_r02head.so gpurun_out/r02c_pmc > gpurun_out/r02c_pmc.log 2>&1 || exit $?
cat gpurun_out/r02c_pmc/summary_l1.txt gpurun_out/r02c_pmc/summary_l2.txt
timeout -k 10 200 python3 tools_gpu/prof_sections.py cornell_box 800 100 > gpurun_out/r02c_sec_c2.log 2>&1 || exit $?
cat gpurun_out/r02c_sec_c2.log
