#!/bin/bash
# C4 (final_scene) after the LDS walk: section split (profiling build) and SQ issue/wait counters
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 tools_gpu/prof_sections.py final_scene 400 100 > gpurun_out/r02c_sec_c4_cbvh.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r02c_sec_c4_cbvh.log
O=gpurun_out/r02c_pmc_c4_cbvh
mkdir -p $O
j=0
for SET in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_INSTS_VALU_FMA_F64" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA" \
           "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_FLAT TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  j=$((j+1))
  timeout -k 10 120 rocprofv3 --pmc $SET --kernel-trace -d $O/p$j -o run --output-format csv -- python3 tools_gpu/one_render.py final_scene 400 100 > $O/p$j.log 2>&1 || exit $?
done
python3 tools_gpu/pmc_summary.py $O > $O/summary.txt 2>&1
cat $O/summary.txt
