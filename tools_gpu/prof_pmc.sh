#!/bin/bash
# SQ instruction-mix / stall passes on one render; each pass is its own rocprofv3 run (--pmc with
# --kernel-trace only). Usage: bash tools_gpu/prof_pmc.sh OUTDIR [scene width spp]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc2}; SC=${2:-cornell_box}; W=${3:-800}; SPP=${4:-100}
mkdir -p $OUT
i=0
for SET in "SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_SALU SQ_INSTS_SMEM" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT64 SQ_INSTS_BRANCH SQ_INST_CYCLES_SALU SQ_INSTS_LDS SQ_CYCLES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $SET --kernel-trace -d $OUT/p$i -o run --output-format csv -- python3 tools_gpu/one_render.py $SC $W $SPP > $OUT/p$i.log 2>&1 || exit $?
done
python3 tools_gpu/pmc_summary.py $OUT > $OUT/summary.txt 2>&1
