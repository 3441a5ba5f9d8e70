#!/bin/bash
# PMC SQ passes (instruction mix; issue, wait and lane utilisation) of the product library for one
# scene. Usage: bash tools_gpu/pmc_sq.sh SCENE SPP OUTDIR
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
SC=$1; SPP=$2; OUT=$3
mkdir -p $OUT
j=0
for SET in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_INSTS_VALU_FMA_F64" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA"; do
  j=$((j+1))
  timeout -k 10 120 rocprofv3 --pmc $SET --kernel-trace -d $OUT/p$j -o run --output-format csv -- python3 tools_gpu/one_render.py $SC 800 $SPP > $OUT/p$j.log 2>&1 || exit $?
done
python3 tools_gpu/pmc_summary.py $OUT > $OUT/summary.txt 2>&1
