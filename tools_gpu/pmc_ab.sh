#!/bin/bash
# PMC passes (SQ instruction mix, issue/wait) for the product library and a variant, C2 at spp 100.
# Usage: bash tools_gpu/pmc_ab.sh VARIANT.so OUTDIR
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
VAR=$1; OUT=${2:-gpurun_out/pmcab}
mkdir -p $OUT/l1 $OUT/l2
i=0
for LIB in build/librtmi355x.so $VAR; do
  i=$((i+1)); j=0
  for SET in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_INSTS_VALU_FMA_F64" \
             "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA"; do
    j=$((j+1))
    RT_LIB=$LIB timeout -k 10 120 rocprofv3 --pmc $SET --kernel-trace -d $OUT/l$i/p$j -o run --output-format csv -- python3 tools_gpu/one_render.py ${SCENE:-cornell_box} 800 ${SPP:-1000} > $OUT/l$i/p$j.log 2>&1 || exit $?
  done
  python3 tools_gpu/pmc_summary.py $OUT/l$i > $OUT/summary_l$i.txt 2>&1
done
