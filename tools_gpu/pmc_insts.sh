#!/bin/bash
# SQ instruction counts (one PMC pass) of C2 at spp 100 for the product library and each ablation
# variant in $VARDIR: the difference to the product is the ablated section's dynamic instruction count.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmcins}; VARDIR=${VARDIR:-build/variants_ab}
mkdir -p $OUT
for LIB in build/librtmi355x.so $VARDIR/*.so; do
  n=$(basename $LIB .so)
  RT_LIB=$LIB timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_INSTS_VALU_FMA_F64 --kernel-trace -d $OUT/$n -o run --output-format csv -- python3 tools_gpu/one_render.py cornell_box 800 100 > $OUT/$n.log 2>&1 || exit $?
done
