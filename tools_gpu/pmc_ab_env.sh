#!/bin/bash
# PMC SQ passes (tools_gpu/pmc_sq.sh's two counter sets) of one scene under several scene-creation
# environment settings, each in its own profiled process. Usage:
#   bash tools_gpu/pmc_ab_env.sh SCENE SPP OUTDIR 'K=V' ['K=V' ...]   ('-' = no settings)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
SC=$1; SPP=$2; OUT=$3; shift 3
i=0
for SPEC in "$@"; do
  i=$((i+1))
  D=$OUT/v$i
  mkdir -p $D
  echo "$SPEC" > $D/spec.txt
  ENVS=""
  [ "$SPEC" != "-" ] && ENVS=$(echo "$SPEC" | tr ',' ' ')
  j=0
  for SET in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR" \
             "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA" \
             ${PMC_EXTRA:+"$PMC_EXTRA"}; do
    j=$((j+1))
    env $ENVS timeout -k 10 120 rocprofv3 --pmc $SET --kernel-trace -d $D/p$j -o run --output-format csv -- python3 tools_gpu/one_render.py $SC 800 $SPP > $D/p$j.log 2>&1 || exit $?
  done
  python3 tools_gpu/pmc_summary.py $D > $D/summary.txt 2>&1
  echo "== $SPEC"; cat $D/p1.log | grep -v amdgpu.ids | tail -1; cat $D/summary.txt
done
