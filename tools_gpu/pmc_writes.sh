#!/bin/bash
# Where an rt_trace launch's write traffic comes from: vector-memory store instructions (SQ) and
# the L2's memory-side write requests (TCC), each pass its own run of the bench's workload.
# Usage: bash tools_gpu/pmc_writes.sh TAG CFG...   (CFG = c2 | c3 | c4)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=$1; shift
for CFG in "$@"; do
  O=gpurun_out/${TAG}_$CFG
  mkdir -p $O
  j=0
  for SET in "SQ_WAVES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH" \
             "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
    j=$((j+1))
    timeout -s KILL 240 rocprofv3 --pmc $SET --kernel-trace -d $O/p$j -o run --output-format csv -- python3 bench.py --config $CFG --steps 1 --warmup 0 --no-count --no-cpu-baseline > $O/p$j.log 2>&1 || exit $?
  done
  python3 tools_gpu/pmc_summary.py $O > $O/summary.txt 2>&1
  echo "== $CFG"; cat $O/summary.txt
done
