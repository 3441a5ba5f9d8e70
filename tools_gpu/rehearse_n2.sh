#!/bin/bash
# bench.py's N > 1 path on a one-GPU box: two ranks under torch.distributed.run, gloo, both on
# device 0 (RT_BENCH_REHEARSAL=1). Usage: bash tools_gpu/rehearse_n2.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-rehearse_n2}
mkdir -p gpurun_out
RT_BENCH_REHEARSAL=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 \
  > gpurun_out/$TAG.log 2>&1 || { echo N2_FAIL; tail -30 gpurun_out/$TAG.log; exit 1; }
grep '^{' gpurun_out/$TAG.log
