# bench.py's N > 1 path on a one-GPU box: two ranks under torch.distributed.run, gloo, both on
# device 0 (RT_BENCH_REHEARSAL=1); then N = 1 for comparison
set -o pipefail
cd $GRAFT_REPO_ROOT
RT_BENCH_REHEARSAL=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 \
  > gpurun_out/r03_rehearse_n2.log 2>&1 || { echo N2_FAIL; tail -30 gpurun_out/r03_rehearse_n2.log; exit 1; }
grep '^{' gpurun_out/r03_rehearse_n2.log | cut -c1-700
