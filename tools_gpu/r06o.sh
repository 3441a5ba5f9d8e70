cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
RT_BENCH_REHEARSAL=1 timeout -k 10 300 python3 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/r06o_selflaunch_n2.log 2>&1 || { echo SELF_FAIL; tail -20 gpurun_out/r06o_selflaunch_n2.log; exit 1; }
grep '^{' gpurun_out/r06o_selflaunch_n2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('N=2', d['value'], d['n_gpus'], d['gather'], d['ranks']['step_ms_per_rank'])"
timeout -k 10 300 python3 bench.py > gpurun_out/r06o_c2_bench.log 2>&1 || exit $?
grep '^{' gpurun_out/r06o_c2_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('N=1', d['value'], d['roofline']['frac'], d['roofline']['traffic'], d['config']['precision'][:40])"
