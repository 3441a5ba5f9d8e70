#!/bin/bash
# Round-6 head check: the N = 2 self-launch rehearsal, C2 and C4 bench lines, then the -m gpu suite.
# Usage: bash tools_gpu/r06_check.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r06}
mkdir -p gpurun_out
RT_BENCH_REHEARSAL=1 timeout -k 10 300 python3 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/${T}_selflaunch_n2.log 2>&1 || { echo SELF_FAIL; tail -20 gpurun_out/${T}_selflaunch_n2.log; exit 1; }
grep '^{' gpurun_out/${T}_selflaunch_n2.log | cut -c1-400
timeout -k 10 300 python3 bench.py --config c2 --no-cpu-baseline > gpurun_out/${T}_c2_bench.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --config c4 --steps 3 --no-cpu-baseline > gpurun_out/${T}_c4_bench.log 2>&1 || exit $?
for c in c2 c4; do python3 -c "import json; l=[x for x in open('gpurun_out/${T}_'+'$c'+'_bench.log') if x.startswith('{')]; d=json.loads(l[-1]); print('$c', d['value'], d['roofline']['kernel_ms'])"; done
bash tools_gpu/gpu_tests.sh ${T}_gputest
