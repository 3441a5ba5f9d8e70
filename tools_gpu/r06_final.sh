#!/bin/bash
# Round-6 final check at the head: profiles (kernel stats, PMC traffic, bench) of c2/c3/c4, then
# smoke(), the default bench line and the -m gpu suite. Usage: bash tools_gpu/r06_final.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r06q}
for c in c2 c3 c4; do
  bash tools_gpu/profile_round.sh $T $c 3 || { echo "PROFILE_FAIL $c"; exit 1; }
  grep '^{' gpurun_out/prof_${T}_$c/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['roofline']['traffic'], d.get('speedup_vs_cpu'))"
done
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { cat gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
bash tools_gpu/gpu_tests.sh ${T}_gputest tests
