#!/bin/bash
# Round-6 head profile: rocprofv3 kernel stats + PMC traffic passes + bench line for c2, c3, c4
# (tools_gpu/profile_round.sh), then the SQ passes of c2 and c4 (tools_gpu/pmc_sq.sh).
# Usage: bash tools_gpu/r06_profile.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r06p}
for c in c2 c3 c4; do
  bash tools_gpu/profile_round.sh $T $c 3 || { echo "PROFILE_FAIL $c"; exit 1; }
  grep '^{' gpurun_out/prof_${T}_$c/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['roofline']['traffic'], d.get('speedup_vs_cpu'))"
done
bash tools_gpu/pmc_sq.sh cornell_box 1000 gpurun_out/${T}_pmc_sq_c2 || exit 1
bash tools_gpu/pmc_sq.sh final_scene 4900 gpurun_out/${T}_pmc_sq_c4 || exit 1
grep -E "lane util|WAIT|FMA_F64|INSTS_VALU " gpurun_out/${T}_pmc_sq_c2/summary.txt gpurun_out/${T}_pmc_sq_c4/summary.txt
timeout -k 10 400 python3 bench.py --config c5 --steps 2 --warmup 1 > gpurun_out/${T}_c5_bench.log 2>&1 || exit $?
grep '^{' gpurun_out/${T}_c5_bench.log | cut -c1-200
