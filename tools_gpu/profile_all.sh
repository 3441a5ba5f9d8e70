#!/bin/bash
# Round profiles of the three one-GPU BASELINE configs (tools_gpu/profile_round.sh) and their bench
# lines. Usage: bash tools_gpu/profile_all.sh ROUND
cd "$GRAFT_REPO_ROOT" || exit 1
R=${1:-r04}
for c in c2:3 c3:3 c4:1; do
  bash tools_gpu/profile_round.sh $R ${c%:*} ${c#*:} || exit $?
  echo "== ${c%:*}"; grep -h '^{' gpurun_out/prof_${R}_${c%:*}/bench.log | cut -c1-400
  grep -h "rt_trace" gpurun_out/prof_${R}_${c%:*}/stats/*kernel_stats.csv | cut -c1-200
done
