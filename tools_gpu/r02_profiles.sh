#!/bin/bash
# round 2 profiles: kernel stats + PMC traffic + bench line for c2, c3, c4
set -o pipefail
for c in ${CFGS:-c2 c3 c4}; do
  bash tools_gpu/profile_round.sh ${R:-r02} $c ${STEPS:-3} || exit $?
  tail -1 gpurun_out/prof_${R:-r02}_$c/bench.log
done
