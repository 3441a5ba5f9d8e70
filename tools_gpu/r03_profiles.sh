#!/bin/bash
# Round-3 profiles: per config rocprofv3 kernel stats, PMC FETCH_SIZE / WRITE_SIZE passes and the
# bench line (tools_gpu/profile_round.sh), then the default bench (C2, with the CPU baseline).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=${1:-r03a}
for CFG in c2 c3 c4; do
  bash tools_gpu/profile_round.sh $R $CFG 3 || { echo "PROFILE_FAIL $CFG"; exit 1; }
  echo "== $CFG"; tail -1 gpurun_out/prof_${R}_${CFG}/bench.log | cut -c1-600
done
timeout -k 10 600 python3 -u bench.py > gpurun_out/${R}_bench_default.log 2>&1 || { echo BENCH_FAIL; tail -5 gpurun_out/${R}_bench_default.log; exit 1; }
tail -1 gpurun_out/${R}_bench_default.log
