#!/bin/bash
# Round profiles at the current head: C2/C3/C4 kernel stats + PMC traffic + bench lines, then C5.
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools_gpu/profile_round.sh r01c c2 3 || exit $?
bash tools_gpu/profile_round.sh r01c c3 2 || exit $?
bash tools_gpu/profile_round.sh r01c c4 1 || exit $?
timeout -k 10 600 python3 bench.py --config c5 --steps 1 --warmup 1 > gpurun_out/prof_r01c_c5_bench.log 2>&1
