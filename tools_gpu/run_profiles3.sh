#!/bin/bash
# Round profile of the three single-GPU BASELINE configs (rocprof stats, PMC traffic, bench line).
cd "$GRAFT_REPO_ROOT" || exit 1
R=${1:-r01b}
for c in c2 c3 c4; do
  bash tools_gpu/profile_round.sh $R $c 3 || exit $?
done
