#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools_gpu/profile_round.sh r01 c2 3 || exit $?
bash tools_gpu/profile_round.sh r01 c3 2 || exit $?
bash tools_gpu/profile_round.sh r01 c4 1 || exit $?
