#!/bin/bash
# interleaved A/B of the default library against $VARDIR/*.so (ablation/variant builds) on C2 [and C4]
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export VARDIR=${VARDIR:-build/variants_ab}
timeout -k 10 300 python -u tools_gpu/ab_variants.py 800 1000 3 cornell_box > gpurun_out/ab_c2.log 2>&1 || exit $?
if [ "${C4:-0}" = 1 ]; then
timeout -k 10 300 python -u tools_gpu/ab_variants.py 800 400 2 final_scene > gpurun_out/ab_c4.log 2>&1 || exit $?
fi
