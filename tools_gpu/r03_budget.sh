set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VARDIR=build/variants_c4b timeout -k 10 400 python -u tools_gpu/ab_variants.py 800 400 3 final_scene > gpurun_out/r03_ab_c4_budget.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/r03_ab_c4_budget.log; exit 1; }
cat gpurun_out/r03_ab_c4_budget.log
