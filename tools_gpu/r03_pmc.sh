set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools_gpu/pmc_sq.sh cornell_box 961 gpurun_out/pmc_r03_c2 || { echo PMC_FAIL c2; tail gpurun_out/pmc_r03_c2/p*.log; exit 1; }
bash tools_gpu/pmc_sq.sh final_scene 400 gpurun_out/pmc_r03_c4 || { echo PMC_FAIL c4; tail gpurun_out/pmc_r03_c4/p*.log; exit 1; }
bash tools_gpu/pmc_sq.sh cornell_smoke 961 gpurun_out/pmc_r03_c3 || { echo PMC_FAIL c3; tail gpurun_out/pmc_r03_c3/p*.log; exit 1; }
for c in c2 c3 c4; do echo "== $c"; cat gpurun_out/pmc_r03_$c/summary.txt; done
