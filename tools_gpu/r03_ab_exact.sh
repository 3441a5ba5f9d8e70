set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export VARDIR=build/variants_exact
timeout -k 10 200 python -u tools_gpu/ab_variants.py 800 1000 3 cornell_box > gpurun_out/r03_ab_exact_c2.log 2>&1 || { echo FAIL; tail gpurun_out/r03_ab_exact_c2.log; exit 1; }
cat gpurun_out/r03_ab_exact_c2.log
timeout -k 10 200 python -u tools_gpu/ab_variants.py 800 1000 3 cornell_smoke > gpurun_out/r03_ab_exact_c3.log 2>&1 || { echo FAIL; tail gpurun_out/r03_ab_exact_c3.log; exit 1; }
cat gpurun_out/r03_ab_exact_c3.log
timeout -k 10 300 python -u tools_gpu/ab_variants.py 800 400 3 final_scene > gpurun_out/r03_ab_exact_c4.log 2>&1 || { echo FAIL; tail gpurun_out/r03_ab_exact_c4.log; exit 1; }
cat gpurun_out/r03_ab_exact_c4.log
