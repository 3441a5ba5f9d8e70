set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VARDIR=build/variants timeout -k 10 400 python -u tools_gpu/ab_variants.py 800 961 3 cornell_box > gpurun_out/r03_abl_c2.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/r03_abl_c2.log; exit 1; }
cat gpurun_out/r03_abl_c2.log
