set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools_gpu/r03_flips.py c4 10 20 40 > gpurun_out/r03_flips_c4.log 2>&1 || { echo FAIL_C4; tail -20 gpurun_out/r03_flips_c4.log; exit 1; }
cat gpurun_out/r03_flips_c4.log
timeout -k 10 300 python -u tools_gpu/r03_flips.py c2 > gpurun_out/r03_flips_c2.log 2>&1 || { echo FAIL_C2; tail -20 gpurun_out/r03_flips_c2.log; exit 1; }
cat gpurun_out/r03_flips_c2.log
timeout -k 10 300 python -u tools_gpu/r03_flips.py c3 > gpurun_out/r03_flips_c3.log 2>&1 || { echo FAIL_C3; tail -20 gpurun_out/r03_flips_c3.log; exit 1; }
cat gpurun_out/r03_flips_c3.log
