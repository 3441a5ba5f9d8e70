set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "multi or lds_global or chunked" -s > gpurun_out/r03_pytest_multi.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/r03_pytest_multi.log; exit 1; }
grep -E "PASS|FAIL|rt_multi|passed|failed" gpurun_out/r03_pytest_multi.log | tail -8
timeout -k 10 300 python -u tools_gpu/prof_obvh.py final_scene 800 100 > gpurun_out/r03_prof_cbvh_c4.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/r03_prof_cbvh_c4.log; exit 1; }
cat gpurun_out/r03_prof_cbvh_c4.log
VARDIR=build/variants_cbvh timeout -k 10 300 python -u tools_gpu/ab_variants.py 800 400 3 final_scene > gpurun_out/r03_ab_cbvh_c4.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/r03_ab_cbvh_c4.log; exit 1; }
cat gpurun_out/r03_ab_cbvh_c4.log
