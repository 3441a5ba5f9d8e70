set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools_gpu/r03_ab_exact.sh || exit 1
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_parity.py -k "multi or book2 or frames_vs_oracle" -s > gpurun_out/r03_pytest_new.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/r03_pytest_new.log; exit 1; }
grep -E "PASS|FAIL|max \|d\||rt_multi|passed|failed" gpurun_out/r03_pytest_new.log | tail -20
