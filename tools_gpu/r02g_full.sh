set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests -m gpu > gpurun_out/r02g_pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/r02g_pytest.log; exit 1; }
tail -3 gpurun_out/r02g_pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r02g_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/r02g_smoke.log; exit 1; }
tail -1 gpurun_out/r02g_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r02g_bench.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/r02g_bench.log; exit 1; }
tail -1 gpurun_out/r02g_bench.log | cut -c1-400
