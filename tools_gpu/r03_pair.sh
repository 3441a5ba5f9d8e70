set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "lds_global or chunked or ragged or bvh or final_scene or random" > gpurun_out/r03_pytest_pair.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/r03_pytest_pair.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/r03_pytest_pair.log | tail -30
AB_SCENE_ENVS=";RT_NO_PAIR=1" timeout -k 10 300 python -u tools_gpu/ab_scene_env.py final_scene 800 400 3 > gpurun_out/r03_ab_pair_c4.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/r03_ab_pair_c4.log; exit 1; }
cat gpurun_out/r03_ab_pair_c4.log
