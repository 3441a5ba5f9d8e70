set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_parity.py -k "scene_parity or random or jit or zero_pdf or nested or isotropic or image_texture or degenerate" > gpurun_out/r03_pytest_scset.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/r03_pytest_scset.log; exit 1; }
tail -3 gpurun_out/r03_pytest_scset.log
for sc in "cornell_box 800 961" "cornell_smoke 800 961" "final_scene 800 400"; do
AB_SCENE_ENVS=";RT_NO_SCENE_SET=1" timeout -k 10 300 python -u tools_gpu/ab_scene_env.py $sc 3 > gpurun_out/r03_ab_scset.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/r03_ab_scset.log; exit 1; }
echo "== $sc"; head -3 gpurun_out/r03_ab_scset.log
done
