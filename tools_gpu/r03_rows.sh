set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 600 --timeout-method thread -s tests/test_gpu_parity.py -k "chunked or frames_vs_oracle or random or c5 or ragged or degenerate or multi" > gpurun_out/r03_pytest_rows.log 2>&1 || { echo PYTEST_FAIL; grep -E "PASS|FAIL|Error|error" gpurun_out/r03_pytest_rows.log | tail -30; exit 1; }
grep -E "max \|d\||C5 share|passed|failed" gpurun_out/r03_pytest_rows.log | tail -8
for sc in "cornell_box 800 961" "cornell_smoke 800 961"; do
set -- $sc
AB_SCENE_ENVS=";RT_SEG_PAIRS=1000000000" timeout -k 10 300 python -u tools_gpu/ab_scene_env.py $sc 3 > gpurun_out/r03_ab_rows_$1.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/r03_ab_rows_$1.log; exit 1; }
echo "== $sc"; head -3 gpurun_out/r03_ab_rows_$1.log
done
timeout -k 10 300 python -u tools_gpu/scaling_probe.py 800 1000 > gpurun_out/r03_scaling_probe_rows.log 2>&1 || { echo PROBE_FAIL; tail gpurun_out/r03_scaling_probe_rows.log; exit 1; }
RT_SEG_PAIRS=1000000000 RT_TAIL_PAIRS=5120 timeout -k 10 300 python -u tools_gpu/scaling_probe.py 800 1000 > gpurun_out/r03_scaling_probe_segs.log 2>&1 || { echo PROBE_FAIL; tail gpurun_out/r03_scaling_probe_segs.log; exit 1; }
echo "== rows"; cat gpurun_out/r03_scaling_probe_rows.log; echo "== segments"; cat gpurun_out/r03_scaling_probe_segs.log
