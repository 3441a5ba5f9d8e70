set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u tools_gpu/prof_obvh.py final_scene 800 100 > gpurun_out/r03_prof_obvh_c4.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/r03_prof_obvh_c4.log; exit 1; }
cat gpurun_out/r03_prof_obvh_c4.log
for sc in "cornell_box 800 961" "cornell_smoke 800 961"; do
set -- $sc
AB_SCENE_ENVS=";RT_NO_SCENE_SET=1" timeout -k 10 300 python -u tools_gpu/ab_scene_env.py $sc 3 > gpurun_out/r03_ab_scene_set_$1.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/r03_ab_scene_set_$1.log; exit 1; }
echo "== $sc"; head -3 gpurun_out/r03_ab_scene_set_$1.log
done
timeout -k 10 600 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03_c5_bench.log 2>&1 || { echo BENCH_FAIL; tail -5 gpurun_out/r03_c5_bench.log; exit 1; }
tail -1 gpurun_out/r03_c5_bench.log | cut -c1-400
