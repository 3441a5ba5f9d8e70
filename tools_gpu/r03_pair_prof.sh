set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u tools_gpu/prof_obvh.py final_scene 800 100 > gpurun_out/r03_prof_pair_c4.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/r03_prof_pair_c4.log; exit 1; }
RT_NO_PAIR=1 timeout -k 10 200 python -u tools_gpu/prof_obvh.py final_scene 800 100 >> gpurun_out/r03_prof_pair_c4.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/r03_prof_pair_c4.log; exit 1; }
cat gpurun_out/r03_prof_pair_c4.log
