set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for a in "cornell_box 800 100" "final_scene 800 100"; do
timeout -k 10 200 python -u tools_gpu/prof_sections.py $a > gpurun_out/r03_sections.log 2>&1 || { echo SEC_FAIL; tail -20 gpurun_out/r03_sections.log; exit 1; }
cat gpurun_out/r03_sections.log
timeout -k 10 200 python -u tools_gpu/prof_obvh.py $a 2>&1 | tail -12
done
