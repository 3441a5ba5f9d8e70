set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cfg in "20480 1280" "10240 2560" "20480 2560" "40960 1280"; do
set -- $cfg
RT_SEG_PAIRS=$1 RT_TAIL_PAIRS=$2 timeout -k 10 300 python -u tools_gpu/scaling_probe.py 800 1000 > gpurun_out/r03_scaling_probe_seg$1_tail$2.log 2>&1 || { echo PROBE_FAIL; tail gpurun_out/r03_scaling_probe_seg$1_tail$2.log; exit 1; }
echo "== seg $1 tail $2"; grep -v amdgpu.ids gpurun_out/r03_scaling_probe_seg$1_tail$2.log
done
