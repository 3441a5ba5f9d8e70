#!/bin/bash
# Round profile for one BASELINE config: rocprofv3 kernel stats of the bench command, the two PMC
# traffic passes (FETCH_SIZE and WRITE_SIZE in separate runs), then the bench line itself.
# Usage: bash tools_gpu/profile_round.sh ROUND [c2|c3|c4] [bench steps]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=${1:-r02}; CFG=${2:-c2}; STEPS=${3:-3}
O=gpurun_out/prof_${R}_${CFG}
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o bench -- python3 bench.py --config $CFG --steps $STEPS --warmup 1 --no-cpu-baseline > $O/stats.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o bench -- python3 bench.py --config $CFG --steps 1 --warmup 0 --no-count --no-cpu-baseline > $O/fetch.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write -o bench -- python3 bench.py --config $CFG --steps 1 --warmup 0 --no-count --no-cpu-baseline > $O/write.log 2>&1 || exit $?
# workspace bytes one launch stores and its kernel time: bench.py's roofline block
ALGO=$(python3 -c "import json,sys; l=[x for x in open('$O/stats.log') if x.startswith('{')]; print(json.loads(l[-1])['roofline']['workspace_bytes_per_launch'])")
KMS=$(python3 -c "import json,sys; l=[x for x in open('$O/stats.log') if x.startswith('{')]; r=json.loads(l[-1])['roofline']; print(r['kernel_ms'] / r['launches_per_render'])")
python3 tools_gpu/pmc_to_json.py $O/pmc_traffic_$CFG.json "$O/fetch/*counter_collection.csv" "$O/write/*counter_collection.csv" $ALGO $KMS > $O/traffic.log 2>&1 || exit $?
mkdir -p profiles && cp $O/pmc_traffic_$CFG.json profiles/
timeout -k 10 600 python3 bench.py --config $CFG > $O/bench.log 2>&1
