#!/bin/bash
# Round profile: rocprofv3 kernel stats of the bench command + PMC traffic passes, then bench.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=${1:-r01}
mkdir -p gpurun_out/prof_$R profiles
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$R/stats -o bench -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$R/stats.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/prof_$R/fetch -o bench -- python3 bench.py --steps 1 --warmup 0 --no-count --no-cpu-baseline > gpurun_out/prof_$R/fetch.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/prof_$R/write -o bench -- python3 bench.py --steps 1 --warmup 0 --no-count --no-cpu-baseline > gpurun_out/prof_$R/write.log 2>&1 || exit $?
# bench default: 800 x 800 x 961 samples, one rt_trace launch, 12 B of slot per sample
python3 tools_gpu/pmc_to_json.py profiles/pmc_traffic.json "gpurun_out/prof_$R/fetch/*counter_collection.csv" "gpurun_out/prof_$R/write/*counter_collection.csv" $((800*800*961*12)) > gpurun_out/prof_$R/traffic.log 2>&1
cp profiles/pmc_traffic.json gpurun_out/prof_$R/pmc_traffic.json
timeout -k 10 600 python3 bench.py > gpurun_out/prof_$R/bench.log 2>&1
