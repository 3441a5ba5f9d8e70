#!/bin/bash
# parity + bench + rocprofv3 kernel stats + PMC counters
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" > gpurun_out/rc.txt
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/stats -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_stats.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/prof/pmc1 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-count --width 400 --spp 100 > gpurun_out/prof_pmc1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA --kernel-trace -d gpurun_out/prof/pmc2 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-count --width 400 --spp 100 > gpurun_out/prof_pmc2.log 2>&1
