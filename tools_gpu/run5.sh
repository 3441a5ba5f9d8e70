#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" > gpurun_out/rc.txt
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python tools_gpu/ab_variants.py 800 1000 3 > gpurun_out/ab.log 2>&1 || exit $?
timeout -k 10 300 python tools_gpu/prof_sections.py cornell_box 800 1000 > gpurun_out/prof_sections.log 2>&1 || exit $?
timeout -k 10 300 python tools_gpu/prof_sections.py cornell_box 800 100 >> gpurun_out/prof_sections.log 2>&1
