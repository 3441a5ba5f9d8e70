cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06k_smoke.log 2>&1 || { cat gpurun_out/r06k_smoke.log; exit 1; }
tail -1 gpurun_out/r06k_smoke.log
timeout -k 10 300 python3 bench.py > gpurun_out/r06k_bench.log 2>&1 || { tail -5 gpurun_out/r06k_bench.log; exit 1; }
grep '^{' gpurun_out/r06k_bench.log | cut -c1-300
bash tools_gpu/gpu_tests.sh r06k_gputest tests
