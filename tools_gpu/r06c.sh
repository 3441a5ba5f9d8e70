cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
AB_SETS="-DRT_SEED_PCG4D" timeout -k 10 400 python3 tools_gpu/ab_macro.py cornell_box 800 1000 2 50 > gpurun_out/r06c_ab_seed_c2.log 2>&1 || { tail -20 gpurun_out/r06c_ab_seed_c2.log; exit 1; }
tail -2 gpurun_out/r06c_ab_seed_c2.log
AB_SETS="-DRT_SEED_PCG4D" timeout -k 10 400 python3 tools_gpu/ab_macro.py cornell_smoke 800 1000 2 10 > gpurun_out/r06c_ab_seed_c3.log 2>&1 || { tail -20 gpurun_out/r06c_ab_seed_c3.log; exit 1; }
tail -2 gpurun_out/r06c_ab_seed_c3.log
AB_SETS="-DRT_F64W" timeout -k 10 400 python3 tools_gpu/ab_macro.py final_scene 800 400 2 40 > gpurun_out/r06c_ab_f32w_c4.log 2>&1 || { tail -20 gpurun_out/r06c_ab_f32w_c4.log; exit 1; }
tail -2 gpurun_out/r06c_ab_f32w_c4.log
bash tools_gpu/gpu_tests.sh r06c_gputest tests
timeout -k 10 300 python3 bench.py --config c4 --steps 3 --no-cpu-baseline > gpurun_out/r06c_c4_bench.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --config c2 --no-cpu-baseline > gpurun_out/r06c_c2_bench.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --config c3 --no-cpu-baseline > gpurun_out/r06c_c3_bench.log 2>&1 || exit $?
for c in c2 c3 c4; do python3 -c "import json; l=[x for x in open('gpurun_out/r06c_'+'$c'+'_bench.log') if x.startswith('{')]; d=json.loads(l[-1]); print('$c', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"; done
