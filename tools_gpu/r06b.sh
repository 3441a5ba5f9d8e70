cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
AB_SETS="-DRT_F64W" timeout -k 10 400 python3 tools_gpu/ab_macro.py cornell_box 800 1000 2 50 > gpurun_out/r06b_ab_f32w_c2.log 2>&1 || { tail -20 gpurun_out/r06b_ab_f32w_c2.log; exit 1; }
tail -2 gpurun_out/r06b_ab_f32w_c2.log
AB_SETS="-DRT_F64W" timeout -k 10 400 python3 tools_gpu/ab_macro.py cornell_smoke 800 1000 2 10 > gpurun_out/r06b_ab_f32w_c3.log 2>&1 || { tail -20 gpurun_out/r06b_ab_f32w_c3.log; exit 1; }
tail -2 gpurun_out/r06b_ab_f32w_c3.log
bash tools_gpu/gpu_tests.sh r06b_gputest tests/test_gpu_parity.py -k "scene_parity or c1 or damaged or jit or zero_pdf or special"
