cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
AB_SETS="-DRT_MIN_WAVES_GEN=6;-DRT_MIN_WAVES_GEN=4" timeout -k 10 400 python3 tools_gpu/ab_macro.py cornell_box 800 1000 2 50 > gpurun_out/r06e_ab_waves_c2.log 2>&1 || { tail -20 gpurun_out/r06e_ab_waves_c2.log; exit 1; }
tail -3 gpurun_out/r06e_ab_waves_c2.log
AB_SETS="-DRT_MIN_WAVES_GEN=6;-DRT_MIN_WAVES_GEN=4" timeout -k 10 400 python3 tools_gpu/ab_macro.py cornell_smoke 800 1000 2 10 > gpurun_out/r06e_ab_waves_c3.log 2>&1 || { tail -20 gpurun_out/r06e_ab_waves_c3.log; exit 1; }
