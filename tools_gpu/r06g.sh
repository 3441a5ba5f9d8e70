cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for cfg in "cornell_box 800 1000 2 50 c2" "cornell_smoke 800 1000 2 10 c3" "final_scene 800 400 2 40 c4"; do
  set -- $cfg
  AB_SETS="-DRT_RNG_STARSTAR" timeout -k 10 400 python3 tools_gpu/ab_macro.py $1 $2 $3 $4 $5 > gpurun_out/r06g_ab_rngstar_$6.log 2>&1 || { tail -20 gpurun_out/r06g_ab_rngstar_$6.log; exit 1; }
  tail -2 gpurun_out/r06g_ab_rngstar_$6.log
done
bash tools_gpu/gpu_tests.sh r06g_gputest tests
