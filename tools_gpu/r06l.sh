cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for cfg in "cornell_box 800 1000 2 50 c2" "final_scene 800 400 2 40 c4"; do
  set -- $cfg
  AB_SETS="-DRT_SCHLICK_CR" timeout -k 10 400 python3 tools_gpu/ab_macro.py $1 $2 $3 $4 $5 > gpurun_out/r06l_ab_schlick_$6.log 2>&1 || { tail -20 gpurun_out/r06l_ab_schlick_$6.log; exit 1; }
  tail -2 gpurun_out/r06l_ab_schlick_$6.log
done
