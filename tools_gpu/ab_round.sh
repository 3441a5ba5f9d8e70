cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
V="$GRAFT_REPO_ROOT/build/abvar"
for sc in "cornell_box 800 961 5" "cornell_smoke 800 961 5" "final_scene 800 400 5"; do
  timeout -k 10 300 python -u tools_gpu/ab_src.py $sc $V/v0 $V/v1 $V/v2 >> gpurun_out/r04_ab1.log 2>&1 || exit 1
done
grep -E "kernel ms|jit" gpurun_out/r04_ab1.log
bash tools_gpu/rehearse_n2.sh r04_rehearse_n2 | cut -c1-3000
