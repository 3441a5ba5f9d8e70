cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
AB_SETS="-DRT_ABL_TWICE_BVH=1;-DRT_ABL_TWICE_BVH=2;-DRT_ABL_LEAF2;-DRT_ABL_NOISE2;-DRT_ABL_RUV2;-DRT_ABL_FRESH2;-DRT_ABL_HIT2;-DRT_ABL_RNG2;-DRT_ABL_TRAV2" timeout -k 10 600 python3 tools_gpu/ab_macro.py final_scene 800 400 1 40 > gpurun_out/r06h_abl_c4.log 2>&1 || { tail -20 gpurun_out/r06h_abl_c4.log; exit 1; }
tail -10 gpurun_out/r06h_abl_c4.log
