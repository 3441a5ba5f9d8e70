cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
AB_SETS="-DRT_ABL_TRAV2;-DRT_ABL_LPDF2;-DRT_ABL_FRESH2;-DRT_ABL_RNG2;-DRT_ABL_HIT2;-DRT_ABL_NOXS" timeout -k 10 500 python3 tools_gpu/ab_macro.py cornell_box 800 1000 2 50 > gpurun_out/r06f_abl_c2.log 2>&1 || { tail -20 gpurun_out/r06f_abl_c2.log; exit 1; }
tail -7 gpurun_out/r06f_abl_c2.log
AB_SETS="-DRT_ABL_TRAV2;-DRT_ABL_RUV2;-DRT_ABL_FRESH2;-DRT_ABL_RNG2;-DRT_ABL_HIT2" timeout -k 10 500 python3 tools_gpu/ab_macro.py cornell_smoke 800 1000 2 10 > gpurun_out/r06f_abl_c3.log 2>&1 || { tail -20 gpurun_out/r06f_abl_c3.log; exit 1; }
tail -6 gpurun_out/r06f_abl_c3.log
