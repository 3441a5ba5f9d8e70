cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
AB_SETS="-DRT_F2I_BRANCH;-DRT_PERLIN_PROD;-DRT_F2I_BRANCH -DRT_PERLIN_PROD" timeout -k 10 600 python3 tools_gpu/ab_macro.py final_scene 800 400 2 40 > gpurun_out/r06i_ab_noise_c4.log 2>&1 || { tail -20 gpurun_out/r06i_ab_noise_c4.log; exit 1; }
tail -4 gpurun_out/r06i_ab_noise_c4.log
bash tools_gpu/gpu_tests.sh r06i_gputest tests/test_gpu_parity.py -k "saturating or perlin or noise or scene_parity or random_scene or checker"
