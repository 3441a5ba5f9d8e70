cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
RT_FULL_FRAME_PARITY=1 bash tools_gpu/gpu_tests.sh r06j_c4_full tests/test_gpu_parity.py tests/test_c4_frame_parity_gpu.py -k "C4b or remaining"
