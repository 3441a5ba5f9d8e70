cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
PMC_EXTRA="TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" timeout -k 10 900 bash tools_gpu/pmc_ab_env.sh final_scene 4900 gpurun_out/r06d_pmc_rows - RT_NO_BVH_ROWS=1 > gpurun_out/r06d_pmc_rows.log 2>&1 || { tail -30 gpurun_out/r06d_pmc_rows.log; exit 1; }
cat gpurun_out/r06d_pmc_rows.log
