cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python3 tools_gpu/ab_envscene.py final_scene 800 400 3 - RT_SAH_W=0.5:0.5:1 RT_SAH_W=0.25:0.25:1 RT_SAH_W=0.5:0.5:1,RT_SAH_W_BOXES=1 RT_SAH_W=2:2:1 RT_SAH_W=1:1:0.5 RT_SAH_W=0.05:0.05:1,RT_SAH_W_BOXES=1 > gpurun_out/r06m_ab_sahw_c4.log 2>&1 || { tail -20 gpurun_out/r06m_ab_sahw_c4.log; exit 1; }
tail -8 gpurun_out/r06m_ab_sahw_c4.log
