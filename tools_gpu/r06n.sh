cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
AB_SETS="-mllvm -amdgpu-sched-strategy=iterative-minreg;-mllvm -amdgpu-sched-strategy=max-ilp;-mllvm -misched=ilpmin" timeout -k 10 600 python3 tools_gpu/ab_jitopts.py cornell_box 800 1000 > gpurun_out/r06n_jitopts_c2.log 2>&1 || { tail -20 gpurun_out/r06n_jitopts_c2.log; exit 1; }
cat gpurun_out/r06n_jitopts_c2.log
