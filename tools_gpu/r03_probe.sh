set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools_gpu/probe_c4_launches.py 2>&1 | grep -v amdgpu.ids
