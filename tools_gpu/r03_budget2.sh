set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools_gpu/prof_sections.py final_scene 800 100 2>&1 | grep -E "kernel|lanes alive"
RT_PROF_LIB=build/prof_b10/librtmi355x.so timeout -k 10 200 python -u tools_gpu/prof_sections.py final_scene 800 100 2>&1 | grep -E "kernel|lanes alive"
