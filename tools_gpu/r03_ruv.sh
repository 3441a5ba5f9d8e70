set -o pipefail
cd $GRAFT_REPO_ROOT
for a in "800 961 3 cornell_smoke" "800 400 3 final_scene"; do
VARDIR=build/variants_ruv timeout -k 10 300 python -u tools_gpu/ab_variants.py $a 2>&1 | grep -v amdgpu.ids
done
