set -o pipefail
cd $GRAFT_REPO_ROOT
for sc in cornell_smoke cornell_box; do
VARDIR=build/variants_gen timeout -k 10 300 python -u tools_gpu/ab_variants.py 800 961 3 $sc 2>&1 | grep -v amdgpu.ids
done
