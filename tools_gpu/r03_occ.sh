set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for sc in cornell_box cornell_smoke; do
VARDIR=build/variants_jocc timeout -k 10 300 python -u tools_gpu/ab_variants.py 800 961 3 $sc > gpurun_out/r03_ab_occ_$sc.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/r03_ab_occ_$sc.log; exit 1; }
echo "== $sc"; cat gpurun_out/r03_ab_occ_$sc.log
done
