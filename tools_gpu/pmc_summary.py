"""Sum rt_trace PMC counters over dispatches from tools_gpu/prof_pmc.sh output."""
import collections
import csv
import glob
import sys

out = sys.argv[1]
agg = collections.defaultdict(float)
for f in sorted(glob.glob(f"{out}/p*/*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if "rt_trace" in r.get("Kernel_Name", ""):
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
for k in sorted(agg):
    print(f"{k:28s} {agg[k]:.5g}")
if agg.get("SQ_ACTIVE_INST_VALU"):
    print(f"lane utilisation (THREAD_CYCLES_VALU / 64 ACTIVE_INST_VALU) "
          f"{agg['SQ_THREAD_CYCLES_VALU'] / (64 * agg['SQ_ACTIVE_INST_VALU']):.3f}")
wc = agg.get("SQ_WAVE_CYCLES")
if wc:
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
              "SQ_ACTIVE_INST_SCA"):
        print(f"{k:28s} / WAVE_CYCLES {agg.get(k, 0) / wc:.3f}")
