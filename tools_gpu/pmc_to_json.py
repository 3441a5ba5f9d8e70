"""Reduce rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes to per-launch HBM bytes of rt_trace.

MI355X_MICROARCH.md §HBM: FETCH_SIZE counts half the bytes of a 16-B/lane streaming read and
other access widths are uncalibrated. rt_trace does no streaming reads (scene records come from
K$/L2; the only bulk traffic is the 12-B per-sample slot stores), so the counters are reported
raw (KiB -> bytes, no x2), and WRITE_SIZE is calibrated against the known slot bytes of the
launch (argv[4] = samples per launch x 12 B).
Usage: pmc_to_json.py OUT.json FETCH_GLOB WRITE_GLOB [ALGORITHMIC_WRITE_BYTES]"""
import csv
import glob
import json
import sys

out = sys.argv[1]
algo_write = float(sys.argv[4]) if len(sys.argv) > 4 else None
vals = {}
for name, pat in (("FETCH_SIZE", sys.argv[2]), ("WRITE_SIZE", sys.argv[3])):
    per = []
    for f in glob.glob(pat):
        for r in csv.DictReader(open(f)):
            if "rt_trace" in r["Kernel_Name"] and r["Counter_Name"] == name:
                per.append(float(r["Counter_Value"]))
    vals[name] = sum(per) / max(1, len(per)) if per else None
fetch, write = vals["FETCH_SIZE"], vals["WRITE_SIZE"]
fb = fetch * 1024 if fetch is not None else None
wb = write * 1024 if write is not None else None
res = {
    "kernel": "rt_trace",
    "fetch_bytes_raw": fb,
    "write_bytes_raw": wb,
    "hbm_bytes_per_launch": fb + wb if fb is not None and wb is not None else None,
    "algorithmic_write_bytes": algo_write,
    "write_calibration": (wb / algo_write) if wb and algo_write else None,
    "note": "FETCH_SIZE + WRITE_SIZE per rt_trace launch, raw (no x2: no 16-B streaming reads "
            "in this kernel); write_calibration = WRITE_SIZE / known per-sample slot bytes",
}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
