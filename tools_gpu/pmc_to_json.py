"""Reduce rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes to per-launch HBM bytes of rt_trace.

MI355X_MICROARCH.md §HBM: FETCH_SIZE counts half the bytes of a 16-B/lane streaming read and
other access widths are uncalibrated. rt_trace's reads are scalar scene-record loads (K$/L2),
per-lane BVH/leaf records and scratch spill reloads, none of them 16-B/lane streaming, so
FETCH_SIZE is reported raw (KiB -> bytes, no x2). Its stores are the f64 row partials / tail
samples (24 B per lane-store) plus any scratch spill write-backs, so WRITE_SIZE is calibrated
per launch against the known output bytes of one launch (argv[4], bench.py's
algorithmic_bytes_per_launch): write_calibration = 1 means no extra write traffic.
Usage: pmc_to_json.py OUT.json FETCH_GLOB WRITE_GLOB [WORKSPACE_WRITE_BYTES_PER_LAUNCH [KERNEL_MS]]
The JSON records the kernel-source hash of the profiled tree (surely_rt.roofline) and the
profiled kernel time, so bench.py can refuse a stale profile."""
import csv
import glob
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "surely-raytracing_amd"))
from surely_rt.roofline import kernel_source_sha16  # noqa: E402

out = sys.argv[1]
algo_write = float(sys.argv[4]) if len(sys.argv) > 4 and sys.argv[4] else None
kernel_ms = float(sys.argv[5]) if len(sys.argv) > 5 and sys.argv[5] else None
vals, n = {}, {}
for name, pat in (("FETCH_SIZE", sys.argv[2]), ("WRITE_SIZE", sys.argv[3])):
    per = []
    for f in glob.glob(pat):
        for r in csv.DictReader(open(f)):
            if "rt_trace" in r["Kernel_Name"] and r["Counter_Name"] == name:
                per.append(float(r["Counter_Value"]))
    vals[name] = sum(per) / max(1, len(per)) if per else None
    n[name] = len(per)
fetch, write = vals["FETCH_SIZE"], vals["WRITE_SIZE"]
fb = fetch * 1024 if fetch is not None else None
wb = write * 1024 if write is not None else None
res = {
    "kernel": "rt_trace",
    "launches_profiled": n,
    "fetch_bytes": fb,
    "write_bytes": wb,
    "hbm_bytes_per_launch": fb + wb if fb is not None and wb is not None else None,
    "workspace_write_bytes_per_launch": algo_write,
    "write_calibration": (wb / algo_write) if wb and algo_write else None,
    "kernel_source_sha16": kernel_source_sha16(),
    "profiled_kernel_ms": kernel_ms,
    "note": "FETCH_SIZE + WRITE_SIZE (KiB -> B) averaged over the rt_trace launches of the pass, "
            "raw (no x2: no 16-B streaming reads in this kernel); write_calibration = WRITE_SIZE "
            "/ the launch's f64 workspace stores (1 = no spill / extra write traffic)",
}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
