"""A/B of kernel-source variants selected by -D macros in the scene-specialised kernel
(RT_JIT_OPTS is read when the module is built, so every set runs in its own child process;
sets alternate with the default, ROUNDS times). Reports kernel ms (min / median over the renders
of each child) and the image's max |d| per sample against the default's, for variants whose
arithmetic is meant to differ in the last bits.
Usage: AB_SETS="-DX;-DY" python tools_gpu/ab_macro.py scene W SPP [rounds] [depth]"""
import os
import subprocess
import sys

import numpy as np

scene, W, SPP = sys.argv[1], sys.argv[2], sys.argv[3]
ROUNDS = int(sys.argv[4]) if len(sys.argv) > 4 else 2
DEPTH = sys.argv[5] if len(sys.argv) > 5 else "0"
SETS = [""] + [x.strip() for x in os.environ.get("AB_SETS", "").split(";") if x.strip()]
OUT = os.environ.get("AB_OUT", "gpurun_out/ab_macro")
os.makedirs(OUT, exist_ok=True)
CHILD = r"""
import sys, os
import torch  # as bench.py: torch's bundled hiprtc builds the scene kernels
sys.path.insert(0, "surely-raytracing_amd")
import numpy as np, surely_rt as rt
kw = dict(width=int(sys.argv[2]), spp=int(sys.argv[3]))
if int(sys.argv[4]) > 0:
    kw["depth"] = int(sys.argv[4])
blob, cam = rt.preset_blob(sys.argv[1], **kw)
ds = rt.DeviceScene(blob)
ms = []
for r in range(4):
    acc, st = ds.render(cam, rt.make_opts(cam, seed=1, flags=rt.RT_FLAG_OVERWRITE))
    if r: ms.append(st.ms_kernel)
np.save(sys.argv[5], acc)
print(f"RESULT {min(ms):.3f} {np.median(ms):.3f} {cam.samples_per_pixel} {ds.jit_info()[0]}")
"""
res = {s: [] for s in SETS}
spp_eff = None
for r in range(ROUNDS):
    for i, o in enumerate(SETS):
        env = dict(os.environ, RT_JIT_OPTS=o)
        npy = f"{OUT}/set{i}.npy"
        out = subprocess.run([sys.executable, "-c", CHILD, scene, W, SPP, DEPTH, npy], env=env,
                             capture_output=True, text=True, timeout=300)
        line = [l for l in out.stdout.splitlines() if l.startswith("RESULT")]
        if not line:
            print(f"{o or 'default'}: FAILED {out.stderr[-800:]}", flush=True)
            sys.exit(1)
        mn, md, spp_eff, js = line[0].split()[1:]
        res[o].append((float(mn), float(md)))
        print(f"round {r} {o or 'default':40s} min {mn} med {md} jit {js}", flush=True)
ref = np.load(f"{OUT}/set0.npy").astype(np.float64)
base = min(m for m, _ in res[""])
for i, o in enumerate(SETS):
    img = np.load(f"{OUT}/set{i}.npy").astype(np.float64)
    d = np.abs(img - ref) / float(spp_eff)
    fin = np.isfinite(d)
    mn = min(m for m, _ in res[o])
    print(f"{o or 'default':40s} best min {mn:9.3f} ms ({100 * (mn / base - 1):+.2f} %)  "
          f"max|d|/spp {d[fin].max() if fin.any() else float('nan'):.3e}  "
          f"nan/inf mask equal {bool(np.array_equal(np.isfinite(img), np.isfinite(ref)))}", flush=True)
for i in range(len(SETS)):  # the images are large; gpurun copies back at most 64 MiB
    os.remove(f"{OUT}/set{i}.npy")
