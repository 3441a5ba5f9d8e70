"""A/B of hiprtc compiler options for the scene-specialised kernel (RT_JIT_OPTS is read at the
module build, so every option set runs in its own child process; the default runs first and
last). Images must equal the default's (hash). Usage: python tools_gpu/ab_jitopts.py scene W SPP"""
import hashlib
import os
import subprocess
import sys

scene, W, SPP = sys.argv[1], sys.argv[2], sys.argv[3]
SETS = ["", "-mllvm -amdgpu-sched-strategy=iterative-minreg", "-mllvm -misched=ilpmin",
        "-mllvm -amdgpu-sched-strategy=max-ilp", "-mllvm -misched=ilpmax", ""]
if os.environ.get("AB_SETS"):  # ';'-separated option sets (the default runs first and last)
    SETS = [""] + [x.strip() for x in os.environ["AB_SETS"].split(";")] + [""]
CHILD = r"""
import sys, hashlib, os
if os.environ.get("AB_TORCH", "1") == "1":
    import torch  # as bench.py: torch's bundled hiprtc builds the scene kernels
sys.path.insert(0, "surely-raytracing_amd")
import numpy as np, surely_rt as rt
blob, cam = rt.preset_blob(sys.argv[1], width=int(sys.argv[2]), spp=int(sys.argv[3]))
ds = rt.DeviceScene(blob)
ms = []
for r in range(4):
    acc, st = ds.render(cam, rt.make_opts(cam, seed=1, flags=rt.RT_FLAG_OVERWRITE))
    if r: ms.append(st.ms_kernel)
print(f"RESULT {min(ms):.2f} {np.median(ms):.2f} {hashlib.sha1(acc.tobytes()).hexdigest()[:12]}")
"""
for o in SETS:
    env = dict(os.environ, RT_JIT_OPTS=o)
    out = subprocess.run([sys.executable, "-c", CHILD, scene, W, SPP], env=env, capture_output=True,
                         text=True, timeout=240)
    line = [l for l in out.stdout.splitlines() if l.startswith("RESULT")]
    print(f"{o or 'default':55s} {line[0] if line else 'FAILED ' + out.stderr[-300:]}", flush=True)
    if not line:
        sys.exit(1)
