"""A/B of the scene-specialised BVH kernel (RT_JIT_BVH=1, read once per process) against the
interpreter BVH kernel, alternating child processes; images must hash equal.
Usage: python tools_gpu/ab_jitbvh.py [scene W SPP]"""
import os
import subprocess
import sys

scene = sys.argv[1] if len(sys.argv) > 1 else "final_scene"
W = sys.argv[2] if len(sys.argv) > 2 else "800"
SPP = sys.argv[3] if len(sys.argv) > 3 else "400"
CHILD = r"""
import sys, hashlib
sys.path.insert(0, "surely-raytracing_amd")
import numpy as np, surely_rt as rt
blob, cam = rt.preset_blob(sys.argv[1], width=int(sys.argv[2]), spp=int(sys.argv[3]))
ds = rt.DeviceScene(blob)
ms = []
for r in range(4):
    acc, st = ds.render(cam, rt.make_opts(cam, seed=1, flags=rt.RT_FLAG_OVERWRITE))
    if r: ms.append(st.ms_kernel)
print(f"RESULT {min(ms):.2f} {np.median(ms):.2f} {st.samples / min(ms) / 1e3:.1f} "
      f"{hashlib.sha1(acc.tobytes()).hexdigest()[:12]} jit={ds.jit_info()[0]}")
"""
for jb in ("0", "1", "0", "1"):
    out = subprocess.run([sys.executable, "-c", CHILD, scene, W, SPP],
                         env=dict(os.environ, RT_JIT_BVH=jb), capture_output=True, text=True,
                         timeout=300)
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("RESULT")]
    print(f"RT_JIT_BVH={jb} {line[0] if line else 'FAILED rc=%d %s' % (out.returncode, out.stderr[-400:])}",
          flush=True)
    if not line:
        sys.exit(1)
