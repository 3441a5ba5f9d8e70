"""A/B of render-time environment settings (read at every render, e.g. RT_NO_BVH_ROWS,
RT_SEG_PAIRS), interleaved on ONE device scene in one process; images must be identical.
Usage: python ab_renderenv.py SCENE W SPP ROUNDS 'K=V,K2=V2' ['K=V' ...]  ('-' = no settings)"""
import os
import sys

import torch  # noqa: F401  (the benchmark's hiprtc)
sys.path.insert(0, "surely-raytracing_amd")
import numpy as np  # noqa: E402
import surely_rt as rt  # noqa: E402

scene, W, SPP, ROUNDS = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
blob, cam = rt.preset_blob(scene, width=W, spp=SPP)
opts = rt.make_opts(cam, seed=1)
ds = rt.DeviceScene(blob)
specs = sys.argv[5:]
envs = [{} if sp == "-" else dict(kv.split("=", 1) for kv in sp.split(",")) for sp in specs]


def render(env):
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return ds.render(cam, opts)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k)
            else:
                os.environ[k] = v


ref, _ = render(envs[0])
ms = [[] for _ in specs]
for r in range(ROUNDS):
    for i, env in enumerate(envs):
        acc, st = render(env)
        assert np.array_equal(acc, ref, equal_nan=True), f"{specs[i]}: image differs"
        ms[i].append(st.ms_kernel)
    print(f"round {r}: " + "  ".join(f"{m[-1]:.2f}" for m in ms), flush=True)
base = np.median(ms[0])
for sp, m in zip(specs, ms):
    print(f"{scene} {sp:36s} kernel ms min {min(m):9.2f} med {np.median(m):9.2f} "
          f"({np.median(m) / base - 1:+.2%})", flush=True)
