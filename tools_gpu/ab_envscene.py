"""A/B of scene-creation environment settings (read while the scene is flattened and its trees
are built), interleaved in one process; images must be identical.
Usage: python ab_envscene.py SCENE W SPP ROUNDS 'K=V,K2=V2' ['K=V' ...]  ('-' = no settings)"""
import os
import sys

import torch  # noqa: F401  (the benchmark's hiprtc)
sys.path.insert(0, "surely-raytracing_amd")
import numpy as np  # noqa: E402
import surely_rt as rt  # noqa: E402

scene, W, SPP, ROUNDS = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
blob, cam = rt.preset_blob(scene, width=W, spp=SPP)
opts = rt.make_opts(cam, seed=1)
vs = []
for spec in sys.argv[5:]:
    env = {} if spec == "-" else dict(kv.split("=", 1) for kv in spec.split(","))
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    ds = rt.DeviceScene(blob)
    ds.render(cam, opts)
    st, msg = ds.jit_info()
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k)
        else:
            os.environ[k] = v
    print(f"{spec}: jit {st} {msg.splitlines()[0] if msg else ''}", flush=True)
    vs.append((spec, ds, []))
ref = None
for r in range(ROUNDS):
    for spec, ds, ms in vs:
        acc, st = ds.render(cam, opts)
        if ref is None:
            ref = acc
        if os.environ.get("AB_ANY_IMAGE") != "1":  # AB_ANY_IMAGE=1: timing of variants whose
            # images legitimately differ (another RNG stream)
            assert np.array_equal(acc, ref, equal_nan=True), f"{spec}: image differs"
        ms.append(st.ms_kernel)
    print(f"round {r}: " + "  ".join(f"{m[-1]:.2f}" for _, _, m in vs), flush=True)
base = np.median(vs[0][2])
for spec, _, ms in vs:
    print(f"{scene} {spec:30s} kernel ms min {min(ms):9.2f} med {np.median(ms):9.2f} "
          f"({np.median(ms) / base - 1:+.2%})", flush=True)
