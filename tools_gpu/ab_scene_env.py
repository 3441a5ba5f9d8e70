"""A/B of scene-creation settings in ONE process, interleaved rounds: each entry of AB_SCENE_ENVS
("" = default; "K=V,K2=V2;K=V3") is applied while its scene is created (rt_scene_create reads it
at flatten time, e.g. RT_CBVH2=1), then removed. Usage:
  AB_SCENE_ENVS=";RT_CBVH2=1" python tools_gpu/ab_scene_env.py final_scene 800 400 3"""
import os
import sys

if os.environ.get("AB_TORCH", "1") == "1":
    import torch  # noqa: F401  (as bench.py: torch's bundled hiprtc builds the scene kernels)
sys.path.insert(0, "surely-raytracing_amd")
import numpy as np  # noqa: E402
import surely_rt as rt  # noqa: E402

scene = sys.argv[1]
W, SPP, ROUNDS = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
specs = os.environ.get("AB_SCENE_ENVS", ";").split(";")
blob, cam = rt.preset_blob(scene, width=W, spp=SPP)
scenes = []
for spec in specs:
    env = dict(kv.split("=", 1) for kv in spec.split(",") if kv)
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    scenes.append((spec or "default", rt.DeviceScene(blob), rt.layout_stats(blob)))
    for k, v in old.items():
        if v is None:
            os.environ.pop(k)
        else:
            os.environ[k] = v
res = {s[0]: [] for s in scenes}
ref = None
for r in range(ROUNDS + 1):
    for name, ds, _ in scenes:
        acc, st = ds.render(cam, rt.make_opts(cam, seed=1))
        if ref is None:
            ref = acc
        same = np.array_equal(acc, ref, equal_nan=True)
        if r > 0:
            res[name].append(st.ms_kernel)
        if r == ROUNDS:
            print(f"{name:24s} kernel ms min {min(res[name]):9.2f} med {np.median(res[name]):9.2f}  "
                  f"Msamples/s {st.samples / min(res[name]) / 1e3:8.1f}  same_as_first {same}",
                  flush=True)
for name, _, ls in scenes:
    print(name, ls)
