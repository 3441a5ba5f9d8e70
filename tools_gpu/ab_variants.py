"""A/B the library variants under build/variants in ONE process, interleaved rounds
(cdna_hip_programming.md §5.4 rule 24). Usage: python tools_gpu/ab_variants.py [width spp rounds]"""
import ctypes as C
import glob
import os
import sys
import time

if os.environ.get("AB_TORCH", "1") == "1":
    import torch  # noqa: F401  (bench.py imports torch first: its bundled hiprtc builds the kernels)
sys.path.insert(0, "surely-raytracing_amd")
import numpy as np  # noqa: E402
import surely_rt as rt  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 1 else 800
SPP = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
ROUNDS = int(sys.argv[3]) if len(sys.argv) > 3 else 3
SCENE = sys.argv[4] if len(sys.argv) > 4 else "cornell_box"
VARDIR = os.environ.get("VARDIR", "build/variants")
paths = ["build/librtmi355x.so"] + sorted(glob.glob(f"{VARDIR}/*.so"))
# AB_ENVS="K=V,K2=V2;K=V3": extra entries rendering with the default library under these
# environment settings (read by the library at each render call)
envs = {p: {} for p in paths}
for spec in filter(None, os.environ.get("AB_ENVS", "").split(";")):
    key = "build/librtmi355x.so[" + spec + "]"
    paths.append(key)
    envs[key] = dict(kv.split("=", 1) for kv in spec.split(","))
blob, cam = rt.preset_blob(SCENE, width=W, spp=SPP)
libs, scenes = [], []
for p in paths:
    if "[" in p:
        lib = libs[0]
    else:
        try:
            lib = rt.load_device_lib(p)
        except AttributeError:  # an older ABI (e.g. a previous round's library): plain ctypes
            lib = C.CDLL(p)
    h = C.c_void_p()
    assert lib.rt_scene_create(blob.ref(), 0, C.byref(h)) == 0, lib.rt_last_error()
    libs.append(lib)
    scenes.append(h)
opts = rt.make_opts(cam, seed=1)
res = {p: [] for p in paths}
ref = None
for r in range(ROUNDS + 1):
    for p, lib, h in zip(paths, libs, scenes):
        acc = np.zeros((cam.image_height, cam.image_width, 3), np.float32)
        st = rt.RtStats()
        ev = dict(envs[p])
        o2 = rt.make_opts(cam, seed=1, flags=rt.RT_FLAG_OVERWRITE | int(ev.pop("FLAGS", "0"), 0))
        saved = {k: os.environ.get(k) for k in ev}
        os.environ.update(ev)
        assert lib.rt_render(h, C.byref(cam), C.byref(o2), acc.ctypes.data, C.byref(st)) == 0
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k)
            else:
                os.environ[k] = v
        if ref is None:
            ref = acc
        same = np.array_equal(acc, ref)
        if r > 0:
            res[p].append(st.ms_kernel)
        if r == ROUNDS:
            print(f"{p:45s} kernel ms min {min(res[p]):9.2f} med {np.median(res[p]):9.2f}  "
                  f"Msamples/s {st.samples / min(res[p]) / 1e3:8.1f}  same_as_default {same}", flush=True)
