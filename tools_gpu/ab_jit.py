"""Interleaved A/B of the scene-specialised kernel (default product path) against the interpreter
walker (RT_FLAG_INTERPRETER) in one process; images must be identical.
Usage: python tools_gpu/ab_jit.py [scene width spp rounds]"""
import sys
import time

sys.path.insert(0, "surely-raytracing_amd")
import numpy as np  # noqa: E402
import surely_rt as rt  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "cornell_box"
W = int(sys.argv[2]) if len(sys.argv) > 2 else 800
SPP = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
ROUNDS = int(sys.argv[4]) if len(sys.argv) > 4 else 3
blob, cam = rt.preset_blob(scene, width=W, spp=SPP)
ds = rt.DeviceScene(blob)
t0 = time.time()
acc_j, _ = ds.render(cam, rt.make_opts(cam, seed=1))
print(f"first product render (incl. JIT compile) {time.time() - t0:.2f} s; jit_info {ds.jit_info()[0]}",
      flush=True)
res = {"jit": [], "interp": []}
img = {}
for r in range(ROUNDS):
    for k, fl in (("jit", rt.RT_FLAG_OVERWRITE), ("interp", rt.RT_FLAG_OVERWRITE | rt.RT_FLAG_INTERPRETER)):
        acc, st = ds.render(cam, rt.make_opts(cam, seed=1, flags=fl))
        res[k].append(st.ms_kernel)
        img[k] = acc
for k, v in res.items():
    print(f"{scene} {k:7s} kernel ms min {min(v):9.2f} med {np.median(v):9.2f} "
          f"Msamples/s {st.samples / min(v) / 1e3:8.1f}", flush=True)
print("identical:", np.array_equal(img["jit"], img["interp"]), "first==jit:", np.array_equal(acc_j, img["jit"]))
