"""Ordered-BVH walk statistics (build/prof, -DRT_PROF; not shipped): per walk kind (top-level =
world frame, instance = inside Translate/RotateY), lane box steps and leaves, their wave maxima
(SIMD efficiency = lane sum / (64 x wave-max sum)), wave cycles, and lanes re-walked in the
reference order. Usage: python tools_gpu/prof_obvh.py [scene width spp]"""
import ctypes as C
import os
import sys

if os.environ.get("AB_TORCH", "1") == "1":
    import torch  # noqa: F401  (as bench.py: torch's bundled hiprtc builds the scene kernels)
sys.path.insert(0, "surely-raytracing_amd")
import numpy as np  # noqa: E402
import surely_rt as rt  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "final_scene"
W = int(sys.argv[2]) if len(sys.argv) > 2 else 800
spp = int(sys.argv[3]) if len(sys.argv) > 3 else 100
lib = rt.load_device_lib("build/prof/librtmi355x.so")
blob, cam = rt.preset_blob(scene, width=W, spp=spp)
h = C.c_void_p()
assert lib.rt_scene_create(blob.ref(), 0, C.byref(h)) == 0, lib.rt_last_error()
opts = rt.make_opts(cam, seed=1)
for rep in range(2):
    acc = np.zeros((cam.image_height, cam.image_width, 3), np.float32)
    st = rt.RtStats()
    rc = lib.rt_render(h, C.byref(cam), C.byref(opts), acc.ctypes.data, C.byref(st))
    assert rc == 0, (rc, lib.rt_last_error())
cyc = np.array([st.ops[k] for k in range(8)], dtype=np.float64)
pc = (C.c_uint64 * 24)()
assert lib.rt_scene_prof_counters(h, pc, 24) == 0
o = [int(v) for v in pc]
print(f"{scene} {W} spp {cam.samples_per_pixel}: kernel {st.ms_kernel:.2f} ms (profiling build), "
      f"{st.samples} samples, path-loop wave-cycles {cyc.sum():.3e}")
for nm, b in (("top-level", 0), ("instance", 6)):
    w = o[b + 4]
    if not w:
        continue
    print(f"  {nm}: {w} wave-walks, {100 * o[b + 5] / cyc.sum():.1f} % of path-loop wave-cycles, "
          f"{o[b + 5] / w:.0f} cyc per wave-walk")
    print(f"    box steps: {o[b] / st.samples:.2f} lane/sample, wave-max {o[b + 1] / w:.1f} per walk, "
          f"SIMD eff {o[b] / (64.0 * max(1, o[b + 1])):.3f}")
    print(f"    leaves:    {o[b + 2] / st.samples:.2f} lane/sample, wave-max {o[b + 3] / w:.1f} per walk, "
          f"SIMD eff {o[b + 2] / (64.0 * max(1, o[b + 3])):.3f}")
print(f"  lanes re-walked in the reference order: {o[12]} ({o[12] / st.samples:.2e} per sample)")
pc2 = (C.c_uint64 * 24)()
for nm, k in (("top-level", 13), ("instance", 14)):
    if o[k]:
        print(f"  {nm} leaf tests (lane 0 of each wave, compact walk): {100 * o[k] / cyc.sum():.1f} % "
              f"of path-loop wave-cycles")
