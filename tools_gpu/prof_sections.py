"""Wave-cycle split of the path loop by section (build/prof, -DRT_PROF; not shipped).
Usage: python tools_gpu/prof_sections.py [scene width spp]"""
import ctypes as C
import os
import sys

if os.environ.get("AB_TORCH", "1") == "1":
    import torch  # noqa: F401  (as bench.py: torch's bundled hiprtc builds the scene kernels)

sys.path.insert(0, "surely-raytracing_amd")
import numpy as np  # noqa: E402
import surely_rt as rt  # noqa: E402

NAMES = ["pool/regen", "traverse", "hit record", "emit/metal/dielectric", "lambert sample",
         "light pdf", "beta update", "exit"]
scene = sys.argv[1] if len(sys.argv) > 1 else "cornell_box"
W = int(sys.argv[2]) if len(sys.argv) > 2 else 800
spp = int(sys.argv[3]) if len(sys.argv) > 3 else 100
lib = rt.load_device_lib(os.environ.get("RT_PROF_LIB", "build/prof/librtmi355x.so"))
blob, cam = rt.preset_blob(scene, width=W, spp=spp)
h = C.c_void_p()
assert lib.rt_scene_create(blob.ref(), 0, C.byref(h)) == 0, lib.rt_last_error()
opts = rt.make_opts(cam, seed=1)
for rep in range(2):
    acc = np.zeros((cam.image_height, cam.image_width, 3), np.float32)
    st = rt.RtStats()
    assert lib.rt_render(h, C.byref(cam), C.byref(opts), acc.ctypes.data, C.byref(st)) == 0
cyc = np.array([st.ops[k] for k in range(8)], dtype=np.float64)
print(f"{scene} {W} spp {cam.samples_per_pixel}: kernel {st.ms_kernel:.2f} ms (profiling build)")
print(f"  lanes alive at traversal: {st.ops[8] / max(1, st.ops[9]):.2f} of 64 "
      f"({st.ops[9]} wave-iterations)")
for n, c in zip(NAMES, cyc):
    print(f"  {n:24s} {100 * c / cyc.sum():6.2f} %   {c / st.samples:9.1f} wave-cyc/sample")
o = [st.ops[10 + k] for k in range(16)]
if o[7]:
    tot = cyc.sum()
    print(f"  BVH subtree walks: {o[7]} wave-calls; wave-cycles top-level {100 * o[0] / tot:.1f} %, "
          f"in-transform {100 * o[1] / tot:.1f} %, volume boundary {100 * o[2] / tot:.1f} %")
    print(f"  LANE walker node steps: sum-of-lanes top {o[5]}, in-transform {o[6]}; "
          f"wave max-steps top {o[3]}, in-transform {o[4]}")
    for nm, s_, m_ in (("top", o[5], o[3]), ("in-transform", o[6], o[4])):
        if m_:
            print(f"    {nm}: SIMD efficiency of the AABB steps {s_ / (64.0 * m_):.3f}, "
                  f"{s_ / st.samples:.2f} lane-steps/sample, {64.0 * m_ / st.samples:.2f} wave-step-slots/sample")
if o[12]:
    names = ["leaf dispatch / other leaves", "inner BVH steps", "leaf header load", "QUADS batches"]
    print("  LANE walker sections (wave-level; profiling waits distort a little):")
    for k in range(4):
        print(f"    {names[k]:30s} {100 * o[8 + k] / tot:5.1f} %  count {o[12 + k]:>11d}  "
              f"{o[8 + k] / max(1, o[12 + k]):8.0f} cyc per count")
