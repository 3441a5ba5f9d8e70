"""One render through the C ABI for profiling: python tools_gpu/one_render.py [scene width spp reps]"""
import os
import sys
if os.environ.get("AB_TORCH", "1") == "1":
    import torch  # noqa: F401  (as bench.py: torch's bundled hiprtc builds the scene kernels)
sys.path.insert(0, "surely-raytracing_amd")
import surely_rt as rt  # noqa: E402

if os.environ.get("RT_LIB"):  # profiling a library variant (tools only; the product loads build/)
    rt._dev = rt.load_device_lib(os.environ["RT_LIB"])

scene = sys.argv[1] if len(sys.argv) > 1 else "cornell_box"
W = int(sys.argv[2]) if len(sys.argv) > 2 else 800
spp = int(sys.argv[3]) if len(sys.argv) > 3 else 100
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 1
blob, cam = rt.preset_blob(scene, width=W, spp=spp)
ds = rt.DeviceScene(blob)
for _ in range(reps):
    acc, st = ds.render(cam, rt.make_opts(cam, seed=1))
    print(f"{scene} {W} spp {cam.samples_per_pixel}: {st.ms_kernel:.2f} ms, "
          f"{st.samples / st.ms_kernel / 1e3:.1f} Msamples/s", flush=True)
