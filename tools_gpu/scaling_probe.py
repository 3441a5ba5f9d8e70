"""Strong-scaling probe on one GPU: time one rank's cyclic share (rows r::N) vs the full frame.
efficiency(N) ~= T_full / (N * max_r T_share(r)). Usage: python tools_gpu/scaling_probe.py [W spp]"""
import os
import sys
if os.environ.get("AB_TORCH", "1") == "1":
    import torch  # noqa: F401  (as bench.py: torch's bundled hiprtc builds the scene kernels)
sys.path.insert(0, "surely-raytracing_amd")
import numpy as np  # noqa: E402
import surely_rt as rt  # noqa: E402

if os.environ.get("RT_LIB"):  # a library variant (tools only)
    rt._dev = rt.load_device_lib(os.environ["RT_LIB"])
from surely_rt.parallel import cyclic_rows  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 1 else 800
SPP = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
SCENE = sys.argv[3] if len(sys.argv) > 3 else "cornell_box"
blob, cam = rt.preset_blob(SCENE, width=W, spp=SPP)
ds = rt.DeviceScene(blob)
H = cam.image_height


def t(opts, reps=3):
    ms = []
    for _ in range(reps):
        _, st = ds.render(cam, opts)
        ms.append(st.ms_kernel)
    return min(ms)


t(rt.make_opts(cam))
full = t(rt.make_opts(cam))
print(f"full frame {W}x{H} spp {cam.samples_per_pixel}: {full:.2f} ms", flush=True)
for N in (2, 4, 8):
    shares = []
    for r in range(N):
        b, s, n = cyclic_rows(H, r, N)
        shares.append(t(rt.make_opts(cam, row_begin=b, row_step=s, n_rows=n), reps=2))
    print(f"N={N}: shares ms {np.round(shares, 2).tolist()}  eff={full / (N * max(shares)):.3f}",
          flush=True)
