"""One full frame and the 8 cyclic-row shares of it, for `rocprofv3 --kernel-trace`: the per-kernel
durations separate the path kernel's time from launch and reduction costs in the scaling probe.
Usage: rocprofv3 --kernel-trace --stats -d DIR -- python3 tools_gpu/share_trace.py [W spp N]"""
import sys

import torch  # noqa: F401  (as bench.py: torch's bundled hiprtc builds the scene kernels)

sys.path.insert(0, "surely-raytracing_amd")
import surely_rt as rt  # noqa: E402
from surely_rt.parallel import cyclic_rows  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 1 else 800
SPP = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
N = int(sys.argv[3]) if len(sys.argv) > 3 else 8
blob, cam = rt.preset_blob("cornell_box", width=W, spp=SPP)
ds = rt.DeviceScene(blob)
H = cam.image_height
for rep in range(2):
    _, st = ds.render(cam, rt.make_opts(cam))
    print(f"full: {st.ms_kernel:.2f} ms", flush=True)
    for r in range(N):
        b, s, n = cyclic_rows(H, r, N)
        _, st = ds.render(cam, rt.make_opts(cam, row_begin=b, row_step=s, n_rows=n))
        print(f"share {r}: {st.ms_kernel:.2f} ms", flush=True)
