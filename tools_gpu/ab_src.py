"""A/B of kernel-source variants in ONE process, interleaved rounds. Each variant is a directory
holding the JIT headers (rt_kernel.h, rt_layout.h, rt_rng.h, rt_mi355x.h); "-" = the library's
embedded headers. The variant's RT_JIT_SRC_DIR is set while its scene compiles its
scene-specialised kernel (first render), then removed. Images must be identical.
Usage: python tools_gpu/ab_src.py SCENE W SPP ROUNDS DIR_A DIR_B ..."""
import os
import sys

if os.environ.get("AB_TORCH", "1") == "1":
    import torch  # noqa: F401  (as bench.py)
sys.path.insert(0, "surely-raytracing_amd")
import numpy as np  # noqa: E402
import surely_rt as rt  # noqa: E402

scene = sys.argv[1]
W, SPP, ROUNDS = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
variants = sys.argv[5:]
blob, cam = rt.preset_blob(scene, width=W, spp=SPP)
opts = rt.make_opts(cam, seed=1)
scenes = []
for v in variants:
    if v != "-":
        os.environ["RT_JIT_SRC_DIR"] = v
    ds = rt.DeviceScene(blob)
    ds.render(cam, opts)  # compiles this variant's kernel
    os.environ.pop("RT_JIT_SRC_DIR", None)
    st, msg = ds.jit_info()
    print(f"{v}: jit {st} {msg.splitlines()[0] if msg else ''}", flush=True)
    scenes.append((v, ds))
res = {v: [] for v, _ in scenes}
ref = None
for r in range(ROUNDS):
    for v, ds in scenes:
        acc, st = ds.render(cam, opts)
        if ref is None:
            ref = acc
        assert np.array_equal(acc, ref, equal_nan=True), f"{v}: image differs"
        res[v].append(st.ms_kernel)
    print(f"round {r}: " + "  ".join(f"{res[v][-1]:.2f}" for v, _ in scenes), flush=True)
base = np.median(res[scenes[0][0]])
for v, _ in scenes:
    m = np.median(res[v])
    print(f"{scene} {v:40s} kernel ms min {min(res[v]):9.2f} med {m:9.2f} ({m / base - 1:+.2%})  "
          f"Msamples/s {cam.image_width * cam.image_height * cam.samples_per_pixel / m / 1e3:8.1f}",
          flush=True)
