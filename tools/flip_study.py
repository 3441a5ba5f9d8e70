"""Path-flip study: how often does a last-bit change of the arithmetic alone change
a path at BASELINE C4? Renders the same C4 rows with the f64 oracle (reference operation order)
and with the same oracle whose dot products are fused as the device evaluates them
(liboracle_f64fma.so; everything else identical), and reports flip pixels (f32 sums more than 4
ulps apart), their position (the 1000-sphere cluster's screen box: x 404-627, y 233-408), the
largest per-sample difference and the op-count differences. CPU only; test infrastructure.

Usage: python tools/flip_study.py [row_begin row_step n_rows [spp]]   (default 10 20 40 5000)
"""
import ctypes as C
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO / "tests"), str(REPO / "surely-raytracing_amd")]
import oracle_lib as O  # noqa: E402
import surely_rt as rt  # noqa: E402

b, s, n = (int(x) for x in sys.argv[1:4]) if len(sys.argv) >= 4 else (10, 20, 40)
spp = int(sys.argv[4]) if len(sys.argv) >= 5 else 5000
blob, cam = rt.preset_blob("final_scene", width=800, spp=spp, depth=40)
opts = rt.make_opts(cam, seed=1, row_begin=b, row_step=s, n_rows=n)
t0 = time.time()
ref, ops_r = O.render(blob, cam, opts, precision=64)
t1 = time.time()
L = O.lib(64)
F = C.CDLL(str(O.ORACLE_BUILD / "liboracle_f64fma.so"))
F.oracle_render.restype, F.oracle_render.argtypes = L.oracle_render.restype, L.oracle_render.argtypes
O._libs[64] = F
fma, ops_f = O.render(blob, cam, opts, precision=64)
t2 = time.time()
spp_e = cam.samples_per_pixel
d = np.abs(ref.astype(np.float64) - fma.astype(np.float64))
ulp = np.spacing(np.maximum(np.abs(ref), np.abs(fma))).astype(np.float64)
flip = (d > 4 * ulp).any(axis=2)
ys, xs = np.nonzero(flip)
rows = b + ys * s
in_cluster = ((xs >= 404) & (xs <= 627) & (rows >= 233) & (rows <= 408)).sum()
print(f"C4 rows {b}:{s}:{n}, {spp_e} spp: reference order {t1 - t0:.0f} s, fused dot {t2 - t1:.0f} s")
print(f"flip pixels {flip.sum()} of {flip.size} ({in_cluster} inside the sphere cluster's box); "
      f"max |d| per sample {d.max() / spp_e:.3e}")
for k in ops_r:
    if ops_r[k] != ops_f[k]:
        print(f"  {k}: {ops_r[k]} vs {ops_f[k]} (rel {abs(ops_r[k] - ops_f[k]) / max(ops_r[k], 1):.2e})")
