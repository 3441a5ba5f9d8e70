"""Frame-scale device-vs-oracle comparison: python tools_gpu/r03_flips.py CFG [rows...]

CFG: c2 | c3 | c4.  Renders the HIP product kernel, the HIP op-counting kernel and the f64 oracle
(16 threads) on the same rows and reports, per config:
  * max |d| of the per-sample average and the number of pixels above 1e-4;
  * "flip pixels": raw f32 sums differing by more than 4 f32 ulps (rounding alone moves a sum by
    at most ~1 ulp; a path that took another branch moves it by a whole sample's radiance);
  * op-count differences per category.
Flip pixels are saved to gpurun_out/flips_<cfg>.npz for tracing on the CPU.
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, "surely-raytracing_amd")
sys.path.insert(0, "tests")
import oracle_lib as O  # noqa: E402
import surely_rt as rt  # noqa: E402

CFG = {
    "c2": ("cornell_box", dict(width=800, spp=1000)),
    "c3": ("cornell_smoke", dict(width=800, spp=1000, depth=10)),
    "c4": ("final_scene", dict(width=800, spp=5000, depth=40)),
}
cfg = sys.argv[1]
name, kw = CFG[cfg]
rows = tuple(int(x) for x in sys.argv[2:5]) if len(sys.argv) >= 5 else (0, 1, 800)
threads = int(os.environ.get("ORACLE_THREADS", "16"))
blob, cam = rt.preset_blob(name, **kw)
b, s, n = rows
ds = rt.DeviceScene(blob)
t0 = time.time()
acc_p, st_p = ds.render(cam, rt.make_opts(cam, seed=1, row_begin=b, row_step=s, n_rows=n))
t1 = time.time()
acc_c, st_c = ds.render(cam, rt.make_opts(cam, seed=1, row_begin=b, row_step=s, n_rows=n,
                                          flags=rt.RT_FLAG_OVERWRITE | rt.RT_FLAG_COUNT_OPS))
t2 = time.time()
ds.close()
print(f"{cfg}: rows {rows}, device product {t1 - t0:.1f} s, counting {t2 - t1:.1f} s", flush=True)
same = np.array_equal(acc_p, acc_c, equal_nan=True)
print(f"  product == counting build bitwise: {same}", flush=True)
t3 = time.time()
acc_o, ops_o = O.render(blob, cam, rt.make_opts(cam, seed=1, row_begin=b, row_step=s, n_rows=n),
                        precision=64, threads=threads)
t4 = time.time()
spp = cam.samples_per_pixel
print(f"  oracle {t4 - t3:.1f} s on {threads} threads "
      f"({n * cam.image_width * spp / (t4 - t3) / 1e6:.2f} Msamples/s)", flush=True)
nan_same = np.array_equal(np.isnan(acc_p), np.isnan(acc_o))
inf_same = np.array_equal(np.isinf(acc_p), np.isinf(acc_o))
fin = np.isfinite(acc_p) & np.isfinite(acc_o)
d = np.where(fin, np.abs(acc_p.astype(np.float64) - acc_o.astype(np.float64)), 0.0)
davg = d / spp
ulp = np.spacing(np.maximum(np.abs(acc_p), np.abs(acc_o)).astype(np.float32)).astype(np.float64)
flip = (d > 4 * ulp).any(axis=2) | ~(np.isnan(acc_p) == np.isnan(acc_o)).all(axis=2)
print(f"  NaN masks equal {nan_same}, inf masks equal {inf_same}, NaN channels "
      f"{int(np.isnan(acc_p).sum())}", flush=True)
print(f"  max |d| per sample {davg.max():.3e}; pixels > 1e-4: {int((davg > 1e-4).any(axis=2).sum())}"
      f"; flip pixels: {int(flip.sum())} of {flip.size}", flush=True)
ops_g = st_c.op_counts()
diff = {k: (ops_g[k], ops_o[k]) for k in ops_o if ops_g[k] != ops_o[k]}
print(f"  op counts differing: {len(diff)}", flush=True)
for k, (g, o) in diff.items():
    print(f"    {k}: device {g} oracle {o} (rel {abs(g - o) / max(g, o):.2e})", flush=True)
ys, xs = np.nonzero(flip)
rows_abs = b + ys * s
np.savez(f"gpurun_out/flips_{cfg}.npz", y=rows_abs, x=xs, dev=acc_p[ys, xs], orc=acc_o[ys, xs],
         rows=np.array(rows), ops_dev=np.array([ops_g[k] for k in rt.OP_NAMES]),
         ops_orc=np.array([ops_o[k] for k in rt.OP_NAMES]))
for yy, xx in list(zip(rows_abs, xs))[:20]:
    k = (yy - b) // s
    print(f"    pixel ({xx},{yy}) dev {acc_p[k, xx]} orc {acc_o[k, xx]} "
          f"|d|/spp {davg[k, xx].max():.3e}", flush=True)
