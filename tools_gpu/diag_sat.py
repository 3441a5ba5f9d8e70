"""Diagnostics for test_saturating_texture_coordinates: the device vs the f64 oracle for noise and
checker scales that do and do not saturate the i32 casts (profiles/r06i_diag_sat.log was taken
with round 6's A/B switch for the C++ range checks, since removed, as the second process)."""
import os
import subprocess
import sys

CHILD = r"""
import sys, os
sys.path.insert(0, "surely-raytracing_amd"); sys.path.insert(0, "tests")
import numpy as np, surely_rt as rt, oracle_lib as O
def scene(noise, chk_scale):
    sc = rt.Scene(12)
    chk = sc.lambertian(tex=sc.checker_from_color(chk_scale, (0.9, 0.1, 0.1), (0.1, 0.9, 0.1)))
    marble = sc.lambertian(tex=sc.noise_texture(noise))
    light = sc.diffuse_light((6, 6, 6))
    world = sc.hittable_list(sc.quad((1, -1, 1), (4, 0, 0), (0, 0, 4), chk),
                             sc.quad((-1, -1, 1), (0, 3, 0), (0, 0, 4), chk),
                             sc.sphere((3, 1, 3), 0.8, marble),
                             sc.quad((1, 4, 1), (2, 0, 0), (0, 0, 2), light))
    lights = sc.hittable_list(sc.quad((1, 4, 1), (2, 0, 0), (0, 0, 2), light))
    blob = sc.serialize(world, lights)
    cam = rt.camera_new(1.0, 64, 16, 20, 50, (6, 3, -3), (2, 0, 3), (0, 1, 0), 0, 0, (0.1, 0.1, 0.1))
    return blob, cam
for noise, cs in ((1e10, 1e-10), (4.0, 1e-10), (1e10, 0.5), (4.0, 0.5)):
    blob, cam = scene(noise, cs)
    ds = rt.DeviceScene(blob)
    acc, st = ds.render(cam, rt.make_opts(cam, seed=1, flags=rt.RT_FLAG_OVERWRITE))
    ds.close()
    ref, ops = O.render(blob, cam, rt.make_opts(cam, seed=1), precision=64)
    d = np.abs(acc.astype(np.float64) - ref) / 16
    fin = np.isfinite(d)
    print(f"noise {noise:g} checker {cs:g}: max|d| {d[fin].max():.3e} mean {d[fin].mean():.3e} "
          f"ops equal {st.op_counts() == ops} nan {int((~fin).sum())}", flush=True)
"""
for opts in ("",):
    out = subprocess.run([sys.executable, "-c", CHILD], env=dict(os.environ, RT_JIT_OPTS=opts),
                         capture_output=True, text=True, timeout=300)
    print(f"== RT_JIT_OPTS='{opts}'\n{out.stdout}{out.stderr[-500:] if out.returncode else ''}", flush=True)
