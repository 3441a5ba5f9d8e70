"""ConstantMedium with a BVH boundary: device op counts vs the oracle's on minimal scenes
(boundary = a box's quad list, a BVH of its six quads, a BVH of 2 / 3 / 4 quads, a BVH of one
sphere and one box). Usage: python tools_gpu/diag_vol_bvh.py"""
import sys

sys.path.insert(0, "tests")
sys.path.insert(0, "surely-raytracing_amd")
import numpy as np  # noqa: E402
import oracle_lib as O  # noqa: E402
import surely_rt as rt  # noqa: E402
from test_gpu_parity import _frame_report, _gpu  # noqa: E402


def scene(kind):
    sc = rt.Scene(5)
    white = sc.lambertian((0.7, 0.7, 0.7))
    light = sc.diffuse_light((8.0, 8.0, 8.0))
    a, b = (1.0, 0.5, 1.0), (4.0, 2.5, 4.0)
    if kind == "list":
        bd = sc.make_box(a, b, white)
    elif kind == "bvh6":
        bd = sc.create_bvh(sc.make_box(a, b, white))
    else:
        faces = [sc.quad((1, 0.5, 1), (3, 0, 0), (0, 2, 0), white),      # z = 1
                 sc.quad((1, 0.5, 4), (3, 0, 0), (0, 2, 0), white),      # z = 4
                 sc.quad((1, 0.5, 1), (0, 2, 0), (0, 0, 3), white),      # x = 1
                 sc.quad((4, 0.5, 1), (0, 2, 0), (0, 0, 3), white)]      # x = 4
        n = int(kind[-1])
        bd = sc.create_bvh(sc.hittable_list(*faces[:n]))
    world = sc.hittable_list(sc.constant_medium(bd, 0.3, (0.8, 0.8, 0.8)),
                             sc.quad((-10, 0, -10), (20, 0, 0), (0, 0, 20), white),
                             sc.quad((1, 6, 1), (2, 0, 0), (0, 0, 2), light))
    lights = sc.hittable_list(sc.quad((1, 6, 1), (2, 0, 0), (0, 0, 2), light))
    blob = sc.serialize(world, lights)
    cam = rt.camera_new(1.0, 32, 16, 8, 50, (2.5, 3, -6), (2.5, 1.5, 2.5), (0, 1, 0), 0, 0,
                        (0.3, 0.4, 0.5))
    return blob, cam


for kind in ["list", "bvh6", "bvh2", "bvh3", "bvh4"]:
    blob, cam = scene(kind)
    acc_g, st = _gpu(blob, cam, seed=1, flags=rt.RT_FLAG_OVERWRITE | rt.RT_FLAG_COUNT_OPS)
    acc_i, st_i = _gpu(blob, cam, seed=1, flags=rt.RT_FLAG_OVERWRITE | rt.RT_FLAG_COUNT_OPS |
                       rt.RT_FLAG_INTERPRETER)
    acc_o, ops_o = O.render(blob, cam, rt.make_opts(cam, seed=1, flags=rt.RT_FLAG_OVERWRITE),
                            precision=64)
    _frame_report(kind, acc_g, acc_o, cam.samples_per_pixel)
    ops_g, ops_i = st.op_counts(), st_i.op_counts()
    print("  ops diff:", {k: (ops_g[k], ops_o[k]) for k in ops_o if ops_g[k] != ops_o[k]},
          " interp vs count:", {k: ops_i[k] - ops_g[k] for k in ops_g if ops_i[k] != ops_g[k]},
          flush=True)
