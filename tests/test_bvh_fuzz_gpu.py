"""Seeded dense-BVH scenes against the oracle: the compact-tree walk from LDS (cbvh_walk_t, both
the tmin >= 0 form and a ConstantMedium boundary's tmin = -inf form), its stack entries' bf16
entry times and pop-time culling, the per-axis blocked nodes and the two-smallest tie flag, on
trees far larger and more irregular than the benchmark scenes' (hittable.rs:147-236 BvhNode,
rt_layout.h CBVH).

Each scene holds a top-level BVH of a few hundred items -- spheres of widely varying radius,
exact duplicates (the same sphere twice with different materials: ties at equal t, which the
reference resolves by its walk order), moving spheres, rows of boxes whose faces touch (ties
between coplanar faces), thin quads -- plus a RotateY + Translate instance of a second BVH and a
ConstantMedium whose boundary is a BVH of a box's six quads. Checks, as _compare: the product,
op-counting and interpreter kernels bit-identical, per pixel within TOL of the f64 oracle; and the
LDS walk, the global per-octant streams and the reference-order walk give the same image bit for
bit.

Op counts: every path decision (hits, misses, scatters, light and volume draws, ...) identical;
the box-culling counters (AABB tests and the primitive tests inside culled boxes) within
CULL_RTOL. Boxes of one BVH that share a plane -- the faces of one box (the fog's boundary
tree), boxes that touch -- put Aabb::hit (object.rs:340-370) at an exact tie: a sibling's slab
entry on the plane of the face just hit, (q - o) * (1 / d) against the quad's (D - n.o) / (n.d),
the same number in exact arithmetic. The reference decides it by the last bit of its two
roundings; the device's reciprocals are within an ulp, so it culls some of those
boxes the other way. A box culled at such a tie holds no candidate below the closest t, so
images do not move (tools_gpu/diag_vol_bvh.py isolates it: a boundary of four box faces as a
BVH of two nodes, op counts differ, images identical; profiles/r04v_vol_bvh_diag.log)."""
import numpy as np
import pytest

import surely_rt as rt
import oracle_lib as O
from test_gpu_parity import _compare, _render_env

pytestmark = pytest.mark.gpu
CULL_OPS = ("aabb_tests", "quad_tests", "quad_plane", "quad_interval", "sphere_tests",
            "sphere_roots")
CULL_RTOL = 1e-2


def dense_bvh_scene(seed, parts="sdmqbrif"):
    """parts: s spheres, d duplicates, m moving spheres, q quads, b boxes, r the touching row,
    i the instance, f the fog (a diagnostic can drop some)."""
    rnd = np.random.default_rng(1000 + seed)
    sc = rt.Scene(seed)
    u = lambda a, b: float(rnd.uniform(a, b))  # noqa: E731
    col = lambda: tuple(float(x) for x in rnd.uniform(0.1, 0.9, 3))  # noqa: E731
    light = sc.diffuse_light((10.0, 10.0, 10.0))
    mats = [sc.lambertian(col()), sc.lambertian(col()), sc.metal(col(), u(0.0, 0.4)),
            sc.dielectric(u(1.3, 1.7)), sc.lambertian(tex=sc.checker_from_color(0.7, col(), col()))]
    pick = lambda: mats[int(rnd.integers(0, len(mats)))]  # noqa: E731
    items = []
    for _ in range(int(rnd.integers(150, 260))):
        c = (u(0, 10), u(0.2, 6), u(0, 10))
        kind = rnd.uniform()
        if kind < 0.55:
            r = float(np.exp(rnd.uniform(np.log(0.02), np.log(0.9))))
            m0, m1, dup = pick(), pick(), rnd.uniform() < 0.15
            if "s" in parts:
                items.append(sc.sphere(c, r, m0))
            if dup and "d" in parts:  # an exact duplicate: equal t, the walk order decides
                items.append(sc.sphere(c, r, m1))
        elif kind < 0.7:
            c1, r, m = (c[0] + u(-0.3, 0.3), c[1], c[2]), u(0.05, 0.5), pick()
            if "m" in parts:
                items.append(sc.sphere_moving(c, c1, r, m))
        elif kind < 0.85:
            e0, e1, m = (u(0.2, 1.5), 0, 0), (0, u(-0.3, 0.3), u(0.2, 1.5)), pick()
            if "q" in parts:
                items.append(sc.quad(c, e0, e1, m))
        else:
            s = u(0.2, 1.0)
            b1, m = (c[0] + s, c[1] + u(0.1, 1.0), c[2] + s), pick()
            if "b" in parts:
                items.append(sc.make_box(c, b1, m))
    # a row of boxes whose faces touch (shared planes x = const: coplanar-face ties)
    h = [u(0.3, 1.5) for _ in range(12)]
    for k in range(12 if "r" in parts else 0):
        items.append(sc.make_box((k * 0.8, 0, 10.5), ((k + 1) * 0.8, h[k], 11.3), mats[0]))
    world = [sc.create_bvh(sc.hittable_list(*items))]
    # an instance of a second tree
    inner = [sc.sphere((u(-1.5, 1.5), u(0, 3), u(-1.5, 1.5)), u(0.05, 0.4), pick()) for _ in range(60)]
    inst = sc.translate(sc.rotate_y(sc.create_bvh(sc.hittable_list(*inner)), u(-60, 60)),
                        (u(2, 8), 0.0, u(-3, -1)))
    if "i" in parts:
        world.append(inst)
    # a ConstantMedium whose boundary is a BVH (rays start inside it: tmin = -inf walks)
    fog_box = sc.create_bvh(sc.make_box((u(1, 3), 0.5, u(1, 3)), (u(5, 7), u(2, 4), u(5, 7)), mats[0]))
    fog = sc.constant_medium(fog_box, u(0.05, 0.4), col())
    if "f" in parts:
        world.append(fog)
    world.append(sc.quad((-20, 0, -20), (40, 0, 0), (0, 0, 40), mats[0]))
    lamp = sc.quad((3, 12, 3), (4, 0, 0), (0, 0, 4), light)
    world.append(lamp)
    lights = sc.hittable_list(sc.quad((3, 12, 3), (4, 0, 0), (0, 0, 4), light))
    blob = sc.serialize(sc.hittable_list(*world), lights)
    cam = rt.camera_new(1.0, 64, 16, 12, 50, (5, 7, -12), (5, 2, 5), (0, 1, 0), 0, 0,
                        (0.4, 0.5, 0.7) if seed % 2 else (0.0, 0.0, 0.0))
    return blob, cam


@pytest.mark.parametrize("seed", range(1, 7))
def test_dense_bvh_scene_parity(gpu_available, seed):
    blob, cam = dense_bvh_scene(seed)
    assert rt.layout_stats(blob)["compact_bvhs"] >= 2
    acc_g, acc_o, st = _compare(blob, cam, check_ops=False)
    assert np.isfinite(acc_g).any() and acc_g[np.isfinite(acc_g)].mean() > 0.0
    _, ops_o = O.render(blob, cam, rt.make_opts(cam, seed=1, flags=rt.RT_FLAG_OVERWRITE),
                        precision=64)
    ops_g = st.op_counts()
    path = {k: (ops_g[k], ops_o[k]) for k in ops_o if k not in CULL_OPS and ops_g[k] != ops_o[k]}
    assert not path, path
    cull = {k: (ops_g[k], ops_o[k]) for k in CULL_OPS
            if abs(ops_g[k] - ops_o[k]) > CULL_RTOL * max(ops_g[k], ops_o[k])}
    assert not cull, cull
    lds = _render_env(blob, cam, {})
    streams = _render_env(blob, cam, {"RT_NO_CBVH_LDS": 1})
    ref = _render_env(blob, cam, {}, flags=rt.RT_FLAG_OVERWRITE | rt.RT_FLAG_REFERENCE_BVH)
    assert np.array_equal(lds, streams, equal_nan=True)
    assert np.array_equal(lds, ref, equal_nan=True)


def column_grid_scene(seed, parts="gsimdc"):
    """A BVH of leaves on a regular x/z lattice (final_scene's ground, book2 main.rs, is the
    benchmark case): boxes touching their neighbours
    (shared side planes), heights drawn from a few values (coplanar tops across cells), spheres
    inside cells, empty cells (cell sizes, origins and most heights dyadic, so that shared
    planes are one double), and the same kind of grid again inside a RotateY + Translate
    instance. The camera looks along the grid at a grazing angle, so walks cross many columns, and
    scattered rays start on the box tops and sides. parts (a diagnostic can drop some): g the main
    grid, s its spheres, i the instance; m, d, c: metal, dielectric, checker-textured items
    (without them, the two plain Lambertians)."""
    rnd = np.random.default_rng(2000 + seed)
    sc = rt.Scene(seed)
    u = lambda a, b: float(rnd.uniform(a, b))  # noqa: E731
    col = lambda: tuple(float(x) for x in rnd.uniform(0.1, 0.9, 3))  # noqa: E731
    light = sc.diffuse_light((12.0, 12.0, 12.0))
    # (the checker's period is not a multiple of the lattice's, for the same reason as below)
    mats = [sc.lambertian(col()), sc.lambertian(col()), sc.metal(col(), u(0.0, 0.3)),
            sc.dielectric(1.5), sc.lambertian(tex=sc.checker_from_color(0.2718281828, col(), col()))]
    allowed = [0, 1] + [k for k, p in ((2, "m"), (3, "d"), (4, "c")) if p in parts]
    pick = lambda: mats[allowed[int(rnd.integers(0, 5)) % len(allowed)]]  # noqa: E731

    def grid(nx, nz, w, x0, z0, y0=0.0625):
        heights = [float(rnd.integers(3, 17)) / 8 for _ in range(3)]  # dyadic: exact planes
        items = []
        for i in range(nx):
            for j in range(nz):
                a, b = x0 + i * w, z0 + j * w
                corner = (i, j) in ((0, 0), (nx - 1, nz - 1))
                kind = 0.0 if corner else rnd.uniform()
                if kind < 0.6 or i == j:  # a box filling the cell (every row and column has one)
                    h = heights[int(rnd.integers(0, 3))] if rnd.uniform() < 0.7 else u(0.1, 2.5)
                    items.append(sc.make_box((a, y0, b), (a + w, h, b + w), pick()))
                elif kind < 0.8:
                    r = u(0.1, 0.45) * w
                    c = (a + 0.5 * w, y0 + r + u(0.0, 1.0), b + 0.5 * w)
                    if "s" in parts:
                        items.append(sc.sphere(c, r, pick()))
        return sc.create_bvh(sc.hittable_list(*items))

    # dyadic cell sizes and origins: neighbours' shared planes are the same double, as in
    # final_scene's integer lattice; no face on a coordinate plane (x, y or z = 0 is a boundary
    # of the checker, floor(p / scale), where the sign of the hit point's last bit decides)
    nx, nz = int(rnd.integers(5, 13)), int(rnd.integers(5, 13))
    w = float(rnd.integers(4, 10)) / 8
    main = grid(nx, nz, w, (0.5 - np.floor(4 * nx * w)) / 8, (0.5 - np.floor(4 * nz * w)) / 8)
    inst = sc.translate(sc.rotate_y(grid(6, 5, 0.375, -1.0625, -0.9375), u(-50, 50)),
                        (u(-2, 2), 2.6, u(-2, 2)))
    world = ([main] if "g" in parts else []) + ([inst] if "i" in parts else [])
    world.append(sc.quad((-30, -0.01, -30), (60, 0, 0), (0, 0, 60), mats[0]))
    world.append(sc.quad((-1, 9, -1), (2, 0, 0), (0, 0, 2), light))
    lights = sc.hittable_list(sc.quad((-1, 9, -1), (2, 0, 0), (0, 0, 2), light))
    blob = sc.serialize(sc.hittable_list(*world), lights)
    look_from = (-0.6 * nx * w, u(1.0, 3.0), -0.6 * nz * w)
    cam = rt.camera_new(1.0, 64, 16, 12, 60, look_from, (0.3 * nx * w, 0.5, 0.3 * nz * w),
                        (0, 1, 0), 0, 0, (0.5, 0.6, 0.8) if seed % 2 else (0.0, 0.0, 0.0))
    return blob, cam


@pytest.mark.parametrize("seed", range(1, 7))
def test_lattice_bvh_scene_parity(gpu_available, seed):
    """BVHs of leaves on a regular x/z lattice (shared side planes, coplanar tops: the ties the
    ordered walks must hand to the reference order): the compact-tree walk (the default) bit for
    bit against the global streams, the reference-order walk (RT_FLAG_REFERENCE_BVH; the
    op-counting build always walks it) and the interpreter kernel, and against the f64 oracle as
    the dense scenes (_compare: per pixel within TOL, every path decision's op count identical,
    the box-culling counters within CULL_RTOL). (Round 5's column-grid walk of these scenes was
    measured no faster than the tree and removed in round 6)"""
    blob, cam = column_grid_scene(seed)
    acc_g, _, st = _compare(blob, cam, check_ops=False)
    assert np.isfinite(acc_g).any() and acc_g[np.isfinite(acc_g)].mean() > 0.0
    _, ops_o = O.render(blob, cam, rt.make_opts(cam, seed=1, flags=rt.RT_FLAG_OVERWRITE),
                        precision=64)
    ops_g = st.op_counts()
    path = {k: (ops_g[k], ops_o[k]) for k in ops_o if k not in CULL_OPS and ops_g[k] != ops_o[k]}
    assert not path, path
    g = _render_env(blob, cam, {})
    for env, flags in (({"RT_NO_CBVH_LDS": 1}, None),
                       ({}, rt.RT_FLAG_OVERWRITE | rt.RT_FLAG_INTERPRETER),
                       ({}, rt.RT_FLAG_OVERWRITE | rt.RT_FLAG_REFERENCE_BVH)):
        other = _render_env(blob, cam, env, **({"flags": flags} if flags else {}))
        assert np.array_equal(g, other, equal_nan=True), (env, flags)
