"""GPU (gfx950) vs CPU oracle parity, through the C ABI (librtmi355x.so).

Tolerance (north star: "per-pixel RGB within 1e-4 of the seeded CPU output"): the per-pixel
linear average (raw sum / spp) of the device must be within 1e-4 of the f64 oracle's for every
pixel and channel. Both compute the path in f64 with the same per-sample RNG stream; the device
uses fma and ocml while the oracle uses the reference's plain operation order and libm, so
path decisions agree (identical op counts are asserted) and sums differ only by rounding.
"""
import os

import numpy as np
import pytest

import oracle_lib as O
import surely_rt as rt

pytestmark = pytest.mark.gpu
TOL = 1e-4
C4_OPS_RTOL = 1e-4


def _gpu(blob, cam, **kw):
    ds = rt.DeviceScene(blob)
    try:
        opts = rt.make_opts(cam, **kw)
        acc, st = ds.render(cam, opts)
    finally:
        ds.close()
    return acc, st


def _compare(blob, cam, seed=1, flags=rt.RT_FLAG_OVERWRITE, check_ops=True, ops_rtol=0.0, **kw):
    acc_g, st = _gpu(blob, cam, seed=seed, flags=flags | rt.RT_FLAG_COUNT_OPS, **kw)
    # the product kernels (no op counters) take shortcuts the counting build does not: span-1
    # BVH leaves are tested once (RTL_DUP), ConstantMedium boundaries are queried in one walk
    # (volume_two_hits). They must reproduce the counting build's image bit for bit.
    acc_p, _ = _gpu(blob, cam, seed=seed, flags=flags, **kw)
    assert np.array_equal(acc_p, acc_g, equal_nan=True), \
        f"product vs counting kernel: max |d| {np.nanmax(np.abs(acc_p - acc_g))}"
    # product renders run the scene-specialised kernel (rt_jit.cpp); the interpreter walker's
    # product kernel must give the same image bit for bit
    acc_i, _ = _gpu(blob, cam, seed=seed, flags=flags | rt.RT_FLAG_INTERPRETER, **kw)
    assert np.array_equal(acc_p, acc_i, equal_nan=True), \
        f"scene-specialised vs interpreter kernel: max |d| {np.nanmax(np.abs(acc_p - acc_i))}"
    opts = rt.make_opts(cam, seed=seed, flags=flags, **kw)
    acc_o, ops_o = O.render(blob, cam, opts, precision=64)
    _check_values(acc_g, acc_o, cam, kw.get("sj_count", 0))
    if check_ops:
        ops_g = st.op_counts()
        bad = {k: (ops_g[k], ops_o[k]) for k in ops_o
               if abs(ops_g[k] - ops_o[k]) > ops_rtol * max(ops_g[k], ops_o[k])}
        assert not bad, bad
    return acc_g, acc_o, st


def _check_values(acc_g, acc_o, cam, sj_count=0):
    """Per pixel and channel: the same NaN / +-inf positions as the oracle (the reference's
    special values, render.rs:287-292), and finite values within TOL of the oracle's per-sample
    average."""
    spp = cam.sqrt_spp * (sj_count or cam.sqrt_spp)
    assert np.array_equal(np.isnan(acc_g), np.isnan(acc_o)), \
        f"NaN masks differ at {np.argwhere(np.isnan(acc_g) != np.isnan(acc_o))[:8].tolist()}"
    assert np.array_equal(np.isposinf(acc_g), np.isposinf(acc_o)), "+inf masks differ"
    assert np.array_equal(np.isneginf(acc_g), np.isneginf(acc_o)), "-inf masks differ"
    fin = np.isfinite(acc_g)
    diff = np.abs(acc_g[fin].astype(np.float64) - acc_o[fin].astype(np.float64)) / spp
    assert diff.size == 0 or diff.max() <= TOL, f"max |d| = {diff.max()}"


def test_device_present(gpu_available):
    assert gpu_available >= 1


def test_cornell_c1_parity(gpu_available):
    """BASELINE config 1: Cornell box with mixture-PDF light sampling, 200x200, 16 spp."""
    blob, cam = rt.preset_blob("cornell_box", width=200, spp=16)
    acc_g, acc_o, st = _compare(blob, cam)
    assert st.samples == 200 * 200 * 16
    assert acc_g.mean() > 0.05


@pytest.mark.parametrize("name,kw", [
    ("cornell_box", dict(width=61, spp=9)),
    ("final_scene", dict(width=45, spp=4, depth=12, aspect=16.0 / 9.0)),
])
def test_ragged_tiles_parity(gpu_available, name, kw):
    """Image widths and heights that are not multiples of the 8x8 pool tile: the right-edge
    tiles decode their pixels by division (the full-width tiles by shifts) and the bottom tiles
    hold fewer rows; every pixel is still rendered once, against the oracle."""
    blob, cam = rt.preset_blob(name, **kw)
    assert cam.image_width % 8 != 0
    acc_g, acc_o, st = _compare(blob, cam)
    assert st.samples == cam.image_width * cam.image_height * cam.samples_per_pixel


def test_max_depth_zero_renders_black(gpu_available):
    """ray_color's depth guard at depth 0 (render.rs:260-262): every sample returns black
    without a world query (the camera-ray block ends it; op counts as the oracle's)."""
    blob, cam = rt.preset_blob("cornell_box", width=24, spp=4)
    cam.max_depth = 0
    acc_g, acc_o, st = _compare(blob, cam)
    assert not acc_g.any() and not acc_o.any()
    ops = st.op_counts()
    assert ops["world_queries"] == 0 and ops["depth_cutoff"] == ops["samples"] == 24 * 24 * 4


@pytest.mark.parametrize("name,variant,width,spp,depth", [
    ("cornell_box", "mixed_pdf", 96, 16, 50),
    ("cornell_smoke", "", 96, 9, 10),
    ("final_scene", "", 96, 4, 12),
    ("quads", "", 64, 16, 50),
    ("simple_light", "", 96, 16, 50),
    ("two_spheres", "", 96, 9, 50),
    ("two_perlin_spheres", "", 96, 9, 50),
    ("random_balls", "", 96, 4, 50),
    ("three_spheres", "", 96, 9, 50),
    ("earth", "", 64, 9, 50),
])
def test_scene_parity(gpu_available, name, variant, width, spp, depth):
    blob, cam = rt.preset_blob(name, variant=variant, width=width, spp=spp, depth=depth)
    _compare(blob, cam)


def test_image_texture_parity(gpu_available):
    """ImageTexture with a synthetic RGB8 image (earthmap.jpg is absent upstream) on a sphere
    (get_sphere_uv, object.rs:114-120) and a quad (u, v = planar coords)."""
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, size=(37, 53, 3), dtype=np.uint8)
    sc = rt.Scene(7)
    tex = sc.image_texture(img)
    mat = sc.lambertian(tex=tex)
    light = sc.diffuse_light((4, 4, 4))
    world = sc.hittable_list(sc.sphere((0, 0, 0), 1.5, mat),
                             sc.quad((-3, -2, -3), (6, 0, 0), (0, 0, 6), mat),
                             sc.quad((-1, 3, -1), (2, 0, 0), (0, 0, 2), light))
    lights = sc.quad((-1, 3, -1), (2, 0, 0), (0, 0, 2), light)
    blob = sc.serialize(world, lights)
    cam = rt.camera_new(1.0, 64, 16, 20, 40, (0, 2, 8), (0, 0, 0), (0, 1, 0), 0, 0, (0.2, 0.3, 0.4))
    _compare(blob, cam)


def test_saturating_texture_coordinates(gpu_available):
    """Rust's saturating `as i32` (texture.rs:71-81 CheckerTexture; the same conversion takes the
    Perlin lattice cell, perlin.rs:30-54) on coordinates far outside the i32 range: a checker of
    scale 1e-10 (floor(1e10 p) saturates to i32::MAX / MIN, whose parity picks the colour) on
    quads whose every coordinate has |p| >= 1, beside a noise-textured sphere. The device issues
    v_cvt_i32_f64 directly (rt_kernel.h f2i_sat); the oracle restates the Rust cast. (A noise
    scale that saturates the lattice, ~1e9 at these coordinates, makes the turbulence depend on
    the hit point's last bits times 1e9 -- 3e-3 between the device and the oracle,
    tools_gpu/diag_sat.py -- so the noise keeps an ordinary scale.)"""
    sc = rt.Scene(12)
    chk = sc.lambertian(tex=sc.checker_from_color(1e-10, (0.9, 0.1, 0.1), (0.1, 0.9, 0.1)))
    marble = sc.lambertian(tex=sc.noise_texture(4.0))
    light = sc.diffuse_light((6, 6, 6))
    world = sc.hittable_list(sc.quad((1, -1, 1), (4, 0, 0), (0, 0, 4), chk),
                             sc.quad((-1, -1, 1), (0, 3, 0), (0, 0, 4), chk),
                             sc.sphere((3, 1, 3), 0.8, marble),
                             sc.quad((1, 4, 1), (2, 0, 0), (0, 0, 2), light))
    lights = sc.hittable_list(sc.quad((1, 4, 1), (2, 0, 0), (0, 0, 2), light))
    blob = sc.serialize(world, lights)
    cam = rt.camera_new(1.0, 64, 16, 20, 50, (6, 3, -3), (2, 0, 3), (0, 1, 0), 0, 0, (0.1, 0.1, 0.1))
    acc_g, _, st = _compare(blob, cam)
    assert st.op_counts()["noise_evals"] > 0


def test_checker_volume_transform_mix(gpu_available):
    """Nested Translate(RotateY(BVH)) + ConstantMedium over a rotated box + checker + metal."""
    sc = rt.Scene(11)
    chk = sc.lambertian(tex=sc.checker_from_color(0.5, (0.9, 0.1, 0.1), (0.1, 0.9, 0.1)))
    white = sc.lambertian((0.7, 0.7, 0.7))
    metal = sc.metal((0.8, 0.8, 0.9), 0.3)
    light = sc.diffuse_light((6, 6, 6))
    balls = sc.hittable_list()
    for k in range(40):
        c = (sc.random_range(-2, 2), sc.random_range(0, 2), sc.random_range(-2, 2))
        sc.add(balls, sc.sphere(c, 0.25, metal if k % 3 == 0 else white))
    inst = sc.translate(sc.rotate_y(sc.create_bvh(balls), 30), (0.5, 0.2, -0.5))
    box = sc.translate(sc.rotate_y(sc.make_box((0, 0, 0), (1, 2, 1), white), -20), (-2, 0, 1))
    fog = sc.constant_medium(box, 0.8, (0.9, 0.9, 0.9))
    lq = sc.quad((-1, 4, -1), (2, 0, 0), (0, 0, 2), light)
    # ground at y=-0.3: a checker evaluated ON its own discontinuity plane (y = 0) depends on
    # the last-bit rounding of p.y (fma vs plain), in the reference as well (texture.rs:71-81)
    world = sc.hittable_list(sc.quad((-5, -0.3, -5), (10, 0, 0), (0, 0, 10), chk), inst, fog, lq)
    lights = sc.hittable_list(sc.quad((-1, 4, -1), (2, 0, 0), (0, 0, 2), light))
    blob = sc.serialize(world, lights)
    cam = rt.camera_new(1.0, 80, 16, 20, 45, (0, 3, 8), (0, 1, 0), (0, 1, 0), 0, 0, (0, 0, 0))
    _compare(blob, cam)


def test_volume_boundary_one_walk(gpu_available):
    """ConstantMedium boundaries the flattener marks for the one-walk query: a sphere, and a list
    of axis-aligned quads (a box with its top face duplicated, so rays through that face have two
    equal candidates below rec1.t + 1e-4 and take the interpreter fallback for rec2)."""
    sc = rt.Scene(5)
    white = sc.lambertian((0.73, 0.73, 0.73))
    light = sc.diffuse_light((8, 8, 8))
    a, b = (-1.0, 0.0, -1.0), (1.0, 1.5, 1.0)
    faces = [sc.quad((a[0], a[1], b[2]), (2, 0, 0), (0, 1.5, 0), white),
             sc.quad((b[0], a[1], b[2]), (0, 0, -2), (0, 1.5, 0), white),
             sc.quad((b[0], a[1], a[2]), (-2, 0, 0), (0, 1.5, 0), white),
             sc.quad((a[0], a[1], a[2]), (0, 0, 2), (0, 1.5, 0), white),
             sc.quad((a[0], b[1], b[2]), (2, 0, 0), (0, 0, -2), white),
             sc.quad((a[0], b[1], b[2]), (2, 0, 0), (0, 0, -2), white),  # duplicate top
             sc.quad((a[0], a[1], a[2]), (2, 0, 0), (0, 0, 2), white)]
    box_fog = sc.constant_medium(sc.rotate_y(sc.hittable_list(*faces), 25), 0.9, (0.9, 0.8, 0.7))
    ball_fog = sc.constant_medium(sc.sphere((2.0, 0.8, 0.5), 0.8, white), 1.5, (0.3, 0.5, 0.9))
    floor = sc.quad((-6, -0.01, -6), (12, 0, 0), (0, 0, 12), white)
    lq = sc.quad((-1, 4, -1), (2, 0, 0), (0, 0, 2), light)
    world = sc.hittable_list(floor, box_fog, ball_fog, lq)
    lights = sc.hittable_list(sc.quad((-1, 4, -1), (2, 0, 0), (0, 0, 2), light))
    blob = sc.serialize(world, lights)
    cam = rt.camera_new(1.0, 72, 16, 12, 40, (0.5, 2.5, 7), (0.3, 0.8, 0), (0, 1, 0), 0, 0, (0.05, 0.05, 0.05))
    acc_g, _, st = _compare(blob, cam)
    assert st.op_counts()["volume_draws"] > 0


def test_bvh_over_instances_volumes_and_general_quads(gpu_available):
    """A BvhNode tree whose leaves are instanced boxes (Translate/RotateY inside the per-lane
    walker: frame changes, EXIT links, 1/d recomputed), a ConstantMedium (never elided as a
    duplicate: it draws), non-axis-aligned quads (the general quad test), moving spheres and
    spheres; 5 and 7 leaves give span-1 nodes, i.e. DUP records over each kind of subtree."""
    sc = rt.Scene(21)
    white = sc.lambertian((0.73, 0.73, 0.73))
    red = sc.lambertian((0.65, 0.05, 0.05))
    glass = sc.dielectric(1.5)
    light = sc.diffuse_light((10, 10, 10))
    items = sc.hittable_list()
    for k in range(7):
        x = -3.0 + k
        if k % 3 == 0:
            sc.add(items, sc.translate(sc.rotate_y(sc.make_box((0, 0, 0), (0.6, 0.9, 0.6), red),
                                                   15 * k), (x, 0, -0.3)))
        elif k % 3 == 1:
            sc.add(items, sc.quad((x, 0.1, 0.5), (0.5, 0.4, 0.0), (0.0, 0.3, 0.6), white))
        else:
            sc.add(items, sc.sphere_moving((x, 0.4, 0), (x, 0.6, 0.1), 0.3, glass))
    sc.add(items, sc.constant_medium(sc.sphere((0.5, 1.5, 0.2), 0.5, white), 2.0, (0.8, 0.8, 0.9)))
    sc.add(items, sc.sphere((1.5, 1.4, -0.5), 0.35, white))
    inner = sc.create_bvh(items)
    world = sc.hittable_list(sc.quad((-6, -0.01, -6), (12, 0, 0), (0, 0, 12), white),
                             sc.translate(sc.rotate_y(inner, -10), (0.2, 0, 0)),
                             sc.quad((-1, 4, -1), (2, 0, 0), (0, 0, 2), light))
    lights = sc.hittable_list(sc.quad((-1, 4, -1), (2, 0, 0), (0, 0, 2), light))
    blob = sc.serialize(world, lights)
    st = rt.layout_stats(blob)
    assert st["bvh_records"] > 0 and st["dup_records"] > 0
    cam = rt.camera_new(1.0, 72, 16, 20, 40, (0.5, 2.0, 8), (0, 0.6, 0), (0, 1, 0), 0, 0, (0.1, 0.1, 0.12))
    _compare(blob, cam)


def test_isotropic_material_outside_a_volume(gpu_available):
    """Isotropic is an ordinary Material in the reference (material.rs:229-248): a sphere may use
    it directly, with no ConstantMedium in the scene; the volume-capable kernel must run."""
    sc = rt.Scene(4)
    iso = sc.isotropic((0.8, 0.6, 0.4))
    white = sc.lambertian((0.7, 0.7, 0.7))
    light = sc.diffuse_light((8, 8, 8))
    world = sc.hittable_list(sc.sphere((0, 1, 0), 1.0, iso),
                             sc.quad((-4, 0, -4), (8, 0, 0), (0, 0, 8), white),
                             sc.quad((-1, 4, -1), (2, 0, 0), (0, 0, 2), light))
    lights = sc.hittable_list(sc.quad((-1, 4, -1), (2, 0, 0), (0, 0, 2), light))
    blob = sc.serialize(world, lights)
    cam = rt.camera_new(1.0, 48, 9, 10, 40, (0, 2, 7), (0, 1, 0), (0, 1, 0), 0, 0, (0.1, 0.1, 0.1))
    acc_g, _, st = _compare(blob, cam)
    assert st.op_counts()["isotropic"] > 0


def _jit_state(blob, cam):
    ds = rt.DeviceScene(blob)
    try:
        ds.render(cam, rt.make_opts(cam))
        return ds.jit_info()
    finally:
        ds.close()


def test_damaged_cached_code_object_is_recompiled_and_kept(gpu_available, tmp_path):
    """A cached code object that fails to load (damaged here; in the field also a transient load
    failure) is recompiled for this process only: the scene still runs its scene-specialised
    kernel, and the cache file is left in place (deleting it made every later process
    compile with another compiler). Each render runs in its own process, since the module cache
    keeps a loaded kernel for the process."""
    import subprocess
    import sys
    from pathlib import Path

    pkg = str(Path(__file__).resolve().parent.parent / "surely-raytracing_amd")
    code = ("import sys; sys.path.insert(0, %r); import surely_rt as rt; "
            "blob, cam = rt.preset_blob('cornell_box', width=16, spp=1); "
            "ds = rt.DeviceScene(blob); ds.render(cam, rt.make_opts(cam)); "
            "print('JIT', ds.jit_info()[0]); ds.close()") % pkg
    env = dict(os.environ, RT_JIT_CACHE_DIR=str(tmp_path), RT_JIT_CACHE_WRITE="1")
    env.pop("RT_JIT_OPTS", None)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=180)
    assert r.returncode == 0 and "JIT 1" in r.stdout, r.stderr[-2000:]
    files = sorted(tmp_path.glob("*.co"))
    assert len(files) == 1
    junk = b"not a code object" * 64
    files[0].write_bytes(junk)
    env.pop("RT_JIT_CACHE_WRITE")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=180)
    assert r.returncode == 0 and "JIT 1" in r.stdout, r.stderr[-2000:]
    assert "failed to load; recompiling (file kept)" in r.stderr
    assert files[0].exists() and files[0].read_bytes() == junk


def test_jit_kernel_runs_for_cornell(gpu_available):
    """BASELINE C2's and C3's scenes render through their scene-specialised kernels (compiled by
    hiprtc on the first product render), not the interpreter."""
    blob, cam = rt.preset_blob("cornell_box", width=48, spp=4)
    state, msg = _jit_state(blob, cam)
    assert state == 1, msg
    blob, cam = rt.preset_blob("cornell_smoke", width=48, spp=4)
    assert _jit_state(blob, cam)[0] == 1  # ConstantMedium records call volume_hit
    blob, cam = rt.preset_blob("final_scene", width=32, spp=1, depth=4)
    # BVH scenes: BVH subtree records call the per-lane walker from the generated top level
    state, msg = _jit_state(blob, cam)
    assert state == 1, msg


def test_jit_general_quads_moving_spheres_nested_transforms(gpu_available):
    """Every record kind the generator emits: general (non axis-aligned) quads, axis quads on
    all three axes, moving spheres (time), nested Translate/RotateY chains with EXITs back to a
    transformed parent frame, checker texture (TEX kernel), metal / dielectric / light."""
    sc = rt.Scene(5)
    chk = sc.lambertian(tex=sc.checker_from_color(0.7, (0.9, 0.2, 0.1), (0.1, 0.3, 0.9)))
    white = sc.lambertian((0.73, 0.73, 0.73))
    glass = sc.dielectric(1.5)
    metal = sc.metal((0.8, 0.7, 0.6), 0.2)
    light = sc.diffuse_light((7, 7, 7))
    inner = sc.hittable_list(sc.make_box((0, 0, 0), (0.8, 1.6, 0.8), white),
                             sc.translate(sc.rotate_y(sc.sphere_moving((0.2, 2.0, 0.2), (0.4, 2.2, 0.1), 0.3, metal), 25), (0.1, 0.0, 0.3)))
    nested = sc.translate(sc.rotate_y(inner, -18), (-1.2, 0, 0.4))
    world = sc.hittable_list(
        # ground off the checker's discontinuity plane y = 0 (see the mix test above)
        sc.quad((-4, -0.3, -4), (8, 0, 0), (0, 0, 8), chk),
        sc.quad((-3, 0.2, -2), (2.0, 1.0, 0.5), (0.3, 0.0, 1.5), white),  # general quad
        nested,
        sc.sphere((1.3, 0.7, 0.3), 0.7, glass),
        sc.sphere_moving((1.5, 0.4, -1.5), (1.5, 0.9, -1.5), 0.4, white),
        sc.quad((-1, 4, -1), (2, 0, 0), (0, 0, 2), light),
        sc.quad((3.5, 0.5, -1), (0, 2, 0), (0, 0, 2), light))
    lights = sc.hittable_list(sc.quad((-1, 4, -1), (2, 0, 0), (0, 0, 2), light),
                              sc.sphere((1.3, 0.7, 0.3), 0.7, glass))
    blob = sc.serialize(world, lights)
    cam = rt.camera_new(1.0, 72, 16, 30, 40, (0, 2.5, 8), (0, 1, 0), (0, 1, 0), 0, 0, (0.05, 0.05, 0.08))
    state, msg = _jit_state(blob, cam)
    assert state == 1, msg
    _compare(blob, cam)


def test_reference_semantics_flag(gpu_available):
    """RT_FLAG_SEMANTICS_REFERENCE: empty light list + diffuse material is an error, as the
    reference panics (hittable.rs:115-129 via render.rs:140-142)."""
    blob, cam = rt.preset_blob("quads", width=16, spp=1)
    ds = rt.DeviceScene(blob)
    with pytest.raises(rt.RtError) as e:
        ds.render(cam, rt.make_opts(cam, flags=rt.RT_FLAG_OVERWRITE | rt.RT_FLAG_SEMANTICS_REFERENCE))
    assert e.value.code == rt.RT_ERR_EMPTY_LIGHTS
    # cornell_box has lights: reference semantics render fine and match the oracle
    blob, cam = rt.preset_blob("cornell_box", width=48, spp=4)
    _compare(blob, cam, flags=rt.RT_FLAG_OVERWRITE | rt.RT_FLAG_SEMANTICS_REFERENCE)


def test_determinism_and_accumulate(gpu_available):
    blob, cam = rt.preset_blob("cornell_box", width=64, spp=9)
    ds = rt.DeviceScene(blob)
    a1, _ = ds.render(cam, rt.make_opts(cam, seed=5))
    a2, _ = ds.render(cam, rt.make_opts(cam, seed=5))
    assert np.array_equal(a1, a2)
    a3, _ = ds.render(cam, rt.make_opts(cam, seed=6))
    assert not np.array_equal(a1, a3)
    # accumulate: accum += sums (render.rs:189 adds into a pre-zeroed buffer)
    acc = np.ones_like(a1)
    ds.render(cam, rt.make_opts(cam, seed=5, flags=0), accum=acc)
    np.testing.assert_allclose(acc, a1 + 1.0, rtol=1e-6, atol=1e-5)


def test_row_tiling_invariance(gpu_available):
    """Cyclic row tiling (multi-GPU decomposition) reproduces the single-call frame bitwise."""
    from surely_rt.parallel import cyclic_rows, deinterleave, max_rows

    blob, cam = rt.preset_blob("cornell_box", width=72, spp=9)
    ds = rt.DeviceScene(blob)
    full, _ = ds.render(cam, rt.make_opts(cam, seed=9))
    H = cam.image_height
    for world in (2, 3, 8):
        m = max_rows(H, world)
        g = np.zeros((world, m, cam.image_width, 3), np.float32)
        for r in range(world):
            b, s, n = cyclic_rows(H, r, world)
            part, _ = ds.render(cam, rt.make_opts(cam, seed=9, row_begin=b, row_step=s, n_rows=n))
            g[r, :n] = part
        assert np.array_equal(deinterleave(g, H, world), full)


def test_stratum_subsets_add_up(gpu_available):
    """Rendering s_j strata in two calls adds up to the full render (sums in s_j order)."""
    blob, cam = rt.preset_blob("cornell_box", width=40, spp=16)
    ds = rt.DeviceScene(blob)
    full, _ = ds.render(cam, rt.make_opts(cam, seed=2))
    a, _ = ds.render(cam, rt.make_opts(cam, seed=2, sj_begin=0, sj_count=2))
    b, _ = ds.render(cam, rt.make_opts(cam, seed=2, sj_begin=2, sj_count=2))
    np.testing.assert_allclose(a + b, full, rtol=2e-6, atol=1e-5)


def test_book3_statistics_full_spp(gpu_available):
    """final_images/book3.png (600x600, 1000->961 spp): same mean sRGB8, the same geometric
    black-pixel count, and matching 30x30-pixel block means."""
    import json
    from pathlib import Path

    ref = json.loads((Path(__file__).parent / "golden" / "final_images_stats.json").read_text())
    for name in ("book3.png", "mixed_pdf.png"):
        m = ref[name]
        blob, cam = rt.preset_blob(m["preset"], variant=m["variant"], width=m["width"],
                                   spp=m["spp"], depth=m["depth"])
        acc, st = _gpu(blob, cam, seed=1)
        assert st.samples == 600 * 600 * 961
        rgb = rt.write_color(acc, cam.samples_per_pixel)
        mean = rgb.reshape(-1, 3).mean(0)
        assert np.abs(mean - np.array(m["mean_srgb8"])).max() < 1.0, (mean, m["mean_srgb8"])
        black = int((rgb.reshape(-1, 3).sum(1) == 0).sum())
        assert abs(black - m["black_pixels"]) <= 0.005 * m["black_pixels"], black
        blocks = rgb.astype(np.float64).reshape(20, 30, 20, 30, 3).mean(axis=(1, 3))
        d = np.abs(blocks - np.array(m["block20_srgb8"]))
        assert d.mean() < 0.6 and d.max() < 4.0, (d.mean(), d.max())


def test_book2_region_statistics(gpu_available):
    """BASELINE C4's scene (final_scene, depth 40) on the device at book2.png's own size (800x800)
    with 1024 spp for four scene-build seeds: the linear means of the five fixed objects' disks
    (motion blur, glass, fuzz-1.0 metal, subsurface ConstantMedium, Perlin turbulence; the
    regions and tolerance of tests/test_oracle_render.py::test_final_scene_matches_book2_regions)
    match the reference's final_images/book2.png."""
    import test_oracle_render as T

    means = T._book2_region_means(lambda blob, cam, opts: _gpu(blob, cam, seed=opts.seed,
                                                               row_begin=opts.row_begin,
                                                               n_rows=opts.n_rows)[0],
                                  800, 1024, (1, 2, 3, 4))
    T._check_book2(means)


def test_c2_full_size_properties(gpu_available):
    """BASELINE config 2 (800x800, 1000->961 spp): finite, deterministic, tiling-invariant."""
    from surely_rt.parallel import cyclic_rows

    blob, cam = rt.preset_blob("cornell_box", width=800, spp=1000)
    ds = rt.DeviceScene(blob)
    full, st = ds.render(cam, rt.make_opts(cam, seed=1))
    assert st.samples == 800 * 800 * 961
    assert np.isfinite(full).mean() > 0.9999
    b, s, n = cyclic_rows(800, 1, 4)
    part, _ = ds.render(cam, rt.make_opts(cam, seed=1, row_begin=b, row_step=s, n_rows=n))
    assert np.array_equal(part, full[1::4])
    rgb = rt.write_color(full, cam.samples_per_pixel)
    assert abs(rgb.reshape(-1, 3).mean(0)[0] - 79.55) < 1.5


def test_trace_kernel_timing_history(gpu_available):
    """rt_scene_trace_ms reports the rt_trace launches of the last renders (one value per render,
    chunks summed), each within the render's own device time."""
    blob, cam = rt.preset_blob("cornell_box", width=96, spp=16)
    ds = rt.DeviceScene(blob)
    sts = [ds.render(cam, rt.make_opts(cam, seed=s))[1] for s in (1, 2, 3)]
    ms = ds.trace_ms(8)
    assert len(ms) == 3
    for t, st in zip(ms, sts):
        assert 0.0 < t <= st.ms_kernel + 1e-3
    assert ds.trace_ms(2) == ms[1:]


# ---------------------------------------------------------------- BASELINE configs at their own
# settings (width, spp, depth): C2 and C3 whole frames, C4 on five bands of 40 rows each (every
# fourth row of the frame, 200 rows)
def _frame_report(cfg, acc_g, acc_o, spp):
    """max |d| of the per-sample average, pixels above TOL, and pixels whose f32 sums differ by
    more than 4 ulps (a sample that took another path, or -- since round 6 -- radiance weights
    rounded in f32; rounding moves a sum by <= 1 ulp). Also the tail of the distribution (VERDICT
    r5 item 5): the ten largest per-pixel |d| (per sample), the pixels above TOL / 2, and the
    largest |d| of a pixel's sum, i.e. the radiance difference of its flipped sample(s) -- a single
    flipped sample fails TOL only above TOL * spp (C4: 0.49). Returns (flip pixels, max |d|)."""
    fin = np.isfinite(acc_g) & np.isfinite(acc_o)
    d = np.where(fin, np.abs(acc_g.astype(np.float64) - acc_o.astype(np.float64)), 0.0)
    ulp = np.spacing(np.maximum(np.abs(acc_g), np.abs(acc_o))).astype(np.float64)
    flips = int((d > 4 * ulp).any(axis=2).sum())
    dp = d.max(axis=2)
    top = np.sort(dp.ravel())[-10:][::-1] / spp
    print(f"{cfg}: max |d| {d.max() / spp:.3e}, pixels > {TOL}: "
          f"{int((d / spp > TOL).any(axis=2).sum())}, flip pixels {flips} of "
          f"{acc_g.shape[0] * acc_g.shape[1]}")
    print(f"{cfg}: tail: ten largest per-pixel |d| " + " ".join(f"{x:.2e}" for x in top) +
          f"; pixels > {TOL / 2:g}: {int((dp / spp > TOL / 2).sum())}; largest sum |d| "
          f"(flipped-sample radiance) {d.max():.4f} against {TOL * spp:.2f} that breaks {TOL}")
    return flips, d.max() / spp


# Flip-pixel ceilings of the five C4 bands: 1.25 x the counts at the round-4 head (753, 778, 790,
# 712, 746; profiles/r04y_gputest.log), so a change that makes the device drift further from the
# oracle's paths fails here although every pixel stays within TOL.
C4_FLIP_CEILING = {2: 941, 6: 972, 10: 987, 14: 890, 18: 932}
# C2 / C3 whole frames (same paths as the oracle, identical op counts): max |d| per sample from
# the f32 radiance weights alone (<= 1e-6)
C23_TOL = 1e-6


@pytest.mark.timeout(900)
@pytest.mark.parametrize("cfg,name,kw,rows,ops_rtol", [
    ("C2", "cornell_box", dict(width=800, spp=1000), (0, 1, 800), 0.0),
    ("C3", "cornell_smoke", dict(width=800, spp=1000, depth=10), (0, 1, 800), 0.0),
] + [
    (f"C4b{b}", "final_scene", dict(width=800, spp=5000, depth=40), (b, 20, 40), C4_OPS_RTOL)
    for b in (2, 6, 10, 14, 18)
])
def test_baseline_config_frames_vs_oracle(gpu_available, cfg, name, kw, rows, ops_rtol):
    """BASELINE configs at full resolution, spp and depth (C2: 800x800 x 961 spp, depth 50; C3:
    depth 10, main.rs:589; C4: 4900 spp, depth 40, main.rs:726): HIP vs the f64 oracle on the
    WHOLE frame for C2 and C3 (615 M samples each) and, for C4, on five bands of 40 rows (band b:
    rows b, b + 20, ..., b + 780; b = 2, 6, ..., 18: every fourth row, 785 M samples), per pixel
    (values within TOL, NaN / inf positions identical) and op counts (C4: C4_OPS_RTOL)."""
    blob, cam = rt.preset_blob(name, **kw)
    assert cam.image_width == 800 and cam.image_height == 800
    b, s_, n = rows
    acc_g, acc_o, st = _compare(blob, cam, row_begin=b, row_step=s_, n_rows=n, ops_rtol=ops_rtol)
    assert st.samples == n * 800 * cam.samples_per_pixel
    flips, dmax = _frame_report(cfg, acc_g, acc_o, cam.samples_per_pixel)
    if ops_rtol == 0.0:
        # C2 / C3: every path decision identical (op counts above); only the f32 radiance weights
        # round differently from the oracle's f64 (rt_kernel.h wt): within C23_TOL per sample
        assert dmax <= C23_TOL, (cfg, dmax)
    else:
        assert flips <= C4_FLIP_CEILING[b], (cfg, flips)


@pytest.mark.timeout(300)
def test_c5_eight_way_share_is_one_launch(gpu_available):
    """BASELINE C5 (3840x2160, 10000 spp, depth 50) on 8 GPUs: one rank's cyclic share (rows
    r, r + 8, ...: 270 rows, 10.4 G samples) renders in ONE path-kernel launch (the workspace
    cap fits it) and gives the same rows as a two-chunk render of the same share."""
    blob, cam = rt.preset_blob("cornell_box", width=3840, spp=10000, aspect=16.0 / 9.0)
    ds = rt.DeviceScene(blob)
    try:
        acc, st = ds.render(cam, rt.make_opts(cam, seed=1, row_begin=3, row_step=8, n_rows=270))
        assert st.launches == 1 and st.samples == 270 * 3840 * 10000
        assert np.isfinite(acc).mean() > 0.9999 and acc.mean() > 0.0
        print(f"C5 share: {st.ms_kernel:.0f} ms, {st.samples / st.ms_kernel / 1e3:.0f} Msamples/s")
        rows = rt.make_opts(cam, seed=1, row_begin=3 + 8 * 100, row_step=8, n_rows=2)
        two = _render_env(blob, cam, {"RT_WORKSPACE_MB": 64}, row_begin=rows.row_begin,
                          row_step=8, n_rows=2)
        assert np.array_equal(two, acc[100:102])
    finally:
        ds.close()


def test_c5_camera_rows_vs_oracle(gpu_available):
    """C5 (book3 Cornell scene at 16:9, 3840x2160, 10000 spp, depth 50): the wide camera on two
    rows and a stratum subset (s_j 40..42 of 100: full-spp jitter, 300 samples per pixel)."""
    blob, cam = rt.preset_blob("cornell_box", width=3840, spp=10000, aspect=16.0 / 9.0)
    assert (cam.image_width, cam.image_height, cam.sqrt_spp) == (3840, 2160, 100)
    _compare(blob, cam, row_begin=700, row_step=700, n_rows=2, sj_begin=40, sj_count=3)


def _render_env(blob, cam, env, **kw):
    import os
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return _gpu(blob, cam, **kw)[0]
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.mark.parametrize("name,kw", [
    ("cornell_box", dict(width=96, spp=100)),
    ("final_scene", dict(width=64, spp=16, depth=40)),
])
def test_chunked_and_tail_split_renders_are_bitwise_equal(gpu_available, name, kw):
    """The stratum-row chunk loop (RT_WORKSPACE_MB too small for one launch: several launches
    carry the f64 running sums across rt_reduce calls) and the split of a launch's (tile, s_j)
    pairs into row items (the lane forms the row total), segment items (rt_reduce forms it from
    block partials) and per-sample tail items (RT_SEG_PAIRS, RT_TAIL_PAIRS) leave the image bit
    for bit unchanged. (BVH kernels keep their row totals in the dynamic LDS beside the compact
    trees: the RT_SEG_PAIRS settings render row items there too.)"""
    blob, cam = rt.preset_blob(name, **kw)
    one = _render_env(blob, cam, {})
    for env in ({"RT_WORKSPACE_MB": 1}, {"RT_TAIL_PAIRS": 0}, {"RT_TAIL_PAIRS": 1 << 30},
                {"RT_TAIL_PAIRS": 7, "RT_WORKSPACE_MB": 1},
                {"RT_SEG_PAIRS": 0, "RT_TAIL_PAIRS": 0}, {"RT_SEG_PAIRS": 0},
                {"RT_SEG_PAIRS": 5, "RT_TAIL_PAIRS": 3},
                {"RT_SEG_PAIRS": 0, "RT_TAIL_PAIRS": 0, "RT_WORKSPACE_MB": 1}):
        other = _render_env(blob, cam, env)
        assert np.array_equal(one, other, equal_nan=True), env


def test_row_items_at_frame_scale_are_bitwise_equal(gpu_available):
    """cornell_box at 800x800 and 256 spp (160 k (tile, s_j) pairs, enough for the default split
    to render row items): the default split, segment items only, and row items
    only (no band, no tail) give the same image bit for bit, and the default's workspace is one
    value per (pixel, s_j) plus the band and the tail."""
    blob, cam = rt.preset_blob("cornell_box", width=800, spp=256)
    assert cam.sqrt_spp == 16
    acc, st = _gpu(blob, cam)
    per_value = 64 * 3 * 8  # one 64-pixel slot of f64 RGB
    rows_only = 800 // 8 * 800 // 8 * cam.sqrt_spp * per_value
    assert st.launches == 1 and rows_only < st.out_bytes < 2 * rows_only, st.out_bytes
    for env in ({"RT_SEG_PAIRS": 1 << 30, "RT_TAIL_PAIRS": 4096},
                {"RT_SEG_PAIRS": 0, "RT_TAIL_PAIRS": 0}):
        other = _render_env(blob, cam, env)
        assert np.array_equal(acc, other, equal_nan=True), env


def test_bvh_row_items_at_frame_scale_are_bitwise_equal(gpu_available):
    """final_scene at 800x800 and 64 spp (80 k (tile, s_j) pairs: the default split renders row
    items, their row totals in the dynamic LDS after the compact trees and stacks; rt_layout
    plan_lds): the default split, segment items only, row items only and the BVH kernel without
    LDS row totals (RT_NO_BVH_ROWS) give the same image bit for bit, and the default's
    workspace is about one f64 value per (pixel, s_j) (render.rs:185-189)."""
    blob, cam = rt.preset_blob("final_scene", width=800, spp=64, depth=40)
    assert cam.sqrt_spp == 8
    assert rt.lds_check(blob, n_rays=0)["row_lds_off"] != 0xFFFFFFFF
    acc, st = _gpu(blob, cam)
    per_value = 64 * 3 * 8  # one 64-pixel slot of f64 RGB
    rows_only = 800 // 8 * 800 // 8 * cam.sqrt_spp * per_value
    assert st.launches == 1 and rows_only < st.out_bytes < 1.5 * rows_only, st.out_bytes
    for env in ({"RT_SEG_PAIRS": 1 << 30, "RT_TAIL_PAIRS": 4096},
                {"RT_SEG_PAIRS": 0, "RT_TAIL_PAIRS": 0}, {"RT_NO_BVH_ROWS": 1}):
        other = _render_env(blob, cam, env)
        assert np.array_equal(acc, other, equal_nan=True), env


def test_bvh_walks_from_lds_global_and_reference_order_are_bitwise_equal(gpu_available):
    """final_scene at depth 40: the compact ordered BVHs walked from LDS (cbvh_walk, the product
    default), the per-octant ordered streams walked from global memory (RT_NO_CBVH_LDS) and the
    reference tree in the reference order (RT_FLAG_REFERENCE_BVH, hittable.rs:216-236) return
    the same records, so the three images are equal bit for bit."""
    blob, cam = rt.preset_blob("final_scene", width=96, spp=16, depth=40)
    assert rt.layout_stats(blob)["compact_bvhs"] == 2
    lds = _render_env(blob, cam, {})
    streams = _render_env(blob, cam, {"RT_NO_CBVH_LDS": 1})
    ref = _render_env(blob, cam, {}, flags=rt.RT_FLAG_OVERWRITE | rt.RT_FLAG_REFERENCE_BVH)
    assert np.array_equal(lds, streams, equal_nan=True)
    assert np.array_equal(lds, ref, equal_nan=True)


def _zero_pdf_scene():
    """A floor whose light-sampled bounces have pdf_val = 0 exactly, and whose sub-paths then
    return 0. The light list holds a quad 1e-9 below the floor's plane (not in the world): a
    direction sampled towards it from the floor has |n.d| ~ 1e-9 < 1e-8, so Quad::pdf_value
    misses (object.rs:457, 492-501), the top light misses too, and the direction points
    (robustly, 1e-9 >> rounding) below the floor, so the cosine PDF and scattering_pdf are 0.
    The sub-path runs nearly horizontally into a wall whose BACK face is a DiffuseLight:
    emitted = 0 and no scatter (material.rs:210-222), so L = 0 and the reference computes
    (attenuation * 0 * 0) / 0 = NaN (render.rs:289-290) for the whole sample."""
    sc = rt.Scene(9)
    white = sc.lambertian((0.73, 0.73, 0.73))
    light = sc.diffuse_light((6, 6, 6))
    floor = sc.quad((-4, 0, -4), (8, 0, 0), (0, 0, 8), white)
    top = sc.quad((-1, 4, -1), (2, 0, 0), (0, 0, 2), light)
    walls = [sc.quad((6, -1, -6), (0, 4, 0), (0, 0, 12), light),    # normals point outwards:
             sc.quad((-6, -1, -6), (0, 0, 12), (0, 4, 0), light),   # rays from inside see
             sc.quad((-6, -1, 6), (0, 4, 0), (12, 0, 0), light),    # their back faces
             sc.quad((-6, -1, -6), (12, 0, 0), (0, 4, 0), light)]
    world = sc.hittable_list(floor, top, sc.sphere((0, 1, 0), 1.0, white), *walls)
    lights = sc.hittable_list(sc.quad((4.5, -1e-9, -1), (1, 0, 0), (0, 0, 2), light),
                              sc.quad((-1, 4, -1), (2, 0, 0), (0, 0, 2), light))
    blob = sc.serialize(world, lights)
    cam = rt.camera_new(1.0, 48, 16, 10, 60, (0, 3, 5), (0, 0.5, 0), (0, 1, 0), 0, 0, (0, 0, 0))
    return blob, cam


def test_zero_pdf_bounce_nan_semantics(gpu_available):
    """render.rs:287-292: a bounce with pdf_val = 0 makes the sample NaN even when its sub-path
    returns 0 (_zero_pdf_scene). The forward beta/L product alone would leave those samples
    finite (nothing is added after the bounce); the HIP path must put NaN in exactly the
    oracle's pixels and channels."""
    blob, cam = _zero_pdf_scene()
    acc_g, acc_o, _ = _compare(blob, cam)
    assert np.isnan(acc_g).mean() > 0.2 and np.isfinite(acc_g).any()


def test_black_pixels_of_the_600_cornell_camera(gpu_available):
    """book3.png's all-black pixels (31,671; tests/golden/final_images_stats.json). The count is
    not exact by construction: a pixel whose corner is clipped by the box opening is black only
    if every jittered sample misses, which depends on the reference's unseeded draws, and a
    pixel seeing dark geometry maps to 0 below sRGB8 0.5 (color.rs:30). The HIP render and the
    oracle must agree EXACTLY (same seed), and both within 0.2 % of the published count."""
    import json
    from pathlib import Path

    ref = json.loads((Path(__file__).parent / "golden" / "final_images_stats.json").read_text())
    m = ref["book3.png"]
    blob, cam = rt.preset_blob(m["preset"], variant=m["variant"], width=m["width"],
                               spp=m["spp"], depth=m["depth"])
    rows = (0, 37, 17)  # 17 rows through the top, the box and the floor
    acc_g, _ = _gpu(blob, cam, seed=1, row_begin=rows[0], row_step=rows[1], n_rows=rows[2])
    acc_o, _ = O.render(blob, cam, rt.make_opts(cam, seed=1, row_begin=rows[0], row_step=rows[1],
                                                n_rows=rows[2]), precision=64)
    rgb_g = rt.write_color(acc_g, cam.samples_per_pixel)
    rgb_o = rt.write_color(acc_o, cam.samples_per_pixel)
    black_g = rgb_g.reshape(-1, 3).sum(1) == 0
    assert np.array_equal(black_g, rgb_o.reshape(-1, 3).sum(1) == 0)
    full, _ = _gpu(blob, cam, seed=1)
    black = int((rt.write_color(full, cam.samples_per_pixel).reshape(-1, 3).sum(1) == 0).sum())
    print(f"black pixels: {black} (book3.png: {m['black_pixels']})")
    assert abs(black - m["black_pixels"]) <= 0.002 * m["black_pixels"], black


# ---------------------------------------------------------------- scene graphs the reference
# accepts that round 1 rejected (rt_flatten.cpp)
def test_nested_light_list_parity(gpu_available):
    """A HittableList inside the light list (object.rs:57, 66 -> hittable.rs:115-129): the
    mixture's light PDF folds the inner list's values times 1/len inside the outer fold, and a
    light sample draws random_int twice (outer, then inner)."""
    sc = rt.Scene(12)
    white = sc.lambertian((0.73, 0.73, 0.73))
    red = sc.lambertian((0.65, 0.05, 0.05))
    light = sc.diffuse_light((9, 9, 9))
    glass = sc.dielectric(1.5)
    world = sc.hittable_list(
        sc.quad((-5, 0, -5), (10, 0, 0), (0, 0, 10), white),
        sc.quad((-5, 0, -3), (10, 0, 0), (0, 6, 0), red),
        sc.quad((-1, 4, -1), (2, 0, 0), (0, 0, 2), light),
        sc.quad((2.5, 3, 0), (1, 0, 0), (0, 0, 1), light),
        sc.sphere((0, 1, 1), 1.0, glass))
    inner = sc.hittable_list(sc.sphere((0, 1, 1), 1.0, glass),
                             sc.quad((2.5, 3, 0), (1, 0, 0), (0, 0, 1), light))
    lights = sc.hittable_list(sc.quad((-1, 4, -1), (2, 0, 0), (0, 0, 2), light), inner)
    blob = sc.serialize(world, lights)
    assert rt.layout_stats(blob)["lights"] == 2
    cam = rt.camera_new(1.0, 64, 16, 20, 40, (0, 2.5, 9), (0, 1.5, 0), (0, 1, 0), 0, 0, (0, 0, 0))
    state, msg = _jit_state(blob, cam)
    assert state == 1, msg
    _compare(blob, cam)


def test_deep_transform_chain_parity(gpu_available):
    """Translate / RotateY nested six deep (transform.rs:12-40 nests without a limit): the hit
    record is replayed through the whole chain (rt_layout.h RTL_XFORM_LONG) in the interpreter
    and in the scene-specialised walker, including EXIT back to a 5-deep parent frame."""
    sc = rt.Scene(13)
    white = sc.lambertian((0.73, 0.73, 0.73))
    chk = sc.lambertian(tex=sc.checker_from_color(0.9, (0.9, 0.2, 0.1), (0.1, 0.3, 0.9)))
    light = sc.diffuse_light((8, 8, 8))
    obj = sc.hittable_list(sc.make_box((0, 0, 0), (0.8, 0.8, 0.8), chk),
                           sc.sphere((0.4, 1.2, 0.4), 0.3, white))
    for k in range(6):
        obj = sc.rotate_y(obj, 12 + 5 * k) if k % 2 == 0 else sc.translate(obj, (0.1 * k, 0.05, -0.1))
    obj = sc.hittable_list(obj, sc.sphere((1.5, 0.3, 0.5), 0.3, white))  # EXIT to a deep frame
    for k in range(3):
        obj = sc.translate(sc.rotate_y(obj, -7), (0.05, 0, 0.05))
    world = sc.hittable_list(sc.quad((-4, -0.01, -4), (8, 0, 0), (0, 0, 8), white), obj,
                             sc.quad((-1, 4, -1), (2, 0, 0), (0, 0, 2), light))
    lights = sc.hittable_list(sc.quad((-1, 4, -1), (2, 0, 0), (0, 0, 2), light))
    blob = sc.serialize(world, lights)
    state, msg = _jit_state(blob, cam := rt.camera_new(1.0, 64, 16, 20, 40, (0, 2.5, 7),
                                                       (0.5, 0.5, 0), (0, 1, 0), 0, 0,
                                                       (0.05, 0.05, 0.05)))
    assert state == 1, msg
    _compare(blob, cam)


def test_render_multi_devices_bitwise(gpu_available):
    """rt_render_multi (one process, N devices, cyclic rows, host de-interleave): with the box's
    one GPU listed 2 and 3 times it must give the single-device frame bit for bit, also when
    accumulating into a non-zero buffer."""
    blob, cam = rt.preset_blob("cornell_box", width=72, spp=16)
    ds = rt.DeviceScene(blob)
    full, _ = ds.render(cam, rt.make_opts(cam, seed=4))
    base = np.random.default_rng(1).random(full.shape, dtype=np.float32)
    acc_one = base.copy()
    ds.render(cam, rt.make_opts(cam, seed=4, flags=0), accum=acc_one)
    ds.close()
    for devs in ([0, 0], [0, 0, 0]):
        got, st = rt.render_multi(blob, cam, rt.make_opts(cam, seed=4), devs)
        assert np.array_equal(got, full), devs
        assert st.samples == 72 * 72 * 16 and st.launches == len(devs)
        acc = base.copy()
        rt.render_multi(blob, cam, rt.make_opts(cam, seed=4, flags=0), devs, accum=acc)
        assert np.array_equal(acc, acc_one), devs


def test_multi_handle_renders_frames_without_reupload(gpu_available):
    """rt_multi_* (ABI v3): the scene is uploaded to each listed device once; every frame is
    rendered in cyclic rows on all of them and gathered peer to peer into a devices[0] buffer.
    With the box's one GPU listed 2 and 3 times the frame equals rt_render's bit for bit, also
    when accumulating; the second frame does no upload and no staging allocation
    (rt_multi_info counters)."""
    from hip_buf import DevBuf

    blob, cam = rt.preset_blob("cornell_box", width=72, spp=16)
    ds = rt.DeviceScene(blob)
    full, _ = ds.render(cam, rt.make_opts(cam, seed=4))
    base = np.random.default_rng(1).random(full.shape, dtype=np.float32)
    acc_one = base.copy()
    ds.render(cam, rt.make_opts(cam, seed=4, flags=0), accum=acc_one)
    ds.close()
    for devs in ([0, 0], [0, 0, 0]):
        m = rt.MultiScene(blob, devs)
        out = DevBuf(full.shape)
        st1 = m.render_device(cam, rt.make_opts(cam, seed=4), out.ptr, stats=True)
        assert np.array_equal(out.download(), full), devs
        assert st1.samples == 72 * 72 * 16
        info1 = m.info()
        out.upload(np.zeros_like(full))
        st2 = m.render_device(cam, rt.make_opts(cam, seed=4), out.ptr, stats=True)
        assert np.array_equal(out.download(), full), devs
        info2 = m.info()
        assert info1["uploads"] == info2["uploads"] == len(devs)
        assert info2["frames"] == 2 and info2["stage_allocs"] == info1["stage_allocs"] == 1
        print(f"rt_multi {devs}: frame 1 {st1.ms_total:.2f} ms, frame 2 {st2.ms_total:.2f} ms")
        out.upload(base)
        m.render_device(cam, rt.make_opts(cam, seed=4, flags=0), out.ptr, stats=True)
        assert np.array_equal(out.download(), acc_one), devs
        out.free()
        m.close()


def test_nested_constant_medium_parity(gpu_available):
    """A ConstantMedium whose boundary holds another ConstantMedium (constant_medium.rs:46-55:
    `boundary.hit` is the inner medium's hit, with its own random draw per query), two levels
    deep, in the reference's draw order."""
    sc = rt.Scene(14)
    white = sc.lambertian((0.73, 0.73, 0.73))
    light = sc.diffuse_light((8, 8, 8))
    inner = sc.constant_medium(sc.sphere((0, 1, 0), 0.6, white), 3.0, (0.9, 0.3, 0.2))
    mid = sc.constant_medium(sc.hittable_list(sc.sphere((0, 1, 0), 1.0, white), inner), 1.5,
                             (0.2, 0.5, 0.9))
    outer = sc.constant_medium(sc.hittable_list(sc.sphere((0, 1, 0), 1.4, white), mid), 0.6,
                               (0.8, 0.8, 0.8))
    world = sc.hittable_list(sc.quad((-4, -0.01, -4), (8, 0, 0), (0, 0, 8), white), outer,
                             sc.quad((-1, 4, -1), (2, 0, 0), (0, 0, 2), light))
    lights = sc.hittable_list(sc.quad((-1, 4, -1), (2, 0, 0), (0, 0, 2), light))
    blob = sc.serialize(world, lights)
    cam = rt.camera_new(1.0, 64, 16, 20, 40, (0, 2, 6), (0, 1, 0), (0, 1, 0), 0, 0, (0.05, 0.05, 0.05))
    acc_g, _, st = _compare(blob, cam)
    assert st.op_counts()["volume_draws"] > 0


def _random_scene(seed):
    """A seeded random room for parity fuzzing: walls and a ceiling light, then spheres (static,
    moving), boxes (some under RotateY + Translate), axis-aligned and general quads, a
    ConstantMedium, checker / noise textures, every material kind, part of it inside a BVH, and a
    light list of the ceiling quad plus a sphere light."""
    rnd = np.random.default_rng(seed)
    sc = rt.Scene(seed)
    u = lambda a, b: float(rnd.uniform(a, b))  # noqa: E731
    col = lambda: tuple(float(x) for x in rnd.uniform(0.1, 0.9, 3))  # noqa: E731
    white = sc.lambertian((0.73, 0.73, 0.73))
    light = sc.diffuse_light((12.0, 12.0, 12.0))
    walls = [sc.quad((10, 0, 0), (0, 10, 0), (0, 0, 10), sc.lambertian(col())),
             sc.quad((0, 0, 0), (0, 10, 0), (0, 0, 10), sc.lambertian(col())),
             sc.quad((0, 0, 0), (10, 0, 0), (0, 0, 10), white),
             sc.quad((10, 10, 10), (-10, 0, 0), (0, 0, -10), white),
             sc.quad((0, 0, 10), (10, 0, 0), (0, 10, 0), white)]
    lamp = sc.quad((3.5, 9.99, 3.5), (3, 0, 0), (0, 0, 3), light)
    tex = [sc.checker_from_color(u(0.5, 2.0), col(), col()), sc.noise_texture(u(0.5, 4.0))]
    mats = [sc.lambertian(col()), sc.lambertian(tex=tex[0]), sc.lambertian(tex=tex[1]),
            sc.metal(col(), u(0.0, 0.5)), sc.dielectric(u(1.3, 1.7)), sc.isotropic(col())]
    objs, bvh_items = [], []
    for k in range(int(rnd.integers(8, 14))):
        kind = int(rnd.integers(0, 5))
        m = mats[int(rnd.integers(0, len(mats)))]
        c = (u(1.5, 8.5), u(1.0, 7.0), u(1.5, 8.5))
        if kind == 0:
            o = sc.sphere(c, u(0.3, 1.2), m)
        elif kind == 1:
            o = sc.sphere_moving(c, (c[0], c[1] + u(0, 0.5), c[2]), u(0.3, 1.0), m)
        elif kind == 2:
            s = u(0.5, 2.0)
            o = sc.make_box((0, 0, 0), (s, u(0.5, 3.0), s), m)
            o = sc.translate(sc.rotate_y(o, u(-40, 40)), (c[0] - 1, 0, c[2] - 1))
        elif kind == 3:
            o = sc.quad(c, (u(0.5, 1.5), 0, 0), (0, u(0.5, 1.5), 0), m)
        else:
            o = sc.quad(c, (u(0.5, 1.5), u(-0.5, 0.5), 0), (0, u(0.2, 1.0), u(0.5, 1.5)), m)
        (bvh_items if rnd.uniform() < 0.5 else objs).append(o)
    fog = sc.constant_medium(sc.sphere((u(3, 7), u(2, 5), u(3, 7)), u(0.8, 1.6), white), u(0.2, 1.0),
                             col())
    bulb_c = (u(2, 8), 8.5, u(2, 8))
    bulb = sc.sphere(bulb_c, 0.4, light)
    items = walls + [lamp, fog, bulb] + objs
    if bvh_items:
        items.append(sc.create_bvh(sc.hittable_list(*bvh_items)))
    world = sc.hittable_list(*items)
    lights = sc.hittable_list(sc.quad((3.5, 9.99, 3.5), (3, 0, 0), (0, 0, 3), light),
                              sc.sphere(bulb_c, 0.4, light))
    # odd seeds: a thin lens; every third seed: a sky background; every fourth: no light list
    # (the material-only scatter path of render.rs ray_color)
    blob = sc.serialize(world, None if seed % 4 == 0 else lights)
    defocus = (0.8, 14.0) if seed % 2 else (0.0, 0.0)
    bg = (0.7, 0.8, 1.0) if seed % 3 == 0 else (0.0, 0.0, 0.0)
    cam = rt.camera_new(u(0.8, 1.6), 40, 9, 10, u(40, 70), (5, 5, -9), (5, 4.5, 5), (0, 1, 0),
                        *defocus, bg)
    return blob, cam


@pytest.mark.parametrize("seed", range(1, 13))
def test_random_scene_parity(gpu_available, seed):
    """Seeded random scenes (_random_scene) through the whole product path: the scene-specialised
    kernel equals the interpreter and the op-counting build bit for bit, and the image and op
    counts match the oracle."""
    blob, cam = _random_scene(seed)
    acc_g, acc_o, st = _compare(blob, cam)
    assert np.isfinite(acc_g).any() and acc_g[np.isfinite(acc_g)].mean() > 0.0


@pytest.mark.parametrize("case", ["empty_world", "1x1_1spp_depth1", "1x1_4spp", "3x3_1spp",
                                  "odd_17x11"])
def test_degenerate_sizes_parity(gpu_available, case):
    """Edge sizes of render.rs's loop: an empty world (every sample is the background,
    render.rs:270-272), a one-pixel image (image_height >= 1, render.rs:70-71), one sample per
    pixel (sqrt_spp = 1, render.rs:75-76), depth 1, and an odd size that fills no 8x8 tile."""
    sc = rt.Scene(2)
    world = (sc.hittable_list() if case == "empty_world" else
             sc.hittable_list(sc.sphere((0, 0, 0), 0.5, sc.lambertian((0.5, 0.5, 0.5))),
                              sc.quad((-2, -0.5, -2), (4, 0, 0), (0, 0, 4), sc.metal((0.8, 0.8, 0.8), 0.1))))
    blob = sc.serialize(world)
    wd, spp, depth, aspect = {"empty_world": (17, 4, 5, 1.5), "1x1_1spp_depth1": (1, 1, 1, 1.0),
                              "1x1_4spp": (1, 4, 2, 1.0), "3x3_1spp": (3, 1, 50, 1.0),
                              "odd_17x11": (17, 9, 10, 1.5)}[case]
    cam = rt.camera_new(aspect, wd, spp, depth, 50, (0, 0.3, -3), (0, 0, 0), (0, 1, 0), 0, 0,
                        (0.7, 0.8, 1.0))
    acc_g, acc_o, st = _compare(blob, cam)
    assert acc_g.shape == (cam.image_height, wd, 3)
    if case == "empty_world":
        n = cam.samples_per_pixel
        assert np.allclose(acc_g, np.array([0.7, 0.8, 1.0], np.float32) * n, rtol=1e-6)
