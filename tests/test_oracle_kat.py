"""Known-answer tests pinning the CPU oracle to the reference formulas.

The reference ships no tests or golden vectors, so each expectation below is
derived analytically from the cited reference function. These tests are what make the oracle
trustworthy as the parity checker for the GPU path.
"""
import math

import numpy as np
import pytest

import oracle_lib as O
import surely_rt as rt

PI = math.pi


def _scene(build):
    sc = rt.Scene(1)
    world, lights = build(sc)
    return sc.serialize(world, lights)


def _hit(blob, o, d, tmin=1e-4, tmax=math.inf, tm=0.0):
    return O.world_hit(blob, list(o) + list(d) + [tm], tmin, tmax)


# ---------------------------------------------------------------- RNG (App. A S4)
def test_rng_deterministic_uniform_and_keyed():
    a = O.rng_draws(1, 123, 45, 1000)
    assert np.array_equal(a, O.rng_draws(1, 123, 45, 1000))
    assert (a >= 0).all() and (a < 1).all()
    assert not np.array_equal(a, O.rng_draws(1, 124, 45, 1000))
    assert not np.array_equal(a, O.rng_draws(1, 123, 46, 1000))
    assert not np.array_equal(a, O.rng_draws(2, 123, 45, 1000))
    # 32-bit uniforms: u = x * 2^-32 exactly
    u = O.rng_u32(1, 123, 45, 10).astype(np.float64) * 2.0 ** -32
    assert np.array_equal(u, a[:10])
    # uniformity over many keys (first draw of each stream and a later one)
    first = np.array([O.rng_draws(7, p, s, 8) for p in range(64) for s in range(64)])
    for col in (0, 7):
        hist, _ = np.histogram(first[:, col], bins=16, range=(0, 1))
        chi2 = ((hist - hist.mean()) ** 2 / hist.mean()).sum()
        assert chi2 < 45, chi2  # 15 dof, p ~ 1e-4
    # adjacent keys are uncorrelated
    c = np.corrcoef(first[:-1, 0], first[1:, 0])[0, 1]
    assert abs(c) < 0.05


def _rng_restated(seed, pixel, sample, n):
    """pcg2d key with seed-keyed increments, then xoroshiro64* (csrc/rt_rng.h rng_seed / rng_step,
    DESIGN.md §4.1 RNG), restated in Python integers."""
    m = 0xFFFFFFFF
    lo, hi = seed & m, (seed >> 32) & m
    k0 = (((lo ^ 0x85EBCA6B) * 0x9E3779B9) + 1013904223) & m
    k1 = (((hi ^ 0xC2B2AE35) * 0x9E3779B9) + (k0 ^ 0x27D4EB2F)) & m
    v0, v1 = (pixel * 1664525 + k0) & m, (sample * 1664525 + k1) & m
    for _ in range(2):
        v0 = (v0 + v1 * 1664525) & m
        v1 = (v1 + v0 * 1664525) & m
        v0 ^= v0 >> 16
        v1 ^= v1 >> 16
    if v0 | v1 == 0:
        v0 = 0x9E3779B9
    rotl = lambda x, k: ((x << k) | (x >> (32 - k))) & m  # noqa: E731
    out = []
    for _ in range(n):
        out.append((v0 * 0x9E3779BB) & m)
        s1 = v1 ^ v0
        v0 = rotl(v0, 26) ^ s1 ^ ((s1 << 9) & m)
        v1 = rotl(s1, 13)
    return np.array(out, dtype=np.uint64)


@pytest.mark.parametrize("seed,pixel,sample", [(1, 0, 0), (1, 123, 45), (7, 639999, 960),
                                               ((5 << 32) | 3, 2**31 + 7, 9999)])
def test_rng_is_the_documented_generator(seed, pixel, sample):
    """The oracle's stream is exactly pcg2d + xoroshiro64* (round 6, S4), so the device's
    generator (the GPU tests require equal images) is the documented one too."""
    got = O.rng_u32(seed, pixel, sample, 16).astype(np.uint64)
    assert np.array_equal(got, _rng_restated(seed, pixel, sample, 16))


# ---------------------------------------------------------------- camera (render.rs:218-249)
def test_camera_ray_stratified_jitter():
    cam = rt.camera_new(1.0, 600, 1000, 50, 40.0, (278, 278, -800), (278, 278, 0), (0, 1, 0),
                        0.0, 0.0, (0, 0, 0))
    i, j, s_i, s_j = 300, 123, 7, 29
    r = O.camera_ray(cam, 1, i, j, s_i, s_j)
    u = O.rng_draws(1, j * 600 + i, s_j * 31 + s_i, 3)
    p00, du, dv = np.array(cam.pixel00_loc), np.array(cam.pixel_delta_u), np.array(cam.pixel_delta_v)
    px = -0.5 + (1 / 31) * (s_i + u[0])
    py = -0.5 + (1 / 31) * (s_j + u[1])
    ps = p00 + i * du + j * dv + px * du + py * dv
    np.testing.assert_allclose(r[:3], [278, 278, -800])
    np.testing.assert_allclose(r[3:6], ps - np.array([278, 278, -800]), rtol=1e-12, atol=1e-12)
    assert r[6] == u[2]  # ray time = third draw (render.rs:233)


def test_camera_defocus_disk():
    """defocus_disk_sample render.rs:238-241: origin within the disk of radius
    focus_dist * tan(angle/2) around the camera centre."""
    cam = rt.camera_new(16 / 9, 100, 4, 5, 20.0, (13, 2, 3), (0, 0, 0), (0, 1, 0), 0.6, 10.0, (0, 0, 0))
    rad = 10.0 * math.tan(math.radians(0.3))
    ds = []
    for k in range(200):
        r = O.camera_ray(cam, 3, k % 100, k // 100, 0, 1)
        ds.append(np.linalg.norm(r[:3] - np.array([13, 2, 3])))
    assert max(ds) <= rad * (1 + 1e-12) and min(ds) < rad and max(ds) > 0.5 * rad


# ---------------------------------------------------------------- intersection
def test_sphere_hit_outside_inside_and_strict_interval():
    """Sphere::hit object.rs:145-184 + set_face_normal hittable.rs:22-37."""
    blob = _scene(lambda sc: (sc.hittable_list(sc.sphere((0, 0, 0), 1, sc.lambertian((1, 1, 1)))), None))
    h = _hit(blob, (0, 0, -5), (0, 0, 1))
    np.testing.assert_allclose(h[:7], [4, 0, 0, -1, 0, 0, -1])
    assert h[7] == 1  # front face
    h = _hit(blob, (0, 0, 0), (0, 0, 2))  # from inside, non-unit direction: t = 0.5
    np.testing.assert_allclose(h[:7], [0.5, 0, 0, 1, 0, 0, -1])
    assert h[7] == 0
    # strict interval: a root exactly at tmax is rejected
    assert _hit(blob, (0, 0, -5), (0, 0, 1), tmax=4.0) is None
    assert _hit(blob, (0, 0, -5), (0, 0, 1), tmax=4.0 + 1e-9) is not None
    # moving sphere: centre at time t (object.rs:107-112)
    blob = _scene(lambda sc: (sc.hittable_list(
        sc.sphere_moving((0, 0, 0), (2, 0, 0), 1, sc.lambertian((1, 1, 1)))), None))
    h = _hit(blob, (1, 0, -5), (0, 0, 1), tm=0.5)
    assert h[0] == pytest.approx(4.0) and h[1] == pytest.approx(1.0)


def test_quad_hit_inclusive_interval_and_edges():
    """Quad::hit object.rs:453-490: inclusive interval and inclusive [0,1] planar bounds."""
    blob = _scene(lambda sc: (sc.hittable_list(
        sc.quad((-1, -1, 3), (2, 0, 0), (0, 2, 0), sc.lambertian((1, 1, 1)))), None))
    h = _hit(blob, (0, 0, 0), (0, 0, 1))
    # normal = unit(u x v) = (0,0,1); the ray travels along +z -> back face
    np.testing.assert_allclose(h[:7], [3, 0, 0, 3, 0, 0, -1])
    assert h[7] == 0
    assert _hit(blob, (0, 0, 0), (0, 0, 1), tmax=3.0) is not None  # t == tmax accepted
    assert _hit(blob, (-1, -1, 0), (0, 0, 1)) is not None        # corner a = b = 0
    assert _hit(blob, (1, 1, 0), (0, 0, 1)) is not None          # corner a = b = 1
    assert _hit(blob, (1.0000001, 0, 0), (0, 0, 1)) is None
    assert _hit(blob, (0, 0, 0), (1, 0, 0)) is None                # parallel: |n.d| < 1e-8


def test_list_later_quad_wins_ties_and_bvh_right_wins():
    """HittableList::hit (hittable.rs:88-109) passes [min, closest] with an inclusive quad
    interval, so a later coplanar quad replaces an earlier one; BvhNode::hit (216-236) tests the
    right child with max = left.t, so the right child wins ties."""
    def build(bvh):
        def f(sc):
            m0, m1 = sc.lambertian((1, 0, 0)), sc.lambertian((0, 1, 0))
            q0 = sc.quad((-1, -1, 3), (2, 0, 0), (0, 2, 0), m0)
            q1 = sc.quad((-1, -1, 3), (2, 0, 0), (0, 2, 0), m1)
            lst = sc.hittable_list(q0, q1)
            return (sc.create_bvh(lst) if bvh else lst), None
        return f
    h = _hit(_scene(build(False)), (0, 0, 0), (0, 0, 1))
    mats = h[8]
    blob = _scene(build(True))
    hb = _hit(blob, (0, 0, 0), (0, 0, 1))
    assert hb is not None and h is not None
    # materials are registered in the order quads are serialised; the list winner is the
    # second quad; the BVH winner is whichever child ended up on the right
    assert mats == 1.0
    assert hb[8] in (0.0, 1.0)


def test_transforms_rotate_translate():
    """RotateY/Translate::hit transform.rs:57-135: object-space hit moved back to world."""
    def f(sc):
        box = sc.make_box((0, 0, 0), (1, 1, 1), sc.lambertian((1, 1, 1)))
        return sc.hittable_list(sc.translate(sc.rotate_y(box, 90), (10, 0, 0))), None
    blob = _scene(f)
    # rotate_y(90): (x,z) -> (x cos + z sin, -x sin + z cos) = (z, -x): box spans x in [0,1], z in [-1,0]
    h = _hit(blob, (10.5, 0.5, 5), (0, 0, -1))
    assert h[0] == pytest.approx(5.0, abs=1e-12)
    np.testing.assert_allclose(h[1:4], [10.5, 0.5, 0.0], atol=1e-12)
    np.testing.assert_allclose(h[4:7], [0, 0, 1], atol=1e-12)


def test_constant_medium_boundary():
    """ConstantMedium::hit constant_medium.rs:41-95 with density -> infinity hits at entry;
    with a density -> 0 it never hits."""
    def f(density):
        def g(sc):
            b = sc.sphere((0, 0, 0), 1, sc.dielectric(1.5))
            return sc.hittable_list(sc.constant_medium(b, density, (1, 1, 1))), None
        return g
    h = _hit(_scene(f(1e12)), (0, 0, -5), (0, 0, 1))
    assert h is not None and h[0] == pytest.approx(4.0, abs=1e-6)
    np.testing.assert_allclose(h[4:7], [1, 0, 0])  # arbitrary normal (constant_medium.rs:84)
    assert _hit(_scene(f(1e-12)), (0, 0, -5), (0, 0, 1)) is None


# ---------------------------------------------------------------- get_sphere_uv (object.rs:134-141)
def test_sphere_uv_axis_points():
    pts = np.array([(1, 0, 0), (0, 1, 0), (0, 0, 1), (-1, 0, 0), (0, -1, 0), (0, 0, -1)], float)
    uv = O.sphere_uv(pts)
    # u = (atan2(-z, x) + pi) / 2pi, v = acos(-y) / pi
    exp = [(math.atan2(-z, x) + PI) / (2 * PI) for x, y, z in pts]
    np.testing.assert_allclose(uv[:, 0], exp, atol=1e-15)
    np.testing.assert_allclose(uv[:, 1], [0.5, 1.0, 0.5, 0.5, 0.0, 0.5], atol=1e-15)


# ---------------------------------------------------------------- PDFs (pdf.rs, object.rs)
def _fib_sphere(n):
    k = np.arange(n) + 0.5
    z = 1 - 2 * k / n
    phi = PI * (1 + 5 ** 0.5) * k
    r = np.sqrt(1 - z * z)
    return np.stack([r * np.cos(phi), r * np.sin(phi), z], 1)


def test_light_pdfs_integrate_to_one():
    """Quad::pdf_value (object.rs:492-501) and Sphere::pdf_value (190-202) are densities over
    solid angle; HittableList::pdf_value averages them (hittable.rs:115-124): each integrates
    to 1 over the sphere of directions."""
    blob, _ = rt.preset_blob("cornell_box", width=8, spp=1)
    dirs = _fib_sphere(2_000_000)
    for origin in [(278, 0.5, 278), (100, 300, 500), (554, 200, 100)]:
        pdf = O.light_pdf_batch(blob, origin, dirs)
        integral = pdf.mean() * 4 * PI
        assert integral == pytest.approx(1.0, abs=0.02), (origin, integral)


def test_light_generate_matches_pdf():
    """HittablePDF::generate (pdf.rs:95-97) samples the density HittablePDF::value evaluates:
    E_generate[f(dir)/pdf(dir)] == integral of f over directions (f = 1 on the lights' support)."""
    blob, _ = rt.preset_blob("cornell_box", width=8, spp=1)
    origin = (278, 0.5, 278)
    d = O.light_generate(blob, origin, 20000, seed=3)
    pdf = O.light_pdf_batch(blob, origin, d)
    assert (pdf > 0).mean() > 0.999
    # half the samples go to each light (random_int over 2 lights)
    quad = np.abs(d[:, 1] / np.linalg.norm(d, axis=1))
    dirs = _fib_sphere(1_000_000)
    support = (O.light_pdf_batch(blob, origin, dirs) > 0).mean() * 4 * PI
    est = np.mean(1.0 / pdf)
    assert est == pytest.approx(support, rel=0.03)
    assert quad.min() > 0


def test_cosine_sampling_distribution():
    """random_cosine_direction (vec3.rs:240-250) in the Onb of w (onb.rs:32-47): unit vectors,
    E[cos] = 2/3, E[cos^2] = 1/2."""
    w = np.array([0.3, -0.5, 0.8])
    d = O.cosine_dirs(w, 100000, seed=5)
    np.testing.assert_allclose(np.linalg.norm(d, axis=1), 1, atol=1e-12)
    c = d @ (w / np.linalg.norm(w))
    assert (c >= 0).all()
    assert c.mean() == pytest.approx(2 / 3, abs=0.005)
    assert (c * c).mean() == pytest.approx(0.5, abs=0.005)


# ---------------------------------------------------------------- fp32 study build math
@pytest.mark.parametrize("fn", ["sin2pi", "cos2pi", "log", "sin", "acos", "atan2"])
def test_f32_study_math_accuracy(fn):
    """The f32 precision-study build (oracle/rt_oracle.c ORACLE_F64=0) uses polynomial
    transcendentals (tools/fit_fmath.py); each is within a few float ulps of libm."""
    rng = np.random.default_rng(0)
    n = 200000
    y = None
    if fn in ("sin2pi", "cos2pi"):
        x = rng.random(n).astype(np.float32)
        ref = np.sin(2 * PI * x.astype(np.float64)) if fn == "sin2pi" else np.cos(2 * PI * x.astype(np.float64))
    elif fn == "log":
        x = np.exp(rng.uniform(-40, 5, n)).astype(np.float32)
        ref = np.log(x.astype(np.float64))
    elif fn == "sin":
        x = rng.uniform(-200, 200, n).astype(np.float32)
        ref = np.sin(x.astype(np.float64))
    elif fn == "acos":
        x = rng.uniform(-1, 1, n).astype(np.float32)
        ref = np.arccos(x.astype(np.float64))
    else:
        x = rng.normal(size=n).astype(np.float32)
        y = rng.normal(size=n).astype(np.float32)
        ref = np.arctan2(x.astype(np.float64), y.astype(np.float64))
    got = O.fmath(fn, x, y).astype(np.float64)
    ulp = np.spacing(np.abs(ref).astype(np.float32)).astype(np.float64)
    err = np.abs(got - ref) / np.maximum(ulp, np.spacing(np.float32(1e-3)))
    assert err.max() < 8, err.max()


def _turb_reference(ranvec, perms, p):
    """perlin.rs:30-96 restated line by line in Python floats (f64, the reference's order)."""
    def sat_i32(f):
        if f != f:
            return 0
        return int(max(-2147483648.0, min(2147483647.0, f)))

    def noise(p):
        u = p[0] - math.floor(p[0])
        v = p[1] - math.floor(p[1])
        w = p[2] - math.floor(p[2])
        i, j, k = sat_i32(math.floor(p[0])), sat_i32(math.floor(p[1])), sat_i32(math.floor(p[2]))
        c = [[[ranvec[perms[0][(i + di) & 255] ^ perms[1][(j + dj) & 255] ^ perms[2][(k + dk) & 255]]
               for dk in range(2)] for dj in range(2)] for di in range(2)]
        return trilinear_interp(c, u, w, v)

    def trilinear_interp(c, u, w, v):
        uu = u * u * (3. - 2. * u)
        vv = v * v * (3. - 2. * v)
        ww = w * w * (3. - 2. * w)
        accum = 0.
        for i in range(2):
            for j in range(2):
                for k in range(2):
                    cv = c[i][j][k]
                    wv = (u - i, v - j, w - k)
                    d = (cv[0] * wv[0] + cv[1] * wv[1]) + cv[2] * wv[2]  # vec3.rs:168
                    accum += ((i * uu + (1. - i) * (1. - uu)) * (j * vv + (1. - j) * (1. - vv))
                              * (k * ww + (1. - k) * (1. - ww)) * d)
        return accum

    accum, weight, tp = 0., 1., list(p)
    for _ in range(7):  # turb_depth(p, 7)
        accum += weight * noise(tp)
        weight *= 0.5
        tp = [x * 2. for x in tp]
    return abs(accum)


def test_perlin_turb_matches_the_reference_formulas():
    """Perlin::turb (perlin.rs:56-72; noise 30-54, trilinear_interp 74-96), the noise texture
    of C4's marble sphere (texture.rs:127-130): the f64 oracle equals a line-by-line Python
    restatement bit for bit, on random tables and points incl. negative coordinates."""
    rng = np.random.default_rng(11)
    ranvec = rng.normal(size=(256, 3))
    ranvec /= np.linalg.norm(ranvec, axis=1, keepdims=True)
    perms = np.stack([rng.permutation(256) for _ in range(3)]).astype(np.int32)
    pts = np.concatenate([rng.uniform(-300, 300, size=(200, 3)), rng.uniform(-2, 2, size=(56, 3))])
    out = np.zeros(len(pts))
    O.lib(64).oracle_perlin_turb(ranvec.ctypes.data, perms.ctypes.data, pts.ctypes.data, len(pts),
                                 out.ctypes.data)
    ref = [_turb_reference(ranvec.tolist(), perms.tolist(), p) for p in pts.tolist()]
    assert np.array_equal(out, np.array(ref))
    assert 0.0 < out.mean() < 2.0
