"""Host scene builder (C++ mirror of the reference constructors) and output stage KATs.
Expected values are derived by hand from the reference formulas (cited per test)."""
import math
import struct

import numpy as np
import pytest

import surely_rt as rt


def f64(slot) -> float:
    return struct.unpack("<d", struct.pack("<Q", int(slot)))[0]


def test_nearest_square_and_camera_cornell():
    """render.rs:38-41 (spp -> floor(sqrt)^2) and Camera::new 62-133 at main.rs:496-508."""
    for spp, eff in [(1000, 961), (5000, 4900), (16, 16), (10000, 10000), (2, 1)]:
        cam = rt.camera_new(1.0, 10, spp, 5, 40.0, (278, 278, -800), (278, 278, 0), (0, 1, 0),
                            0.0, 0.0, (0, 0, 0))
        assert cam.samples_per_pixel == eff and cam.sqrt_spp ** 2 == eff
    cam = rt.camera_new(1.0, 600, 1000, 50, 40.0, (278, 278, -800), (278, 278, 0), (0, 1, 0),
                        0.0, 0.0, (0, 0, 0))
    assert (cam.image_width, cam.image_height) == (600, 600)
    # focus_dist <= 0 -> 1; viewport_height = 2*tan(20deg); w = (0,0,-1), u = (-1,0,0), v = (0,1,0)
    h = 2.0 * math.tan(math.radians(20.0))
    du = -h / 600.0
    assert cam.pixel_delta_u[0] == pytest.approx(du, rel=1e-14)
    assert cam.pixel_delta_v[1] == pytest.approx(-h / 600.0, rel=1e-14)
    # pixel00 = center - focus*w - vu/2 - vv/2 + 0.5*(du+dv) = (278 + h/2 + du/2, 278 + h/2 - ..., -799)
    assert cam.pixel00_loc[2] == pytest.approx(-799.0)
    assert cam.pixel00_loc[0] == pytest.approx(278 + h / 2 + du / 2, rel=1e-14)
    assert cam.recip_sqrt_spp == pytest.approx(1 / 31)
    # 16:9 at 3840 wide -> 2160 exactly
    cam = rt.camera_new(16 / 9, 3840, 10000, 50, 40, (0, 0, 0), (0, 0, -1), (0, 1, 0), 0, 0, (0, 0, 0))
    assert cam.image_height == 2160


def test_quad_constructor_fields():
    """Quad::new object.rs:427-446: n = u x v, normal = unit(n), w = n/(n.n), D = normal.q,
    area = |n|; bbox padded (object.rs:372-391)."""
    sc = rt.Scene(1)
    m = sc.lambertian((1, 1, 1))
    q = sc.quad((343, 554, 332), (-130, 0, 0), (0, 0, -105), m)
    blob = sc.serialize(sc.hittable_list(q))
    s = blob.slots
    w = int(s[9])
    rec = s[w + 8:]
    assert int(rec[0]) == 4 and int(rec[1]) == 0  # QUAD, mat 0
    vals = [f64(x) for x in rec[2:2 + 17]]
    qv, u, v, n, ww, d, area = vals[0:3], vals[3:6], vals[6:9], vals[9:12], vals[12:15], vals[15], vals[16]
    assert qv == [343, 554, 332]
    # u x v = (-130,0,0) x (0,0,-105) = (0, -13650, 0)
    assert n == [0.0, -1.0, 0.0]
    assert ww[1] == pytest.approx(-1 / 13650.0)
    assert d == -554.0 and area == 13650.0
    bbox = [f64(x) for x in rec[19:25]]
    assert bbox[2] == pytest.approx(554 - 0.00005) and bbox[3] == pytest.approx(554 + 0.00005)


def test_make_box_and_rotate_translate_bbox():
    """make_box object.rs:509-560 (6 quads); RotateY bbox transform.rs:143-186; Translate 43-54."""
    sc = rt.Scene(1)
    m = sc.lambertian((1, 1, 1))
    box = sc.make_box((0, 0, 0), (165, 330, 165), m)
    assert sc.list_len(box) == 6
    b = sc.bbox(box)
    # each face is padded by delta/2 = 5e-5 along its thin axis (Aabb::pad object.rs:372-391)
    e = 5e-5
    np.testing.assert_allclose(b, [-e, 165 + e, -e, 330 + e, -e, 165 + e], rtol=0, atol=1e-12)
    r = sc.rotate_y(box, 15)
    c, s = math.cos(math.radians(15)), math.sin(math.radians(15))
    xs = [c * x + s * z for x in (-e, 165 + e) for z in (-e, 165 + e)]
    zs = [-s * x + c * z for x in (-e, 165 + e) for z in (-e, 165 + e)]
    np.testing.assert_allclose(sc.bbox(r), [min(xs), max(xs), -e, 330 + e, min(zs), max(zs)],
                               rtol=1e-13)
    t = sc.translate(r, (265, 0, 295))
    np.testing.assert_allclose(sc.bbox(t), sc.bbox(r) + [265, 265, 0, 0, 295, 295], rtol=1e-13)


def _tree(slots, off):
    """Decode the prefix object tree into nested tuples (tag, children)."""
    sizes = {3: 16, 4: 25}
    tag = int(slots[off])
    if tag == 1:
        n = int(slots[off + 1])
        p, kids = off + 8, []
        for _ in range(n):
            k, p = _tree(slots, p)
            kids.append(k)
        return (1, kids), p
    if tag == 2:
        l, p = _tree(slots, off + 7)
        r, p = _tree(slots, p)
        return (2, [l, r]), p
    if tag in sizes:
        return (tag, []), off + sizes[tag]
    head = {5: 10, 6: 9, 7: 9}[tag]
    k, p = _tree(slots, off + head)
    return (tag, [k]), p


def _leaves(t):
    tag, kids = t
    if tag in (3, 4):
        return 1
    return sum(_leaves(k) for k in kids)


def test_bvh_topology_matches_reference_rules():
    """BvhNode::new hittable.rs:147-187: span 1 duplicates the object, span 2 an ordered pair,
    else median split; each object appears once except span-1 duplicates."""
    for n in (1, 2, 3, 5, 8, 13, 400):
        sc = rt.Scene(3)
        m = sc.lambertian((1, 1, 1))
        lst = sc.hittable_list(*[sc.sphere((sc.random_range(0, 10), 0, 0), 0.1, m) for _ in range(n)])
        blob = sc.serialize(sc.create_bvh(lst))
        tree, end = _tree(blob.slots, int(blob.slots[9]))
        assert end == int(blob.slots[4])  # tree ends where the texture table starts
        # expected leaf count: recursion of spans
        def leaves(span):
            if span == 1:
                return 2
            if span == 2:
                return 2
            return leaves(span // 2) + leaves(span - span // 2)
        expect = 2 if n == 1 else leaves(n)
        assert _leaves(tree) == expect


def test_bvh_deterministic_with_seed():
    def build(seed):
        blob, _ = rt.preset_blob("final_scene", width=16, spp=1, build_seed=seed)
        return blob.slots
    assert np.array_equal(build(1), build(1))
    assert not np.array_equal(build(1), build(2))


def test_serialized_header_and_tables():
    blob, cam = rt.preset_blob("final_scene", width=32, spp=4)
    h = blob.header()
    assert h["n_perlin"] == 1 and h["lights_off"] == -1
    s = blob.slots
    assert int(s[0]) == 0x52545343 and int(s[1]) == 1 and int(s[2]) == s.size
    # perlin permutations are permutations of 0..255 (perlin.rs:97-117)
    p0 = int(s[8]) + 768
    for k in range(3):
        perm = s[p0 + 256 * k: p0 + 256 * (k + 1)].astype(np.int64)
        assert sorted(perm.tolist()) == list(range(256))
    # ranvec entries are unit vectors (perlin.rs:19)
    rv = np.array([f64(x) for x in s[int(s[8]):int(s[8]) + 768]]).reshape(256, 3)
    np.testing.assert_allclose(np.linalg.norm(rv, axis=1), 1.0, rtol=1e-14)
    # cornell: lights = HittableList[Quad, Sphere] (main.rs:485-494)
    blob, _ = rt.preset_blob("cornell_box", width=32, spp=4)
    lo = blob.header()["lights_off"]
    assert int(blob.slots[lo]) == 1 and int(blob.slots[lo + 1]) == 2


def test_metal_fuzz_clamped():
    """Metal::new material.rs:118-121 clamps fuzz to 1."""
    sc = rt.Scene(1)
    m = sc.metal((0.8, 0.8, 0.9), 3.0)
    blob = sc.serialize(sc.hittable_list(sc.sphere((0, 0, 0), 1, m)))
    mo = int(blob.slots[6])
    assert int(blob.slots[mo]) == 2 and f64(blob.slots[mo + 4]) == 1.0


@pytest.mark.parametrize("lin,expect", [
    (0.0, 0), (-1.0, 0), (float("nan"), 0), (1.0, 255), (100.0, 255),
    (0.0031308, int(256 * 12.92 * 0.0031308)),
    (0.5, int(256 * (1.055 * 0.5 ** (1 / 2.4) - 0.055))),
    (0.2, int(256 * (1.055 * 0.2 ** (1 / 2.4) - 0.055))),
])
def test_write_color_byte_mapping(lin, expect):
    """color.rs:8-33: scale by 1/spp, sRGB OETF (53-59), clamp [0, 0.999], (256*x) as u8."""
    spp = 4
    acc = np.full((1, 1, 3), lin * spp, np.float32)
    out = rt.write_color(acc, spp)
    assert out[0, 0, 0] == expect


def test_write_color_exposure_and_auto_expose():
    """exposure color.rs:37-39 and auto_expose render.rs:325-339."""
    acc = np.full((2, 2, 3), 2.0, np.float32)
    spp = 1
    lum = 0.2126 * 2 + 0.71516 * 2 + 0.072169 * 2
    mp = lum * lum
    assert rt.auto_expose(acc, spp) == pytest.approx(-math.log(0.6) / math.sqrt(mp))
    ev = 0.7
    out = rt.write_color(acc, spp, exposure=ev)
    x = 1 - math.e ** (-ev * 2.0)
    g = 1.055 * x ** (1 / 2.4) - 0.055
    assert out[0, 0, 1] == int(256 * min(g, 0.999))
    assert rt.auto_expose(np.zeros((2, 2, 3), np.float32), 1) == 1.0


def test_write_ppm_format(tmp_path):
    """render.rs:151 header + one 'r g b' line per pixel, row-major."""
    rgb = np.arange(2 * 3 * 3, dtype=np.uint8).reshape(2, 3, 3)
    p = tmp_path / "x.ppm"
    rt.write_ppm(p, rgb)
    lines = p.read_text().splitlines()
    assert lines[:3] == ["P3", "3 2", "255"]
    assert lines[3] == "0 1 2" and lines[-1] == "15 16 17" and len(lines) == 3 + 6


def test_presets_all_build():
    for name in ["cornell_box", "cornell_smoke", "final_scene", "quads", "simple_light",
                 "two_spheres", "two_perlin_spheres", "random_balls", "three_spheres", "earth"]:
        blob, cam = rt.preset_blob(name, width=20, spp=4)
        assert blob.slots.size > 16 and cam.image_width == 20
    with pytest.raises(rt.RtError):
        rt.preset_blob("nope")
    with pytest.raises(rt.RtError):
        rt.preset_blob("cornell_box", variant="nope")


def test_scene_graphs_round1_rejected_now_validate():
    """A nested light list and a 10-deep Translate/RotateY chain are valid reference inputs
    (object.rs:57, 66; transform.rs): rt_scene_validate accepts them, an empty nested light list
    is the reference's panic (hittable.rs:120) -> RT_ERR_EMPTY_LIGHTS."""
    sc = rt.Scene(3)
    white = sc.lambertian((0.7, 0.7, 0.7))
    light = sc.diffuse_light((4, 4, 4))
    obj = sc.sphere((0, 0, 0), 1.0, white)
    for k in range(10):
        obj = sc.translate(obj, (0.1, 0, 0)) if k % 2 else sc.rotate_y(obj, 10)
    q = sc.quad((-1, 4, -1), (2, 0, 0), (0, 0, 2), light)
    world = sc.hittable_list(obj, q)
    lights = sc.hittable_list(q, sc.hittable_list(sc.sphere((0, 0, 0), 1.0, white), q))
    assert rt.validate(sc.serialize(world, lights)) == 0
    bad = sc.hittable_list(q, sc.hittable_list())
    with pytest.raises(rt.RtError) as e:
        rt.validate(sc.serialize(world, bad))
    assert e.value.code == rt.RT_ERR_EMPTY_LIGHTS
