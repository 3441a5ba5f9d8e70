"""Scene-specialised kernels (rt_jit.cpp) on the host: the generator emits a walker for every
preset scene (BVH subtrees become calls of the per-lane walker), hiprtc compiles it for gfx950
(no device needed),
and the walker visits the records in the interpreter's order with the records' exact constants."""
import re
import struct

import pytest

import surely_rt as rt

PRESETS = ["cornell_box", "cornell_smoke", "final_scene", "quads", "simple_light", "two_spheres",
           "two_perlin_spheres", "random_balls", "three_spheres", "earth"]


@pytest.mark.parametrize("name", PRESETS)
def test_generated_walker_compiles(name):
    blob, cam = rt.preset_blob(name, width=32, spp=4)
    state, msg = rt.jit_check(blob)
    assert state == 1, msg
    assert "struct TravGen" in msg
    # a BVH subtree record hands its [root, skip) range to the per-lane walker
    n_calls = len(re.findall(r"bvh_subtree<true, COUNT, VOLB, BVH>", msg))
    assert (n_calls > 0) == (rt.layout_stats(blob)["bvh_records"] > 0)


def test_final_scene_walker_bvh_calls():
    """final_scene (main.rs:603-709): the ground-box BVH at the world frame, the light quad, and
    the sphere-cluster BVH inside Translate(RotateY(...)) with that instance frame."""
    blob, cam = rt.preset_blob("final_scene", width=32, spp=4)
    state, src = rt.jit_check(blob)
    assert state == 1, src
    calls = re.findall(r"bvh_subtree<true, COUNT, VOLB, BVH>\(P, (\d+)u, (\d+)u, (\d+)u, ro, rd, tm, "
                       r"o, d, (-?\d+),", src)
    assert len(calls) == 2
    assert calls[0][3] == "-1" and calls[1][3] != "-1"
    # the subtree's skip is the record the generated walk continues with; both subtrees (boxes,
    # spheres) have an ordered BVH (rt_obvh.cpp), appended after the records
    for root, skip, obvh, _ in calls:
        assert int(skip) > int(root) and int(obvh) > int(skip)
    assert src.index("translate_in") < src.index("rotate_y_in") < src.index(f"P, {calls[1][0]}u")


def test_cornell_walker_sequence():
    """cornell_box (main.rs:417-494): the six wall/light quads, Translate + RotateY into the box
    frame, its six faces, EXIT to the world frame, the glass sphere; constants as exact literals."""
    blob, cam = rt.preset_blob("cornell_box", width=32, spp=4)
    state, src = rt.jit_check(blob)
    assert state == 1
    world = src[:src.index("void frame_in")]
    calls = re.findall(r"(aquad_test<COUNT, \d>|quad_test<COUNT>|sphere_test_v<COUNT>|translate_in|"
                       r"rotate_y_in|o = ro;)", world)
    assert calls[:6] == ["aquad_test<COUNT, 0>"] * 2 + ["aquad_test<COUNT, 1>"] * 3 + ["aquad_test<COUNT, 2>"]
    assert calls[6:8] == ["translate_in", "rotate_y_in"]
    assert len(calls) == 6 + 2 + 6 + 1 + 1 and calls[14] == "o = ro;" and calls[15] == "sphere_test_v<COUNT>"
    # the sphere's radius 90 and the box offset (265, 0, 295) appear bit-exact (hex floats)
    assert "(0x1.68p+6)" in src and "(0x1.09p+8), (0x0p+0), (0x1.27p+8)" in src
    lits = [float.fromhex(x) for x in re.findall(r"\((-?0x[0-9a-f.]+p[+-]\d+)\)", src)]
    assert all(struct.pack("<d", v) == struct.pack("<d", float.fromhex(v.hex())) for v in lits)
    # rcp of each axis formed once per frame: 3 in the world frame, x and z in the box frame
    # (RotateY leaves d.y as it is, the translation all of d)
    assert len(re.findall(r"r[xyz] = rcp_nr1", world)) == 5
    assert len(re.findall(r"ry = rcp_nr1", world)) == 1
    # the hit record's frame (transform.rs:57-135) for the box: the same chain with the same
    # literals, into the frame root first and back out innermost first; no interpreter fallback
    fin = src[src.index("void frame_in"):src.index("void frame_out")]
    fout = src[src.index("void frame_out"):src.index("lights_pdf")]
    box = "(0x1.09p+8), (0x0p+0), (0x1.27p+8)"
    assert "hf == 308" in fin and fin.index("translate_in(mk(" + box) < fin.index("rotate_y_in(")
    assert "hf == 308" in fout and fout.index("rotate_y_out(") < fout.index("translate_out(mk(" + box)
    assert "frame_ray" not in fin and "rtk::frame_out" not in fout


def test_cornell_lights_pdf_unrolled():
    """The mixture's light-list PDF (cornell_box lights = [light quad, glass sphere],
    main.rs:485-494): the quad's axis-aligned test at t_min 0.001 and its area, the sphere's
    root-free predicate with cos_theta_max shared from the shading block (first sphere light),
    and the 1/len weight of HittableList::pdf_value (hittable.rs:116) as a literal."""
    blob, cam = rt.preset_blob("cornell_box", width=32, spp=4)
    state, src = rt.jit_check(blob)
    assert state == 1
    lp = src[src.index("lights_pdf"):]
    assert lp.count("// light ") == 2
    assert "aquad_test<COUNT, 1>" in lp and "0.001, kInf" in lp
    assert "(0x1.aa9p+13)" in lp  # light area 130 x 105 = 13650
    assert "cos_max = cos_sl0;" in lp
    assert "return sum * (wt)(0x1p-1);" in lp  # radiance weights in f32 (rt_kernel.h wt)
    assert "quad_light_w(dir, t, " in lp and "sphere_light_w(cos_max)" in lp
    # a scene without lights: the value is never used (have_lights false), the function is 0
    blob, cam = rt.preset_blob("random_balls", width=32, spp=4)
    state, src = rt.jit_check(blob)
    assert state == 1 and "// light " not in src[src.index("lights_pdf"):]


def test_volume_boundary_queries_generated():
    """ConstantMedium records (constant_medium.rs:41-95) with a one-walk boundary get a generated
    two-smallest-candidates query: cornell_smoke's two boxes (main.rs:514-598) as Translate +
    RotateY + six axis quads each, final_scene's two sphere boundaries (main.rs:656-670)."""
    blob, cam = rt.preset_blob("cornell_smoke", width=32, spp=4)
    state, src = rt.jit_check(blob)
    assert state == 1, src
    structs = re.findall(r"struct (VolTwo_\d+) \{", src)
    assert len(structs) == 2
    for name in structs:
        assert f"volume_hit<COUNT, true, BVH, VOLI, {name}>" in src
        body = src[src.index(f"struct {name}"):]
        body = body[:body.index("\n};")]
        assert body.count("aquad_core<") == 6
        assert body.index("translate_in") < body.index("rotate_y_in")
    blob, cam = rt.preset_blob("final_scene", width=32, spp=4)
    state, src = rt.jit_check(blob)
    assert state == 1, src
    structs = re.findall(r"struct (VolTwo_\d+) \{", src)
    assert len(structs) == 2 and all("sqrt_nr(disc)" in src for _ in structs)


def _scene_set(src):
    m = re.search(r"static constexpr uint32_t kScene = 0x([0-9a-f]+)u;", src)
    assert m, "walker without a scene set"
    return int(m.group(1), 16)


# rt_layout.h RTL_SC_*
SC_METAL, SC_DIEL, SC_LIGHT, SC_LIGHTS, SC_LLIST, SC_LSPHERE, SC_LOTHER = (1, 2, 4, 8, 16, 32, 64)


@pytest.mark.parametrize("name,expect", [
    # book3 Cornell box (main.rs:417-494): lambertian walls and box, a light, a glass sphere that
    # is also the second light-list entry
    ("cornell_box", SC_DIEL | SC_LIGHT | SC_LIGHTS | SC_LSPHERE),
    # book2 smoke boxes (main.rs:514-598): no light list (render_par), isotropic media
    ("cornell_smoke", SC_LIGHT),
    # book2 final scene (main.rs:603-712): every material kind, no light list
    ("final_scene", SC_METAL | SC_DIEL | SC_LIGHT),
])
def test_scene_set_of_presets(name, expect):
    """The generated walker's kScene names exactly the material kinds and light-list shapes the
    scene holds (rt_jit.cpp): the path kernel compiles out the shading of everything else, so a
    bit may only be cleared for a case the scene cannot reach."""
    blob, cam = rt.preset_blob(name, width=32, spp=4)
    state, src = rt.jit_check(blob)
    assert state == 1, src
    assert _scene_set(src) == expect


def test_scene_set_diagnostic_keeps_every_case(monkeypatch):
    monkeypatch.setenv("RT_NO_SCENE_SET", "1")
    blob, cam = rt.preset_blob("cornell_box", width=32, spp=4)
    state, src = rt.jit_check(blob)
    assert state == 1 and _scene_set(src) == 0xFFFFFFFF


def test_code_object_cache_round_trip(tmp_path, monkeypatch):
    """rt_jit.cpp's code-object cache (DESIGN §4.1b "Two compilers, one binary"): a compile with
    RT_JIT_CACHE_WRITE=1 stores one object keyed by the generated source, the embedded headers and
    the options; the same scene finds it (nothing rewritten); other options get a key of their own."""
    monkeypatch.setenv("RT_JIT_CACHE_DIR", str(tmp_path))
    monkeypatch.setenv("RT_JIT_CACHE_WRITE", "1")
    monkeypatch.delenv("RT_JIT_OPTS", raising=False)
    blob, _ = rt.preset_blob("cornell_box", width=16, spp=1)
    assert rt.jit_check(blob)[0] == 1
    files = sorted(tmp_path.glob("*.co"))
    assert len(files) == 1 and files[0].stat().st_size > 1000
    stamp = files[0].stat().st_mtime_ns
    assert rt.jit_check(blob)[0] == 1
    assert sorted(tmp_path.glob("*.co")) == files and files[0].stat().st_mtime_ns == stamp
    monkeypatch.setenv("RT_JIT_OPTS", "-DRT_MIN_WAVES_GEN=4")
    assert rt.jit_check(blob)[0] == 1
    assert len(list(tmp_path.glob("*.co"))) == 2
