"""The Rust crate rust/rt_mi355x (FFI mirrors + blob writer) and its reference-side arms
rust/reference_glue/*.rs, checked without rustc (there is none in this image):

* the crate's #[repr(C)] structs, extern "C" functions and constants are compared with
  include/rt_mi355x.h field by field (names, widths, order), declaration by declaration;
* every arm of the writer (one `// blob: <kind>` section per record kind in the glue files) is
  reduced to its sequence of writer calls and compared with the Python transliteration below;
* the transliteration (BlobWriter, write_blob, record, write_record, write_tables: the same
  method names and call order as the Rust) re-serialises every preset scene from a parsed copy
  of the C++-built blob and must reproduce it (rt_mi355x.h:47-78).

Materials are values in the reference (Material is Clone), so the Rust writer deduplicates them
by their 8-slot record; the C++ builder shares materials by pointer. Both blobs are therefore
compared after replacing each material id by its record (textures by their records, recursively);
the writer's own output must be a fixed point of parse + write.
"""
import re
import struct

import numpy as np
import pytest

import surely_rt as rt

MAGIC = 0x52545343


def f2u(x: float) -> int:
    return struct.unpack("<Q", struct.pack("<d", x))[0]


def u2f(u: int) -> float:
    return struct.unpack("<d", struct.pack("<Q", int(u)))[0]


# ------------------------------------------------------------------ mirror types (field names
# as in the reference: object.rs, hittable.rs, transform.rs, constant_medium.rs, material.rs,
# texture.rs, perlin.rs, rt_image.rs)
class Obj:
    def __init__(self, kind, **kw):
        self.kind = kind
        self.__dict__.update(kw)


class Tex:
    def __init__(self, kind, **kw):
        self.kind = kind
        self.__dict__.update(kw)


class Mat:
    def __init__(self, kind, **kw):
        self.kind = kind
        self.__dict__.update(kw)


# ------------------------------------------------------------------ blob -> mirror objects
def parse(slots: np.ndarray, texels: np.ndarray):
    s = [int(v) for v in slots]
    assert s[0] == MAGIC and s[2] == len(s)
    perlins = []
    for k in range(s[7]):
        b = s[8] + k * (256 * 3 + 256 * 3)
        ranvec = [tuple(u2f(s[b + 3 * i + j]) for j in range(3)) for i in range(256)]
        b += 768
        perm = [[int(np.int64(np.uint64(s[b + 256 * a + i]))) for i in range(256)] for a in range(3)]
        perlins.append(Tex("perlin", ranvec=ranvec, perm_x=perm[0], perm_y=perm[1], perm_z=perm[2]))
    texs = [None] * s[3]
    raw = [s[s[4] + 8 * k: s[4] + 8 * k + 8] for k in range(s[3])]

    def tex(k):
        if texs[k] is None:
            r = raw[k]
            if r[0] == 1:
                texs[k] = Tex("solid", color_value=tuple(u2f(r[1 + j]) for j in range(3)))
            elif r[0] == 2:
                texs[k] = Tex("checker", inv_scale=u2f(r[1]), even=tex(r[2]), odd=tex(r[3]))
            elif r[0] == 3:
                w, h, off = r[1], r[2], r[3]
                texs[k] = Tex("image", image_width=w, image_height=h,
                              image=bytes(texels[off:off + w * h * 3]))
            else:
                texs[k] = Tex("noise", scale=u2f(r[1]), noise=perlins[r[2]])
        return texs[k]

    for k in range(s[3]):
        tex(k)

    def mat(k):  # a fresh value per use (Material is Clone); textures shared (Arc)
        r = s[s[6] + 8 * k: s[6] + 8 * k + 8]
        if r[0] == 2:
            return Mat("metal", albedo=tuple(u2f(r[1 + j]) for j in range(3)), fuzz=u2f(r[4]))
        if r[0] == 3:
            return Mat("dielectric", ir=u2f(r[1]), tint=tuple(u2f(r[2 + j]) for j in range(3)))
        names = {1: ("lambertian", "texture"), 4: ("diffuse_light", "emit"),
                 5: ("isotropic", "albedo")}[r[0]]
        return Mat(names[0], **{names[1]: texs[r[1]]})

    pos = [0]

    def i():
        pos[0] += 1
        return int(np.int64(np.uint64(s[pos[0] - 1])))

    def f():
        pos[0] += 1
        return u2f(s[pos[0] - 1])

    def v3():
        return (f(), f(), f())

    def bbox():
        return tuple(f() for _ in range(6))

    def obj():
        tag = i()
        if tag == 1:
            n = i()
            bb = bbox()
            return Obj("list", objects=[obj() for _ in range(n)], bbox=bb)
        if tag == 2:
            bb = bbox()
            left = obj()
            return Obj("node", left=left, right=obj(), bbox=bb)
        if tag == 3:
            m, moving = mat(i()), i()
            c, r, cv, bb = v3(), f(), v3(), bbox()
            return Obj("sphere", mat=m, center=c, radius=r, center_vec=cv if moving else None,
                       bbox=bb)
        if tag == 4:
            m = mat(i())
            q, u, v, normal, w, d, area, bb = v3(), v3(), v3(), v3(), v3(), f(), f(), bbox()
            return Obj("quad", mat=m, q=q, u=u, v=v, normal=normal, w=w, d=d, area=area, bbox=bb)
        if tag == 5:
            off, bb = v3(), bbox()
            return Obj("translate", offset=off, bbox=bb, object=obj())
        if tag == 6:
            sn, cs, bb = f(), f(), bbox()
            return Obj("rot_y", sin_theta=sn, cos_theta=cs, bbox=bb, object=obj())
        if tag == 7:
            m, nid, bb = mat(i()), f(), bbox()
            return Obj("volume", phase_function=m, neg_inv_density=nid, boundary_bbox=bb,
                       boundary=obj())
        raise AssertionError(f"tag {tag}")

    pos[0] = s[9]
    world = obj()
    lights = None
    if int(np.int64(np.uint64(s[10]))) >= 0:
        pos[0] = s[10]
        lights = obj()
    return world, lights


# ------------------------------------------------------------------ INTEGRATION.md §1.2, in Python
class BlobWriter:
    def __init__(self):
        self.slots = [0] * 16
        self.texels = bytearray()
        self.mats = []
        self.texs = []
        self.tex_ids = {}
        self.perlins = []
        self.perlin_ids = {}

    def f(self, x):
        self.slots.append(f2u(x))

    def i(self, x):
        self.slots.append(int(x) & 0xFFFFFFFFFFFFFFFF)

    def v3(self, v):
        for x in v:
            self.f(x)

    def bbox(self, b):
        for x in b:
            self.f(x)

    @staticmethod
    def serialize(world, lights):
        w = BlobWriter()
        world_off = len(w.slots)
        write_blob(world, w)
        lights_off = -1
        if lights is not None:
            lights_off = len(w.slots)
            write_blob(lights, w)
        tex_off = len(w.slots)
        for t in list(w.texs):
            base = len(w.slots)
            write_record(t, w)
            while len(w.slots) < base + 8:
                w.i(0)
        mat_off = len(w.slots)
        for m in w.mats:
            w.slots.extend(m)
        perlin_off = len(w.slots)
        for p in list(w.perlins):
            write_tables(p, w)
        head = [MAGIC, 1, len(w.slots), len(w.texs), tex_off, len(w.mats), mat_off,
                len(w.perlins), perlin_off, world_off, lights_off & 0xFFFFFFFFFFFFFFFF,
                len(w.texels)]
        w.slots[:12] = head
        return w

    def texture(self, t):
        if id(t) in self.tex_ids:
            return self.tex_ids[id(t)]
        register_children(t, self)
        k = len(self.texs)
        self.tex_ids[id(t)] = k
        self.texs.append(t)
        return k

    def perlin(self, p):
        if id(p) in self.perlin_ids:
            return self.perlin_ids[id(p)]
        k = len(self.perlins)
        self.perlin_ids[id(p)] = k
        self.perlins.append(p)
        return k

    def material(self, m):
        rec = record(m, self)
        if rec in self.mats:
            return self.mats.index(rec)
        self.mats.append(rec)
        return len(self.mats) - 1


def write_blob(o, w):  # Object::write_blob and the per-type impls
    if o.kind == "list":
        w.i(1), w.i(len(o.objects)), w.bbox(o.bbox)
        for c in o.objects:
            write_blob(c, w)
    elif o.kind == "node":
        w.i(2), w.bbox(o.bbox)
        write_blob(o.left, w)
        write_blob(o.right, w)
    elif o.kind == "sphere":
        mat = w.material(o.mat)
        w.i(3), w.i(mat), w.i(o.center_vec is not None)
        w.v3(o.center), w.f(o.radius)
        w.v3(o.center_vec if o.center_vec is not None else (0.0, 0.0, 0.0))
        w.bbox(o.bbox)
    elif o.kind == "quad":
        mat = w.material(o.mat)
        w.i(4), w.i(mat)
        w.v3(o.q), w.v3(o.u), w.v3(o.v), w.v3(o.normal), w.v3(o.w)
        w.f(o.d), w.f(o.area)
        w.bbox(o.bbox)
    elif o.kind == "translate":
        w.i(5), w.v3(o.offset), w.bbox(o.bbox)
        write_blob(o.object, w)
    elif o.kind == "rot_y":
        w.i(6), w.f(o.sin_theta), w.f(o.cos_theta), w.bbox(o.bbox)
        write_blob(o.object, w)
    elif o.kind == "volume":
        mat = w.material(o.phase_function)
        w.i(7), w.i(mat), w.f(o.neg_inv_density)
        w.bbox(o.boundary_bbox)  # self.boundary.bounding_box()
        write_blob(o.boundary, w)
    else:
        raise AssertionError(o.kind)


def record(m, w):  # Material::record
    r = [0] * 8
    if m.kind == "lambertian":
        r[0], r[1] = 1, w.texture(m.texture)
    elif m.kind == "metal":
        r[0], r[1:4], r[4] = 2, [f2u(x) for x in m.albedo], f2u(m.fuzz)
    elif m.kind == "dielectric":
        r[0], r[1], r[2:5] = 3, f2u(m.ir), [f2u(x) for x in m.tint]
    elif m.kind == "diffuse_light":
        r[0], r[1] = 4, w.texture(m.emit)
    else:
        r[0], r[1] = 5, w.texture(m.albedo)
    return r


def register_children(t, w):  # Texture::register_children
    if t.kind == "checker":
        w.texture(t.even)
        w.texture(t.odd)
    elif t.kind == "noise":
        w.perlin(t.noise)


def write_record(t, w):  # Texture::write_record
    if t.kind == "solid":
        w.i(1), w.v3(t.color_value)
    elif t.kind == "checker":
        e, o = w.tex_ids[id(t.even)], w.tex_ids[id(t.odd)]
        w.i(2), w.f(t.inv_scale), w.i(e), w.i(o)
    elif t.kind == "image":
        w.i(3), w.i(t.image_width), w.i(t.image_height), w.i(len(w.texels))
        w.texels.extend(t.image)
    else:
        w.i(4), w.f(t.scale), w.i(w.perlin_ids[id(t.noise)])


def write_tables(p, w):  # Perlin::write_tables
    for v in p.ranvec:
        w.v3(v)
    for perm in (p.perm_x, p.perm_y, p.perm_z):
        for k in perm:
            w.i(k)


# ------------------------------------------------------------------ canonical comparison
def canonical(slots, texels):
    """The object trees with every material id replaced by its record (texture ids by texture
    records, recursively) and the Perlin / image data inlined."""
    tx = np.frombuffer(texels, np.uint8) if isinstance(texels, (bytes, bytearray)) else texels
    world, lights = parse(np.asarray(slots, np.uint64), np.asarray(tx, np.uint8))

    def tex(t):
        if t.kind == "solid":
            return ("solid", t.color_value)
        if t.kind == "checker":
            return ("checker", t.inv_scale, tex(t.even), tex(t.odd))
        if t.kind == "image":
            return ("image", t.image_width, t.image_height, t.image)
        return ("noise", t.scale, tuple(t.noise.ranvec), tuple(t.noise.perm_x),
                tuple(t.noise.perm_y), tuple(t.noise.perm_z))

    def mat(m):
        return tuple((k, tex(v) if isinstance(v, Tex) else v) for k, v in sorted(m.__dict__.items()))

    def obj(o):
        items = []
        for k, v in sorted(o.__dict__.items()):
            if isinstance(v, Obj):
                v = obj(v)
            elif isinstance(v, Mat):
                v = mat(v)
            elif isinstance(v, list):
                v = tuple(obj(c) for c in v)
            items.append((k, v))
        return tuple(items)

    return obj(world), None if lights is None else obj(lights)


PRESETS = ["cornell_box", "cornell_smoke", "final_scene", "quads", "simple_light", "two_spheres",
           "two_perlin_spheres", "random_balls", "three_spheres", "earth", "sun_spheres"]


@pytest.mark.parametrize("name", PRESETS)
def test_rust_serialiser_reproduces_every_preset(name):
    try:
        blob, cam = rt.preset_blob(name, width=32, spp=4)
    except rt.RtError:
        pytest.skip(f"no preset {name}")
    world, lights = parse(blob.slots, blob.texels)
    w = BlobWriter.serialize(world, lights)
    out = np.array(w.slots, dtype=np.uint64)
    assert canonical(out, bytes(w.texels)) == canonical(blob.slots, blob.texels)
    # the blob is accepted by the device library's validator and is a fixed point
    rt.validate(rt.Blob(out, np.frombuffer(bytes(w.texels), np.uint8)))
    w2 = BlobWriter.serialize(*parse(out, np.frombuffer(bytes(w.texels), np.uint8)))
    assert w2.slots == w.slots and bytes(w2.texels) == bytes(w.texels)
    assert len(w.texs) == int(blob.slots[3]) and len(w.perlins) == int(blob.slots[7])


def test_rust_serialiser_image_and_checker_textures():
    """An image texture (texels appended in texture-id order) and a checker of solids."""
    sc = rt.Scene(3)
    img = np.arange(5 * 4 * 3, dtype=np.uint8).reshape(4, 5, 3)
    m1 = sc.lambertian(tex=sc.image_texture(img))
    m2 = sc.lambertian(tex=sc.checker_from_color(0.5, (0.1, 0.2, 0.3), (0.9, 0.8, 0.7)))
    world = sc.hittable_list(sc.sphere((0, 0, 0), 1, m1), sc.quad((-1, -1, -1), (2, 0, 0),
                                                                  (0, 0, 2), m2))
    blob = sc.serialize(world)
    w = BlobWriter.serialize(*parse(blob.slots, blob.texels))
    assert w.slots == [int(v) for v in blob.slots] and bytes(w.texels) == blob.texels.tobytes()


# ------------------------------------------------------------------ the crate's files
from pathlib import Path  # noqa: E402

REPO = Path(__file__).resolve().parent.parent
CRATE = REPO / "rust" / "rt_mi355x"
GLUE = REPO / "rust" / "reference_glue"
HEADER = (REPO / "include" / "rt_mi355x.h").read_text()
FFI = (CRATE / "src" / "ffi.rs").read_text()
C_SIZES = {"int32_t": 4, "uint32_t": 4, "uint64_t": 8, "double": 8, "int": 4}
R_SIZES = {"i32": 4, "u32": 4, "u64": 8, "f64": 8}


def _strip_c_comments(t):
    return re.sub(r"/\*.*?\*/", "", t, flags=re.S)


def c_struct(name):
    body = re.search(rf"typedef struct {name} \{{(.*?)\}} {name};", _strip_c_comments(HEADER), re.S)
    assert body, name
    fields = []
    for decl in body.group(1).split(";"):
        decl = decl.strip()
        if not decl:
            continue
        m = re.match(r"(?:const\s+)?(\w+)\s*(\*?)\s*(\w+)(?:\[(\d+)\])?$", decl)
        assert m, decl
        ty, ptr, fname, n = m.groups()
        fields.append((fname, 8 if ptr else C_SIZES[ty] * int(n or 1)))
    return fields


def rust_struct(name):
    body = re.search(rf"pub struct {name} \{{(.*?)\n\}}", FFI, re.S)
    assert body, name
    fields = []
    for line in body.group(1).splitlines():
        line = re.sub(r"//.*", "", line).strip()
        if not line:
            continue
        m = re.match(r"pub (\w+): (.+?),$", line)
        assert m, line
        fname, ty = m.groups()
        if ty.startswith("*"):
            size = 8
        elif ty.startswith("["):
            t, n = re.match(r"\[(\w+); (\d+)\]", ty).groups()
            size = R_SIZES[t] * int(n)
        else:
            size = R_SIZES[ty]
        fields.append((fname, size))
    return fields


@pytest.mark.parametrize("name", ["rt_scene_blob", "rt_camera", "rt_render_opts", "rt_stats"])
def test_crate_structs_mirror_the_header(name):
    assert rust_struct(name) == c_struct(name)


def test_crate_declares_every_entry_point_of_the_header():
    decls = {m.group(2): len([a for a in m.group(3).split(",") if a.strip() not in ("", "void")])
             for m in re.finditer(r"^(int|void|uint64_t|const char\*)\s+(rt_\w+)\((.*?)\);",
                                  _strip_c_comments(HEADER), re.S | re.M)}
    assert len(decls) >= 20
    ext = FFI[FFI.index('extern "C" {'):]
    rust = {m.group(1): len([a for a in m.group(2).split(",") if a.strip()])
            for m in re.finditer(r"pub fn (rt_\w+)\((.*?)\)", ext, re.S)}
    assert rust == decls


def test_crate_constants_match_the_header():
    defs = dict(re.findall(r"#define (RT_\w+) \(?(-?(?:0x)?[0-9a-fA-F]+)u?\)?", HEADER))
    enums = dict(re.findall(r"(RT_(?:OBJ|MAT|TEX)_[A-Z_]+) = (\d+)", HEADER))
    consts = dict(re.findall(r"pub const (RT_\w+): \w+ = (-?(?:0x)?[0-9a-fA-F]+);", FFI))
    assert len(consts) >= 30
    for k, v in consts.items():
        ref = defs.get(k, enums.get(k))
        assert ref is not None, k
        assert int(v, 0) == int(ref, 0), (k, v, ref)


def test_crate_files_are_complete():
    """Cargo.toml, build.rs, src/{lib,ffi,blob}.rs and one glue module per reference module;
    every variant of the reference's Object / Transform / Material / Texture enums has its arm,
    and no arm is elided."""
    for f in ["Cargo.toml", "build.rs", "src/lib.rs", "src/ffi.rs", "src/blob.rs"]:
        assert (CRATE / f).is_file(), f
    cargo = (CRATE / "Cargo.toml").read_text()
    assert re.search(r"^\[dependencies\]\s*$", cargo, re.M) and "links = \"rtmi355x\"" in cargo
    glue = {p.name: p.read_text() for p in GLUE.glob("*.rs")}
    assert set(glue) == {"object_blob.rs", "hittable_blob.rs", "transform_blob.rs",
                         "constant_medium_blob.rs", "material_blob.rs", "texture_blob.rs",
                         "rt_image_blob.rs", "perlin_blob.rs", "render_mi355x.rs"}
    text = "\n".join(glue.values()) + (CRATE / "src" / "blob.rs").read_text()
    for bad in ("todo!", "unimplemented!", "...", "/* elided"):
        assert bad not in re.sub(r"//.*", "", text), bad
    for enum, variants in {"Object": ["List", "Node", "Sphere", "Quad", "Transform", "Volume", "_Plane"],
                           "Transform": ["Translate", "RotY"],
                           "Material": ["Lambertian", "Metal", "Dielectric", "DiffuseLight", "Isotropic"],
                           "Texture": ["Solid", "Checker", "Image", "Noise"]}.items():
        for v in variants:
            assert f"{enum}::{v}" in text, f"{enum}::{v}"


def _loop_spans(body):
    """Character ranges of the `for ... { ... }` blocks of a Rust fragment."""
    spans = []
    for m in re.finditer(r"\bfor\b[^{]*\{", body):
        depth, k = 1, m.end()
        while k < len(body) and depth:
            depth += {"{": 1, "}": -1}.get(body[k], 0)
            k += 1
        spans.append((m.start(), k))
    return spans


def rust_arms():
    """kind -> (the writer calls of its `// blob: kind` section, its tag literal). A call inside
    a `for` loop is marked `*` (once in the text, any number of times at run time)."""
    arms = {}
    for p in GLUE.glob("*.rs"):
        parts = re.split(r"//\s*blob:\s*(\w+)[^\n]*\n", p.read_text())
        for kind, body in zip(parts[1::2], parts[2::2]):
            body = re.split(r"\n\s*\}\s*\n\s*(?:\w+::\w+|impl|fn)", body)[0]
            loops = _loop_spans(body)
            seq = []
            for c in re.finditer(r"w\.(i|f|v3|bbox|material|texture|perlin)\(|(\.write_blob)\(", body):
                name = "child" if c.group(2) else c.group(1)
                seq.append(name + ("*" if any(a <= c.start() < b for a, b in loops) else ""))
            tag = re.search(r"w\.i\((\d+)\)|r\[0\] = (\d+);", body)
            arms[kind] = (seq, int(tag.group(1) or tag.group(2)) if tag else None)
    return arms


def _matches(rust_seq, calls):
    """The run-time calls are the Rust sequence with each `X*` repeated one or more times."""
    pat = "".join(f"(?:{t[:-1]},)+" if t.endswith("*") else f"{t}," for t in rust_seq)
    return re.fullmatch(pat, "".join(c + "," for c in calls)) is not None


class _Trace(BlobWriter):
    """The transliteration's writer, recording its calls (children not descended into)."""

    def __init__(self):
        super().__init__()
        self.calls = []

    def f(self, x):
        self.calls.append("f")
        super().f(x)

    def i(self, x):
        self.calls.append(("i", int(x)))
        super().i(x)

    def v3(self, v):
        self.calls.append("v3")
        for x in v:
            BlobWriter.f(self, x)

    def bbox(self, b):
        self.calls.append("bbox")
        for x in b:
            BlobWriter.f(self, x)

    def material(self, m):
        self.calls.append("material")
        return 0

    def texture(self, t):
        self.calls.append("texture")
        return 0

    def perlin(self, p):
        self.calls.append("perlin")
        return 0


def _trace(fn, obj, **ids):
    w = _Trace()
    w.tex_ids.update(ids.get("tex_ids", {}))
    w.perlin_ids.update(ids.get("perlin_ids", {}))
    global write_blob
    real = write_blob

    def shallow(o, ww):
        if ww is w and o is not obj:
            w.calls.append("child")
        else:
            real(o, ww)
    write_blob = shallow
    try:
        fn(obj, w)
    finally:
        write_blob = real
    tag = next(c[1] for c in w.calls if isinstance(c, tuple))
    return [c[0] if isinstance(c, tuple) else c for c in w.calls], tag


def test_rust_arms_match_the_transliteration():
    arms = rust_arms()
    leaf = Obj("sphere", mat=Mat("lambertian", texture=Tex("solid", color_value=(1, 1, 1))),
               center=(0, 0, 0), radius=1.0, center_vec=None, bbox=(0,) * 6)
    solid = Tex("solid", color_value=(1, 2, 3))
    noise = Tex("noise", scale=4.0, noise=Tex("perlin", ranvec=[(1, 0, 0)] * 256,
                                              perm_x=list(range(256)), perm_y=list(range(256)),
                                              perm_z=list(range(256))))
    cases = {
        "sphere": (write_blob, leaf),
        "quad": (write_blob, Obj("quad", mat=leaf.mat, q=(0, 0, 0), u=(1, 0, 0), v=(0, 1, 0),
                                 normal=(0, 0, 1), w=(0, 0, 1), d=0.0, area=1.0, bbox=(0,) * 6)),
        "list": (write_blob, Obj("list", objects=[leaf], bbox=(0,) * 6)),
        "node": (write_blob, Obj("node", left=leaf, right=leaf, bbox=(0,) * 6)),
        "translate": (write_blob, Obj("translate", offset=(1, 2, 3), bbox=(0,) * 6, object=leaf)),
        "rot_y": (write_blob, Obj("rot_y", sin_theta=0.5, cos_theta=0.8, bbox=(0,) * 6, object=leaf)),
        "volume": (write_blob, Obj("volume", phase_function=Mat("isotropic", albedo=solid),
                                   neg_inv_density=-2.0, boundary_bbox=(0,) * 6, boundary=leaf)),
        "solid": (write_record, solid),
        "checker": (write_record, Tex("checker", inv_scale=2.0, even=solid, odd=solid)),
        "image": (write_record, Tex("image", image_width=2, image_height=1, image=bytes(6))),
        "noise": (write_record, noise),
        "perlin": (write_tables, noise.noise),
    }
    ids = {"tex_ids": {id(solid): 0}, "perlin_ids": {id(noise.noise): 0}}
    for kind, (fn, obj) in cases.items():
        assert kind in arms, f"no `// blob: {kind}` arm in rust/reference_glue"
        seq, tag = _trace(fn, obj, **ids) if kind != "perlin" else (["v3"] * 256 + ["i"] * 768, 0)
        rseq, rtag = arms[kind]
        assert _matches(rseq, seq), (kind, rseq, seq)
        if kind != "perlin":
            assert rtag == tag, (kind, rtag, tag)
    mats = {"lambertian": 1, "metal": 2, "dielectric": 3, "diffuse_light": 4, "isotropic": 5}
    for kind, code in mats.items():
        rseq, rtag = arms[kind]
        assert rtag == code, kind
        assert rseq == (["texture"] if code in (1, 4, 5) else []), (kind, rseq)


def test_crate_gather_module_mirrors_rt_gather_h():
    """src/gather.rs declares every entry point of include/rt_gather.h with its arity, behind the
    "rccl-gather" feature that build.rs turns into -lrtgather."""
    header = _strip_c_comments((REPO / "include" / "rt_gather.h").read_text())
    decls = {m.group(2): len([a for a in m.group(3).split(",") if a.strip() not in ("", "void")])
             for m in re.finditer(r"^(int|void|const char\*)\s+(rt_gather_\w+)\((.*?)\);",
                                  header, re.S | re.M)}
    assert len(decls) == 8
    src = (CRATE / "src" / "gather.rs").read_text()
    ext = src[src.index('extern "C" {'):src.index("\n}\n", src.index('extern "C" {'))]
    rust = {m.group(1): len([a for a in m.group(2).split(",") if a.strip()])
            for m in re.finditer(r"pub fn (rt_gather_\w+)\((.*?)\)", ext, re.S)}
    assert rust == decls
    idb = re.search(r"#define RT_GATHER_ID_BYTES (\d+)", header).group(1)
    assert f"pub const RT_GATHER_ID_BYTES: usize = {idb};" in src
    assert '#[link(name = "rtgather")]' in src
    assert 'rccl-gather = []' in (CRATE / "Cargo.toml").read_text()
    assert "CARGO_FEATURE_RCCL_GATHER" in (CRATE / "build.rs").read_text()
    assert '#[cfg(feature = "rccl-gather")]\npub mod gather;' in (CRATE / "src" / "lib.rs").read_text()
