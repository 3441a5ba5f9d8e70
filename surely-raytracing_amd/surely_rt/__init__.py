"""surely_rt — Python host over the two C ABIs of this repository.

* ``include/rt_host.h``   -> ``build/librthost.so``  : the scene-construction API of the
  reference (Quad, Sphere, make_box, RotateY, Translate, ConstantMedium, HittableList,
  create_bvh, Lambertian, Metal, Dielectric, DiffuseLight, Isotropic, textures, Camera::new,
  write_color) restated in C++ and serialised into the flat scene blob.
* ``include/rt_mi355x.h`` -> ``build/librtmi355x.so`` : the gfx950 render loop behind
  ``rt_render`` (the drop-in for render_par_lights, /root/reference/src/render.rs:144-216).

Nothing here computes pixels: the render path is the HIP library, and it fails loudly (raises)
when that library or a GPU is missing — there is no CPU fallback in the product.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

PKG_DIR = Path(__file__).resolve().parent.parent
REPO = PKG_DIR.parent
BUILD = Path(os.environ.get("RT_BUILD_DIR", REPO / "build"))

# ---------------------------------------------------------------------------- ABI structs
RT_OK = 0
RT_ERR_INVALID_ARG = -1
RT_ERR_BAD_BLOB = -2
RT_ERR_UNSUPPORTED = -3
RT_ERR_EMPTY_LIGHTS = -4
RT_ERR_HIP = -5
RT_ERR_NO_DEVICE = -6

RT_FLAG_OVERWRITE = 0x1
RT_FLAG_COUNT_OPS = 0x2
RT_FLAG_SEMANTICS_REFERENCE = 0x4
RT_FLAG_INTERPRETER = 0x8  # product render with the interpreter walker (no scene-specialised kernel)
RT_FLAG_REFERENCE_BVH = 0x10  # product render walks BVH subtrees in the reference tree and order

OP_NAMES = [
    "samples", "world_queries", "quad_tests", "quad_plane", "quad_interval", "quad_hits",
    "sphere_tests", "sphere_roots", "sphere_hits", "aabb_tests", "translate", "rotate_y",
    "volume_tests", "volume_draws", "misses", "emissive_hits", "lambertian", "metal",
    "dielectric", "isotropic", "light_pdf_quad", "light_pdf_sphere", "light_gen", "cosine_gen",
    "noise_evals", "depth_cutoff",
]


class RtSceneBlob(C.Structure):
    _fields_ = [("slots", C.POINTER(C.c_uint64)), ("n_slots", C.c_uint64),
                ("texels", C.POINTER(C.c_uint8)), ("n_texels", C.c_uint64)]


class RtCamera(C.Structure):
    _fields_ = [("image_width", C.c_int32), ("image_height", C.c_int32),
                ("samples_per_pixel", C.c_int32), ("sqrt_spp", C.c_int32),
                ("max_depth", C.c_int32), ("_pad0", C.c_int32),
                ("recip_sqrt_spp", C.c_double), ("center", C.c_double * 3),
                ("pixel00_loc", C.c_double * 3), ("pixel_delta_u", C.c_double * 3),
                ("pixel_delta_v", C.c_double * 3), ("defocus_angle", C.c_double),
                ("defocus_disk_u", C.c_double * 3), ("defocus_disk_v", C.c_double * 3),
                ("background", C.c_double * 3)]

    def copy(self) -> "RtCamera":
        c = RtCamera()
        C.pointer(c)[0] = self
        return c


class RtRenderOpts(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("row_begin", C.c_int32), ("row_step", C.c_int32),
                ("n_rows", C.c_int32), ("flags", C.c_uint32), ("sj_begin", C.c_int32),
                ("sj_count", C.c_int32), ("device", C.c_int32), ("_pad0", C.c_int32)]


class RtStats(C.Structure):
    _fields_ = [("ms_kernel", C.c_double), ("ms_total", C.c_double), ("samples", C.c_uint64),
                ("ops", C.c_uint64 * 32), ("out_bytes", C.c_uint64), ("launches", C.c_uint32),
                ("_pad0", C.c_uint32)]

    def op_counts(self) -> dict:
        return {n: int(self.ops[i]) for i, n in enumerate(OP_NAMES)}


class RtError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"rt error {code}: {msg}")
        self.code = code


# ---------------------------------------------------------------------------- library loading
_host = None
_dev = None

_D3 = C.c_double * 3


def _d3(v) -> "C.Array":
    return _D3(*[float(x) for x in v])


def host_lib() -> C.CDLL:
    global _host
    if _host is None:
        path = BUILD / "librthost.so"
        if not path.exists():
            raise RuntimeError(f"{path} missing: run `make host` (or __graft_entry__.build())")
        lib = C.CDLL(str(path))
        i32, f64, p = C.c_int32, C.c_double, C.c_void_p
        dp = C.POINTER(C.c_double)
        sig = {
            "rth_last_error": (C.c_char_p, []),
            "rth_scene_new": (p, [C.c_uint64]),
            "rth_scene_free": (None, [p]),
            "rth_random_double": (f64, [p]),
            "rth_random_range": (f64, [p, f64, f64]),
            "rth_random_int": (C.c_int64, [p, C.c_int64, C.c_int64]),
            "rth_solid_color": (i32, [p, f64, f64, f64]),
            "rth_checker_texture": (i32, [p, f64, i32, i32]),
            "rth_noise_texture": (i32, [p, f64]),
            "rth_image_texture": (i32, [p, i32, i32, C.c_void_p]),
            "rth_lambertian": (i32, [p, f64, f64, f64]),
            "rth_lambertian_tex": (i32, [p, i32]),
            "rth_metal": (i32, [p, f64, f64, f64, f64]),
            "rth_dielectric": (i32, [p, f64, f64, f64, f64]),
            "rth_diffuse_light": (i32, [p, f64, f64, f64]),
            "rth_diffuse_light_tex": (i32, [p, i32]),
            "rth_isotropic": (i32, [p, f64, f64, f64]),
            "rth_isotropic_tex": (i32, [p, i32]),
            "rth_sphere": (i32, [p, dp, f64, i32]),
            "rth_sphere_moving": (i32, [p, dp, dp, f64, i32]),
            "rth_quad": (i32, [p, dp, dp, dp, i32]),
            "rth_make_box": (i32, [p, dp, dp, i32]),
            "rth_list_new": (i32, [p]),
            "rth_list_add": (i32, [p, i32, i32]),
            "rth_list_create_bvh": (i32, [p, i32]),
            "rth_list_len": (i32, [p, i32]),
            "rth_translate": (i32, [p, i32, dp]),
            "rth_rotate_y": (i32, [p, i32, f64]),
            "rth_constant_medium": (i32, [p, i32, f64, f64, f64, f64]),
            "rth_constant_medium_tex": (i32, [p, i32, f64, i32]),
            "rth_object_bbox": (C.c_int, [p, i32, dp]),
            "rth_serialize": (C.c_int, [p, i32, i32, C.POINTER(RtSceneBlob)]),
            "rth_camera_new": (C.c_int, [f64, i32, i32, i32, f64, dp, dp, dp, f64, f64, dp,
                                         C.POINTER(RtCamera)]),
            "rth_preset": (C.c_int, [p, C.c_char_p, C.c_char_p, i32, i32, i32, f64,
                                     C.POINTER(i32), C.POINTER(i32), C.POINTER(RtCamera)]),
            "rth_auto_expose": (f64, [C.c_void_p, C.c_int64, i32]),
            "rth_write_color": (C.c_int, [C.c_void_p, C.c_int64, f64, C.c_int, f64, C.c_void_p]),
            "rth_write_ppm": (C.c_int, [C.c_char_p, C.c_void_p, i32, i32]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _host = lib
    return _host


def device_lib() -> C.CDLL:
    """The product library. Raises if it is not built: there is no CPU fallback."""
    global _dev
    if _dev is None:
        _dev = load_device_lib(BUILD / "librtmi355x.so")
    return _dev


def load_device_lib(path: Path) -> C.CDLL:
    path = Path(path)
    if not path.exists():
        raise RuntimeError(f"{path} missing: the HIP library is required (run `make device`)")
    lib = C.CDLL(str(path))
    p = C.c_void_p
    sig = {
        "rt_abi_version": (C.c_int, []),
        "rt_last_error": (C.c_char_p, []),
        "rt_device_count": (C.c_int, [C.POINTER(C.c_int)]),
        "rt_scene_validate": (C.c_int, [C.POINTER(RtSceneBlob)]),
        "rt_scene_create": (C.c_int, [C.POINTER(RtSceneBlob), C.c_int, C.POINTER(p)]),
        "rt_scene_destroy": (None, [p]),
        "rt_scene_device_bytes": (C.c_uint64, [p]),
        "rt_render": (C.c_int, [p, C.POINTER(RtCamera), C.POINTER(RtRenderOpts), C.c_void_p,
                                C.POINTER(RtStats)]),
        "rt_render_device": (C.c_int, [p, C.POINTER(RtCamera), C.POINTER(RtRenderOpts),
                                       C.c_void_p, C.c_void_p, C.POINTER(RtStats)]),
        "rt_render_blob": (C.c_int, [C.POINTER(RtSceneBlob), C.POINTER(RtCamera),
                                     C.POINTER(RtRenderOpts), C.c_void_p,
                                     C.POINTER(RtStats)]),
        "rt_scene_layout_stats": (C.c_int, [C.POINTER(RtSceneBlob), C.POINTER(C.c_uint32),
                                            C.c_int]),
        "rt_scene_prof_counters": (C.c_int, [p, C.POINTER(C.c_uint64), C.c_int]),
        "rt_render_multi": (C.c_int, [C.POINTER(RtSceneBlob), C.POINTER(RtCamera),
                                      C.POINTER(RtRenderOpts), C.POINTER(C.c_int), C.c_int,
                                      C.c_void_p, C.POINTER(RtStats)]),
        "rt_scene_trace_ms": (C.c_int, [p, C.POINTER(C.c_float), C.c_int,
                                        C.POINTER(C.c_int)]),
        "rt_scene_jit_info": (C.c_int, [p, C.POINTER(C.c_int), C.c_char_p, C.c_uint32]),
        "rt_multi_create": (C.c_int, [C.POINTER(RtSceneBlob), C.POINTER(C.c_int), C.c_int,
                                      C.POINTER(p)]),
        "rt_multi_render": (C.c_int, [p, C.POINTER(RtCamera), C.POINTER(RtRenderOpts), C.c_void_p,
                                      C.c_void_p, C.POINTER(RtStats)]),
        "rt_multi_info": (C.c_int, [p, C.POINTER(C.c_uint64), C.c_int]),
        "rt_multi_destroy": (None, [p]),
        "rt_jit_check": (C.c_int, [C.POINTER(RtSceneBlob), C.c_char_p, C.POINTER(C.c_int),
                                   C.c_char_p, C.c_uint32]),
        "rt_scene_lds_check": (C.c_int, [C.POINTER(RtSceneBlob), C.c_uint32, C.c_uint32,
                                         C.c_uint64, C.POINTER(C.c_uint64), C.c_int, C.c_char_p,
                                         C.c_uint32]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.rt_abi_version() != 3:
        raise RuntimeError("librtmi355x ABI version mismatch")
    return lib


def _check_host(rc: int) -> int:
    if rc < 0:
        raise RtError(rc, host_lib().rth_last_error().decode())
    return rc


def _check_dev(rc: int) -> int:
    if rc != RT_OK:
        raise RtError(rc, device_lib().rt_last_error().decode())
    return rc


# ---------------------------------------------------------------------------- scene blob
class Blob:
    """Owns a copy of the serialised scene (rt_scene_blob) and exposes the C view."""

    def __init__(self, slots: np.ndarray, texels: np.ndarray):
        self.slots = np.ascontiguousarray(slots, dtype=np.uint64)
        self.texels = np.ascontiguousarray(texels, dtype=np.uint8)
        self._c = RtSceneBlob()
        self._c.slots = self.slots.ctypes.data_as(C.POINTER(C.c_uint64))
        self._c.n_slots = self.slots.size
        self._c.texels = (self.texels.ctypes.data_as(C.POINTER(C.c_uint8))
                          if self.texels.size else C.POINTER(C.c_uint8)())
        self._c.n_texels = self.texels.size

    @property
    def c(self) -> RtSceneBlob:
        return self._c

    def ref(self):
        return C.byref(self._c)

    def header(self) -> dict:
        s = self.slots
        return dict(n_slots=int(s[2]), n_textures=int(s[3]), n_materials=int(s[5]),
                    n_perlin=int(s[7]), world_off=int(s[9]),
                    lights_off=int(np.int64(s[10].view(np.int64))))


class Scene:
    """Reference-named scene construction (main.rs vocabulary) over librthost.

    Ids returned are handles: textures, materials and objects live in separate id spaces.
    """

    def __init__(self, build_seed: int = 1):
        self._lib = host_lib()
        self._h = self._lib.rth_scene_new(C.c_uint64(build_seed))

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h:
            self._lib.rth_scene_free(h)

    # utils.rs
    def random_double(self) -> float:
        return self._lib.rth_random_double(self._h)

    def random_range(self, a: float, b: float) -> float:
        return self._lib.rth_random_range(self._h, a, b)

    def random_int(self, a: int, b: int) -> int:
        return self._lib.rth_random_int(self._h, a, b)

    # texture.rs
    def solid_color(self, rgb) -> int:
        return _check_host(self._lib.rth_solid_color(self._h, *map(float, rgb)))

    def checker_texture(self, scale: float, even: int, odd: int) -> int:
        return _check_host(self._lib.rth_checker_texture(self._h, scale, even, odd))

    def checker_from_color(self, scale: float, c1, c2) -> int:
        return self.checker_texture(scale, self.solid_color(c1), self.solid_color(c2))

    def noise_texture(self, scale: float) -> int:
        return _check_host(self._lib.rth_noise_texture(self._h, scale))

    def image_texture(self, rgb8: np.ndarray | None) -> int:
        if rgb8 is None:
            return _check_host(self._lib.rth_image_texture(self._h, 0, 0, None))
        a = np.ascontiguousarray(rgb8, dtype=np.uint8)
        h, w = a.shape[:2]
        return _check_host(self._lib.rth_image_texture(self._h, w, h, a.ctypes.data))

    # material.rs
    def lambertian(self, rgb=None, tex: int | None = None) -> int:
        if tex is not None:
            return _check_host(self._lib.rth_lambertian_tex(self._h, tex))
        return _check_host(self._lib.rth_lambertian(self._h, *map(float, rgb)))

    def metal(self, rgb, fuzz: float) -> int:
        return _check_host(self._lib.rth_metal(self._h, *map(float, rgb), fuzz))

    def dielectric(self, ir: float, tint=(1.0, 1.0, 1.0)) -> int:
        return _check_host(self._lib.rth_dielectric(self._h, ir, *map(float, tint)))

    def diffuse_light(self, rgb=None, tex: int | None = None) -> int:
        if tex is not None:
            return _check_host(self._lib.rth_diffuse_light_tex(self._h, tex))
        return _check_host(self._lib.rth_diffuse_light(self._h, *map(float, rgb)))

    def isotropic(self, rgb=None, tex: int | None = None) -> int:
        if tex is not None:
            return _check_host(self._lib.rth_isotropic_tex(self._h, tex))
        return _check_host(self._lib.rth_isotropic(self._h, *map(float, rgb)))

    # object.rs / hittable.rs / transform.rs / constant_medium.rs
    def sphere(self, center, radius: float, mat: int) -> int:
        return _check_host(self._lib.rth_sphere(self._h, _d3(center), radius, mat))

    def sphere_moving(self, c1, c2, radius: float, mat: int) -> int:
        return _check_host(self._lib.rth_sphere_moving(self._h, _d3(c1), _d3(c2), radius, mat))

    def quad(self, q, u, v, mat: int) -> int:
        return _check_host(self._lib.rth_quad(self._h, _d3(q), _d3(u), _d3(v), mat))

    def make_box(self, a, b, mat: int) -> int:
        return _check_host(self._lib.rth_make_box(self._h, _d3(a), _d3(b), mat))

    def hittable_list(self, *objs: int) -> int:
        lst = _check_host(self._lib.rth_list_new(self._h))
        for o in objs:
            self.add(lst, o)
        return lst

    def add(self, lst: int, obj: int) -> None:
        _check_host(self._lib.rth_list_add(self._h, lst, obj))

    def create_bvh(self, lst: int) -> int:
        return _check_host(self._lib.rth_list_create_bvh(self._h, lst))

    def list_len(self, lst: int) -> int:
        return _check_host(self._lib.rth_list_len(self._h, lst))

    def translate(self, obj: int, offset) -> int:
        return _check_host(self._lib.rth_translate(self._h, obj, _d3(offset)))

    def rotate_y(self, obj: int, angle_deg: float) -> int:
        return _check_host(self._lib.rth_rotate_y(self._h, obj, angle_deg))

    def constant_medium(self, boundary: int, density: float, rgb=None,
                        tex: int | None = None) -> int:
        if tex is not None:
            return _check_host(self._lib.rth_constant_medium_tex(self._h, boundary, density, tex))
        return _check_host(self._lib.rth_constant_medium(self._h, boundary, density,
                                                         *map(float, rgb)))

    def bbox(self, obj: int) -> np.ndarray:
        out = _D3()
        buf = (C.c_double * 6)()
        _check_host(self._lib.rth_object_bbox(self._h, obj, buf))
        del out
        return np.array(buf[:])

    def serialize(self, world: int, lights: int | None = None) -> Blob:
        b = RtSceneBlob()
        _check_host(self._lib.rth_serialize(self._h, world, -1 if lights is None else lights,
                                            C.byref(b)))
        slots = np.ctypeslib.as_array(b.slots, shape=(b.n_slots,)).copy()
        tex = (np.ctypeslib.as_array(b.texels, shape=(b.n_texels,)).copy() if b.n_texels
               else np.zeros(0, np.uint8))
        return Blob(slots, tex)

    def preset(self, name: str, variant: str = "", width: int = 0, spp: int = 0, depth: int = 0,
               aspect: float = 0.0):
        """main.rs scene function -> (world list id, lights id or None, RtCamera)."""
        w, l = C.c_int32(), C.c_int32()
        cam = RtCamera()
        _check_host(self._lib.rth_preset(self._h, name.encode(), variant.encode(), width, spp,
                                         depth, aspect, C.byref(w), C.byref(l), C.byref(cam)))
        return w.value, (None if l.value < 0 else l.value), cam


def camera_new(aspect_ratio, image_width, samples_per_pixel, max_depth, vfov, lookfrom, lookat,
               vup, defocus_angle, focus_dist, background) -> RtCamera:
    """Camera::new (render.rs:62-133)."""
    cam = RtCamera()
    _check_host(host_lib().rth_camera_new(aspect_ratio, image_width, samples_per_pixel,
                                          max_depth, vfov, _d3(lookfrom), _d3(lookat), _d3(vup),
                                          defocus_angle, focus_dist, _d3(background),
                                          C.byref(cam)))
    return cam


def preset_blob(name: str, variant: str = "", width: int = 0, spp: int = 0, depth: int = 0,
                aspect: float = 0.0, build_seed: int = 1):
    """Build a main.rs preset and serialise it: returns (Blob, RtCamera)."""
    sc = Scene(build_seed)
    w, l, cam = sc.preset(name, variant, width, spp, depth, aspect)
    return sc.serialize(w, l), cam


def make_opts(cam: RtCamera, seed: int = 1, row_begin: int = 0, row_step: int = 1,
              n_rows: int | None = None, flags: int = RT_FLAG_OVERWRITE, sj_begin: int = 0,
              sj_count: int = 0, device: int = 0) -> RtRenderOpts:
    o = RtRenderOpts()
    o.seed = seed
    o.row_begin = row_begin
    o.row_step = row_step
    if n_rows is None:
        n_rows = len(range(row_begin, cam.image_height, row_step))
    o.n_rows = n_rows
    o.flags = flags
    o.sj_begin = sj_begin
    o.sj_count = sj_count
    o.device = device
    return o


# ---------------------------------------------------------------------------- device render
class DeviceScene:
    """A flattened scene resident on one GPU (rt_scene_create)."""

    def __init__(self, blob: Blob, device: int = 0):
        self._lib = device_lib()
        self._blob = blob
        h = C.c_void_p()
        _check_dev(self._lib.rt_scene_create(blob.ref(), device, C.byref(h)))
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._lib.rt_scene_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    @property
    def device_bytes(self) -> int:
        return int(self._lib.rt_scene_device_bytes(self._h))

    def render(self, cam: RtCamera, opts: RtRenderOpts, accum: np.ndarray | None = None):
        """Synchronous render into a host float32 (n_rows, W, 3) array; returns (accum, stats)."""
        shape = (opts.n_rows, cam.image_width, 3)
        if accum is None:
            accum = np.zeros(shape, np.float32)
        assert accum.shape == shape and accum.dtype == np.float32 and accum.flags.c_contiguous
        st = RtStats()
        _check_dev(self._lib.rt_render(self._h, C.byref(cam), C.byref(opts), accum.ctypes.data,
                                       C.byref(st)))
        return accum, st

    def render_device(self, cam: RtCamera, opts: RtRenderOpts, dev_ptr: int, stream: int = 0,
                      stats: bool = False):
        """Asynchronous render into a device buffer (e.g. a torch tensor's data_ptr())."""
        st = RtStats() if stats else None
        _check_dev(self._lib.rt_render_device(self._h, C.byref(cam), C.byref(opts),
                                              C.c_void_p(dev_ptr), C.c_void_p(stream or None),
                                              C.byref(st) if st is not None else None))
        return st

    def jit_info(self) -> tuple[int, str]:
        """(state, message) of the scene-specialised kernel: 1 compiled and in use, 0 not compiled
        yet, -1 not generated for this scene, -2 compilation failed (rt_scene_jit_info)."""
        st = C.c_int(0)
        buf = C.create_string_buffer(1 << 16)
        _check_dev(self._lib.rt_scene_jit_info(self._h, C.byref(st), buf, len(buf)))
        return st.value, buf.value.decode(errors="replace")

    def trace_ms(self, n: int) -> list[float]:
        """Device ms of the rt_trace kernel alone for the last n renders (oldest first)."""
        buf = (C.c_float * max(1, n))()
        got = C.c_int(0)
        _check_dev(self._lib.rt_scene_trace_ms(self._h, buf, n, C.byref(got)))
        return [float(buf[i]) for i in range(got.value)]


def render_par_lights(blob: Blob, cam: RtCamera, seed: int = 1, device: int = 0,
                      flags: int = RT_FLAG_OVERWRITE):
    """Drop-in for render_par_lights (render.rs:144-216) minus the PPM side effect:
    returns the raw per-pixel sums (H, W, 3) float32, as the reference's `pixels` vector."""
    ds = DeviceScene(blob, device)
    try:
        accum, st = ds.render(cam, make_opts(cam, seed=seed, flags=flags, device=device))
    finally:
        ds.close()
    return accum, st


LAYOUT_STATS = ["node_words", "bvh_words", "bvh_records", "dup_records", "volumes",
                "volumes_one_walk_sphere", "volumes_one_walk_quads", "lights", "ordered_bvhs",
                "compact_bvhs", "compact_bvh_bytes"]
# rt_scene_lds_check (include/rt_mi355x.h RT_LDS_CHECK)
LDS_CHECK = ["block", "static_lds", "stage_bytes", "cbvh_lds_off", "cbvh_bytes", "stack_lds_off",
             "cbvh_stack", "lds_bytes", "lds_total", "lds_cu", "trees", "max_depth", "errors",
             "max_store_slot", "max_live", "rays", "steps", "max_read", "row_lds_off"]


def render_multi(blob: "Blob", cam: RtCamera, opts: RtRenderOpts, devices,
                 accum: np.ndarray | None = None):
    """rt_render_multi: the call's rows dealt cyclically over `devices` (one process, N GPUs),
    gathered into one host frame. Returns (accum [n_rows, W, 3] float32, RtStats)."""
    devs = (C.c_int * len(devices))(*devices)
    if accum is None:
        accum = np.zeros((opts.n_rows, cam.image_width, 3), np.float32)
    st = RtStats()
    _check_dev(device_lib().rt_render_multi(blob.ref(), C.byref(cam), C.byref(opts), devs,
                                            len(devices), accum.ctypes.data, C.byref(st)))
    return accum, st


class MultiScene:
    """rt_multi_*: the scene resident on several GPUs of one process, frame after frame; rows are
    dealt cyclically and gathered peer to peer into a buffer on devices[0]."""

    def __init__(self, blob: "Blob", devices):
        self._lib = device_lib()
        self._blob = blob
        self.devices = list(devices)
        devs = (C.c_int * len(self.devices))(*self.devices)
        h = C.c_void_p()
        _check_dev(self._lib.rt_multi_create(blob.ref(), devs, len(self.devices), C.byref(h)))
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._lib.rt_multi_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def render_device(self, cam: RtCamera, opts: RtRenderOpts, dev_ptr: int, stream: int = 0,
                      stats: bool = False):
        """Asynchronous frame into a devices[0] buffer (e.g. a torch tensor's data_ptr())."""
        st = RtStats() if stats else None
        _check_dev(self._lib.rt_multi_render(self._h, C.byref(cam), C.byref(opts),
                                             C.c_void_p(dev_ptr), C.c_void_p(stream or None),
                                             C.byref(st) if st is not None else None))
        return st

    def info(self) -> dict:
        out = (C.c_uint64 * 4)()
        _check_dev(self._lib.rt_multi_info(self._h, out, 4))
        return dict(zip(("frames", "uploads", "stage_allocs", "devices"), (int(v) for v in out)))


def validate(blob: "Blob") -> int:
    """rt_scene_validate: RT_OK, or raises RtError with the library's status and message."""
    return _check_dev(device_lib().rt_scene_validate(blob.ref()))


def layout_stats(blob: "Blob") -> dict:
    """Host-only counts of the flattened device layout (rt_scene_layout_stats)."""
    out = (C.c_uint32 * len(LAYOUT_STATS))()
    _check_dev(device_lib().rt_scene_layout_stats(blob.ref(), out, len(LAYOUT_STATS)))
    return dict(zip(LAYOUT_STATS, (int(v) for v in out)))


def lds_check(blob: "Blob", flags: int = 0, n_rays: int = 4096, seed: int = 1) -> dict:
    """Host-only: the product render's LDS plan and a check of the compact BVHs the LDS walk
    reads, with a host restatement of the walk's stack and region addressing over random rays
    (rt_scene_lds_check). `first_error` is empty when every tree is well formed."""
    out = (C.c_uint64 * len(LDS_CHECK))()
    msg = C.create_string_buffer(512)
    _check_dev(device_lib().rt_scene_lds_check(blob.ref(), flags, n_rays, seed, out,
                                               len(LDS_CHECK), msg, len(msg)))
    d = dict(zip(LDS_CHECK, (int(v) for v in out)))
    d["first_error"] = msg.value.decode(errors="replace")
    return d


def jit_check(blob: "Blob", arch: str = "gfx950") -> tuple[int, str]:
    """Host-only: generate the scene-specialised walker for `blob` and compile it with hiprtc
    (rt_jit_check). (1, walker source) | (-1, why not generated); raises on a compile error."""
    st = C.c_int(0)
    buf = C.create_string_buffer(1 << 20)
    _check_dev(device_lib().rt_jit_check(blob.ref(), arch.encode(), C.byref(st), buf, len(buf)))
    return st.value, buf.value.decode(errors="replace")


def device_count() -> int:
    n = C.c_int(0)
    device_lib().rt_device_count(C.byref(n))
    return n.value


# ---------------------------------------------------------------------------- output stage
def write_color(accum: np.ndarray, samples_per_pixel: float,
                exposure: float | None = None) -> np.ndarray:
    """color.rs write_color over a whole frame: raw sums -> sRGB8 (H, W, 3) uint8."""
    a = np.ascontiguousarray(accum, dtype=np.float32)
    out = np.zeros(a.shape, np.uint8)
    n = a.size // 3
    host_lib().rth_write_color(a.ctypes.data, n, float(samples_per_pixel),
                               0 if exposure is None else 1,
                               0.0 if exposure is None else float(exposure), out.ctypes.data)
    return out


def auto_expose(accum: np.ndarray, samples_per_pixel: int) -> float:
    """render.rs:325-339."""
    a = np.ascontiguousarray(accum, dtype=np.float32)
    return host_lib().rth_auto_expose(a.ctypes.data, a.size // 3, int(samples_per_pixel))


def write_ppm(path: str, rgb8: np.ndarray) -> None:
    """P3 text exactly as render.rs:151 + write_color lines."""
    a = np.ascontiguousarray(rgb8, dtype=np.uint8)
    h, w = a.shape[:2]
    _check_host(host_lib().rth_write_ppm(str(path).encode(), a.ctypes.data, w, h))
