"""ctypes wrapper of the CPU oracle (oracle/rt_oracle.c). TEST INFRASTRUCTURE ONLY.

Loaded by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg — never by the
product path (surely_rt renders only through librtmi355x.so).
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
ORACLE_BUILD = REPO / "oracle" / "_build"

import sys  # noqa: E402

sys.path.insert(0, str(REPO / "surely-raytracing_amd"))
from surely_rt import RtCamera, RtRenderOpts, RtSceneBlob, OP_NAMES  # noqa: E402

_libs = {}


def lib(precision: int = 32) -> C.CDLL:
    if precision not in _libs:
        path = ORACLE_BUILD / f"liboracle_f{precision}.so"
        if not path.exists():
            raise RuntimeError(f"{path} missing: run `make oracle`")
        L = C.CDLL(str(path))
        L.oracle_render.restype = C.c_int
        L.oracle_render.argtypes = [C.POINTER(RtSceneBlob), C.POINTER(RtCamera),
                                    C.POINTER(RtRenderOpts), C.c_void_p, C.c_void_p, C.c_int]
        L.oracle_rng_draws.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_int, C.c_void_p]
        L.oracle_rng_u32.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_int, C.c_void_p]
        L.oracle_sphere_uv.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
        L.oracle_perlin_turb.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
        L.oracle_light_pdf_batch.restype = C.c_int
        L.oracle_light_pdf_batch.argtypes = [C.POINTER(RtSceneBlob), C.c_void_p, C.c_void_p, C.c_int,
                                             C.c_void_p]
        L.oracle_light_generate.restype = C.c_int
        L.oracle_light_generate.argtypes = [C.POINTER(RtSceneBlob), C.c_void_p, C.c_uint64, C.c_int,
                                            C.c_void_p]
        L.oracle_cosine_dirs.argtypes = [C.c_void_p, C.c_uint64, C.c_int, C.c_void_p]
        L.oracle_fmath.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
        L.oracle_camera_ray.argtypes = [C.POINTER(RtCamera), C.c_uint64, C.c_int, C.c_int,
                                        C.c_int, C.c_int, C.c_void_p]
        L.oracle_world_hit.restype = C.c_int
        L.oracle_world_hit.argtypes = [C.POINTER(RtSceneBlob), C.c_void_p, C.c_double,
                                       C.c_double, C.c_void_p]
        L.oracle_light_pdf.restype = C.c_int
        L.oracle_light_pdf.argtypes = [C.POINTER(RtSceneBlob), C.c_void_p, C.c_void_p,
                                       C.c_void_p]
        L.oracle_precision_bits.restype = C.c_int
        _libs[precision] = L
    return _libs[precision]


def render(blob, cam: RtCamera, opts: RtRenderOpts, precision: int = 64, threads: int | None = None,
           accum: np.ndarray | None = None):
    """oracle_render -> (accum float32 [n_rows, W, 3], op-count dict)."""
    if threads is None:
        try:
            threads = len(os.sched_getaffinity(0))
        except AttributeError:
            threads = os.cpu_count() or 1
        threads = max(1, min(16, threads))  # the GPU box's CPU share is 16 (8 here)
    shape = (opts.n_rows, cam.image_width, 3)
    if accum is None:
        accum = np.zeros(shape, np.float32)
    ops = np.zeros(32, np.uint64)
    rc = lib(precision).oracle_render(blob.ref(), C.byref(cam), C.byref(opts), accum.ctypes.data,
                                      ops.ctypes.data, threads)
    if rc != 0:
        raise RuntimeError(f"oracle_render failed: {rc}")
    return accum, {n: int(ops[i]) for i, n in enumerate(OP_NAMES)}


def rng_draws(seed: int, pixel: int, sample: int, n: int, precision: int = 64) -> np.ndarray:
    """random_double() stream of one pixel-sample (f64 build: 32-bit uniforms)."""
    out = np.zeros(n, np.float64)
    lib(precision).oracle_rng_draws(seed, pixel, sample, n, out.ctypes.data)
    return out


def rng_u32(seed: int, pixel: int, sample: int, n: int) -> np.ndarray:
    out = np.zeros(n, np.uint32)
    lib(64).oracle_rng_u32(seed, pixel, sample, n, out.ctypes.data)
    return out


def sphere_uv(points: np.ndarray, precision: int = 64) -> np.ndarray:
    p = np.ascontiguousarray(points, np.float64).reshape(-1, 3)
    out = np.zeros((p.shape[0], 2), np.float64)
    lib(precision).oracle_sphere_uv(p.ctypes.data, p.shape[0], out.ctypes.data)
    return out


def light_pdf_batch(blob, origin, dirs, precision: int = 64) -> np.ndarray:
    o = np.ascontiguousarray(origin, np.float64)
    d = np.ascontiguousarray(dirs, np.float64).reshape(-1, 3)
    out = np.zeros(d.shape[0], np.float64)
    rc = lib(precision).oracle_light_pdf_batch(blob.ref(), o.ctypes.data, d.ctypes.data, d.shape[0],
                                               out.ctypes.data)
    if rc:
        raise RuntimeError(f"oracle_light_pdf_batch: {rc}")
    return out


def light_generate(blob, origin, n, seed=1, precision: int = 64) -> np.ndarray:
    o = np.ascontiguousarray(origin, np.float64)
    out = np.zeros((n, 3), np.float64)
    rc = lib(precision).oracle_light_generate(blob.ref(), o.ctypes.data, seed, n, out.ctypes.data)
    if rc:
        raise RuntimeError(f"oracle_light_generate: {rc}")
    return out


def cosine_dirs(w, n, seed=1, precision: int = 64) -> np.ndarray:
    ww = np.ascontiguousarray(w, np.float64)
    out = np.zeros((n, 3), np.float64)
    lib(precision).oracle_cosine_dirs(ww.ctypes.data, seed, n, out.ctypes.data)
    return out


FN = {"sin2pi": 0, "cos2pi": 1, "log": 2, "sin": 3, "acos": 4, "atan2": 5}


def fmath(fn: str, x: np.ndarray, y: np.ndarray | None = None) -> np.ndarray:
    x = np.ascontiguousarray(x, np.float32)
    y = np.ascontiguousarray(np.zeros_like(x) if y is None else y, np.float32)
    out = np.zeros_like(x)
    lib(32).oracle_fmath(FN[fn], x.ctypes.data, y.ctypes.data, x.size, out.ctypes.data)
    return out


def camera_ray(cam: RtCamera, seed: int, i: int, j: int, s_i: int, s_j: int,
               precision: int = 64) -> np.ndarray:
    out = np.zeros(7, np.float64)
    lib(precision).oracle_camera_ray(C.byref(cam), seed, i, j, s_i, s_j, out.ctypes.data)
    return out


def world_hit(blob, ray7, tmin=1e-4, tmax=float("inf"), precision: int = 64):
    r = np.ascontiguousarray(ray7, np.float64)
    out = np.zeros(9, np.float64)
    h = lib(precision).oracle_world_hit(blob.ref(), r.ctypes.data, tmin, tmax, out.ctypes.data)
    if h < 0:
        raise RuntimeError("bad blob")
    return out if h else None


def light_pdf(blob, origin, direction, precision: int = 64) -> float:
    o = np.ascontiguousarray(origin, np.float64)
    d = np.ascontiguousarray(direction, np.float64)
    out = C.c_double()
    rc = lib(precision).oracle_light_pdf(blob.ref(), o.ctypes.data, d.ctypes.data, C.byref(out))
    if rc != 0:
        raise RuntimeError(f"oracle_light_pdf: {rc}")
    return out.value
