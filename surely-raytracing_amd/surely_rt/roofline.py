"""Algorithmic work of the render loop, from deterministic op counters.

Flops per sample are path- and scene-dependent, so they are COUNTED, not assumed: the device
(RT_FLAG_COUNT_OPS build) and the CPU oracle count the same primitive-test stages, and this
committed table converts counts to f64 flops. Convention: add/sub/mul = 1,
fma = 2, div/sqrt/transcendental = 1, compares free. The table was fixed before the first
measurement and is not tuned to results. Costs follow the reference's formulas:

  quad      object.rs:453-490   dot(n,d) 5 | +t: dot(n,o) 5, sub, div = 7 | +planar coords:
                                 p = o + t d 6, p-q 3, 2 x (cross 9 + dot 5) = 37
  sphere    object.rs:145-184   oc 3, 3 dots 15, c 2, disc 3 = 23 | roots: sqrt + 2x(sub, div) = 5
  aabb      object.rs:340-370   3 axes x (2 sub + 2 mul) = 12
  translate transform.rs:59     3;   rotate_y transform.rs:86-107: 12
  hit rec   hittable.rs:22-37   p 6, frame replay <= 12, normal 8, back-transform <= 14 = 40
  lambert.  material.rs:92-108, onb.rs:32-47, pdf.rs:69-73, render.rs:279-290
            ONB 38 + unit(dir) 10 + 2 pdf dots 12 + mixture 3 + weight 7 = 70
  cosine    vec3.rs:240-250     sin, cos, 3 sqrt... 2 + 3 + 4 + ONB local 15 = 24
  light gen object.rs:122-132, 503-506  mean of quad (15) and sphere (ONB 38 + 20 + local 15)
  light pdf quad object.rs:492-501 (beyond its quad test): 12;  sphere 190-202: 16
  dielectric material.rs:156-191 unit 10, cos 6, sqrt 3, ratio 1, Schlick 8, reflect/refract 20 = 48
  metal     material.rs:124-134 unit 10, reflect 13, random_unit_vector ~31, unit 10, fma 6 = 70
  isotropic material.rs:241-248 random_unit_vector ~31 + mixture 3 + weight 7 = 41
  volume draw constant_medium.rs:60-78: length 6, ln 1, 5 arithmetic = 12
  noise     texture.rs:127-130 + perlin.rs:30-96: 7 octaves x 150 + sin = 1051
  camera    render.rs:218-249   pixel centre 12, jitter 4, offset 9, direction 3 = 28
Logical scene-fetch bytes (north star "HBM GB/s on BVH traversal"): bytes of the f64 node
records each stage reads (rt_layout.h), plus the framebuffer partials.
"""
FLOPS = {
    "samples": 28,
    "world_queries": 0,
    "quad_tests": 5,
    "quad_plane": 7,
    "quad_interval": 37,
    "quad_hits": 0,
    "sphere_tests": 23,
    "sphere_roots": 5,
    "sphere_hits": 0,
    "aabb_tests": 12,
    "translate": 3,
    "rotate_y": 12,
    "volume_tests": 0,
    "volume_draws": 12,
    "misses": 6,
    "emissive_hits": 6 + 40,
    "lambertian": 70 + 40,
    "metal": 70 + 40,
    "dielectric": 48 + 40,
    "isotropic": 41 + 40,
    "light_pdf_quad": 12,
    "light_pdf_sphere": 16,
    "light_gen": 45,
    "cosine_gen": 24,
    "noise_evals": 1051,
    "depth_cutoff": 0,
}

# bytes read from the scene per counted event (f64 node records, rt_layout.h)
BYTES = {
    "quad_tests": 16 + 32,        # header + n.xy, n.z/D
    "quad_interval": 128,         # q, w, u, v
    "sphere_tests": 16 + 32,      # header + c, r (+ cvec when moving, not counted)
    "aabb_tests": 64,
    "translate": 64,
    "rotate_y": 64,
    "world_queries": 16,          # END node
    "lambertian": 48 + 48,        # material + texture records
    "dielectric": 48,
    "metal": 48,
    "isotropic": 48 + 48,
    "emissive_hits": 48 + 48,
    "noise_evals": 7 * 8 * (32 + 3),
}


def flops(ops: dict) -> float:
    return float(sum(FLOPS.get(k, 0) * v for k, v in ops.items()))


def scene_bytes(ops: dict, partial_bytes: int = 0) -> float:
    return float(sum(BYTES.get(k, 0) * v for k, v in ops.items()) + partial_bytes)


# MI355X peaks (/opt/skills/guides/MI355X_MICROARCH.md, chip-level parameters; spec values)
PEAK_FP64_VECTOR_TFLOPS = 78.6   # FP64 vector (half the 157.3 TF FP32 vector rate)
PEAK_FP32_VECTOR_TFLOPS = 157.3
PEAK_HBM_GBPS = 8000.0


# The sources that determine rt_trace's machine code (ahead-of-time and scene-specialised). A PMC
# traffic profile (profiles/pmc_traffic_<config>.json) records this hash; bench.py uses the
# profile's bytes only while the hash matches the tree it runs from.
KERNEL_SOURCES = ("rt_kernel.h", "rt_layout.h", "rt_rng.h", "rt_device.hip", "rt_jit.cpp",
                  "rt_flatten.cpp", "rt_obvh.cpp")


def kernel_source_sha16() -> str:
    import hashlib
    from pathlib import Path

    csrc = Path(__file__).resolve().parent.parent / "csrc"
    h = hashlib.sha256()
    for name in KERNEL_SOURCES:
        h.update(name.encode())
        h.update((csrc / name).read_bytes())
    return h.hexdigest()[:16]
