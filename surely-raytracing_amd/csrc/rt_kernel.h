// rt_kernel.h — the device side of the path tracer: math, primitives, the scene walkers,
// materials / textures / PDFs and the path-kernel body (trace_body).
//
// Replaces the reference's per-pixel render loop (render.rs:144-216) and everything it calls:
// get_ray (render.rs:218-249), ray_color (render.rs:251-311), HittableList/BvhNode::hit
// (hittable.rs:88-109, 216-236), Quad/Sphere/Aabb::hit (object.rs:145-184, 340-370, 453-490),
// Translate/RotateY::hit (transform.rs:57-135), ConstantMedium::hit (constant_medium.rs:41-95),
// Material scatter (material.rs:92-248), PDFs (pdf.rs:44-127), Onb (onb.rs:24-47), textures
// and Perlin noise (texture.rs:17-131, perlin.rs:30-96), vec3 math (vec3.rs).
//
// Compiled twice: ahead of time into librtmi355x.so (rt_device.hip, interpreter traversal) and
// at scene creation by hiprtc (rt_jit.cpp, traversal generated from the scene). It therefore
// uses only what hiprtc provides: no standard-library headers.
#pragma once
#include "rt_layout.h"
#include "rt_mi355x.h"
#include "rt_rng.h"

namespace rtk {
using namespace rtd;

// The path is computed in f64 like the reference (vec3.rs:21-25 f64 everywhere): its fixed
// epsilons (t_min 1e-4 render.rs:267, 1e-3 light PDFs object.rs:193,493, 1e-8 quad
// parallelism object.rs:457) assume f64 hit points; at fp32 the glass sphere and the ground
// boxes self-intersect. MI355X runs FP64 FMA at half its FP32 rate.
constexpr double kPi = 3.14159265358979323846;
constexpr double kInf = __builtin_inf();
template <bool B, class T, class F>
struct cond {
  typedef T type;
};
template <class T, class F>
struct cond<false, T, F> {
  typedef F type;
};
__device__ __forceinline__ int imin(int a, int b) { return a < b ? a : b; }
constexpr int kWaveTile = 8;  // 8x8 pixels per wave
// Stratum columns s_i per pool: a pool is 8x8 pixels x one stratum row s_j x kPoolSi columns.
// A segment item (one pixel's kPoolSi consecutive samples in one lane) lasts ~kPoolSi paths, so
// the launch drains within a few paths per lane (whole-row items, 31 paths at 961 spp, left an
// 8-GPU share of the C2 frame 13 % idle at the end). A power of two.
#ifndef RT_POOL_SI
#define RT_POOL_SI 8
#endif
constexpr int kPoolSi = RT_POOL_SI;
static_assert((kPoolSi & (kPoolSi - 1)) == 0, "kPoolSi: a power of two");
constexpr int kBlock = 256;   // 4 waves per workgroup
// BVH kernels run three waves per SIMD (MinWaves below: <= 168 VGPRs) in ONE 768-thread
// workgroup per CU, so the workgroup may take (almost) the CU's whole 160 KiB LDS for the BVH
// region (rt_layout.h). final_scene: 416 Msamples/s at 512 threads x 2 waves, 443 at 1024 x 4
// (spilling), 523 at 768 x 3 (tools_gpu/ab_variants.py).
#ifndef RT_BLOCK_BVH
#define RT_BLOCK_BVH 768
#endif
constexpr int kBlockBvh = RT_BLOCK_BVH;
template <bool BVH>
struct BlockOf {
  static constexpr int value = BVH ? kBlockBvh : kBlock;
};
// LDS of one workgroup (gfx950: 160 KiB per CU): static (per-lane running sums, counters) plus
// dynamic (whole small scenes, kStageScene; or the Perlin tables and the BVH region).
constexpr size_t kLdsTotal = 160u << 10;
// Minimum waves per SIMD for the path kernel (__launch_bounds__ 2nd argument). 4 caps the
// allocation at 128 VGPRs. Kernels with a per-lane BVH walker run 3 (168 VGPRs; see kBlockBvh);
// kernels without a BVH stay at 4 (cornell_box at 3 or 5: -13 %; cornell_smoke at 3: -8 %,
// at 5: -12 %). tools_gpu/ab_variants.py.
#ifndef RT_MIN_WAVES
#define RT_MIN_WAVES 4
#endif
#ifndef RT_MIN_WAVES_BVH
#define RT_MIN_WAVES_BVH 3
#endif
// Scene-specialised kernels without a BVH (rt_jit.cpp) carry less code (the scene set, §4.1b
// of DESIGN.md) and run more waves per SIMD: five from round 3 (cornell_smoke 96.65 -> 95.78 ms,
// profiles/r03_ab_occ_*.log). Round 6: the f32 radiance weights took cornell_box to 84 VGPRs;
// at six waves (80, a few cold values spilled) it runs -0.67 %, cornell_smoke (ConstantMedium
// kernels, RT_MIN_WAVES_GEN_VOL) -0.03 %, so those stay at five (profiles/r06e_ab_waves_c{2,3}.log).
#ifndef RT_MIN_WAVES_GEN
#define RT_MIN_WAVES_GEN 6
#endif
#ifndef RT_MIN_WAVES_GEN_VOL
#define RT_MIN_WAVES_GEN_VOL 5
#endif
template <bool VOL, bool TEX, bool BVH, bool GEN = false>
struct MinWaves {
  static constexpr int value =
      BVH ? RT_MIN_WAVES_BVH : (GEN ? (VOL ? RT_MIN_WAVES_GEN_VOL : RT_MIN_WAVES_GEN) : RT_MIN_WAVES);
};

struct d3 {
  double x, y, z;
};
#ifdef RT_EXACT_PROBE  // cost probe (not shipped): unfused products, IEEE division and sqrt
__device__ __forceinline__ double rt_unfused_fma(double a, double b, double c) { return a * b + c; }
#define fma(a, b, c) rt_unfused_fma(a, b, c)
#endif
__device__ __forceinline__ d3 mk(double x, double y, double z) { return {x, y, z}; }
__device__ __forceinline__ d3 operator+(d3 a, d3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ d3 operator-(d3 a, d3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ d3 operator-(d3 a) { return {-a.x, -a.y, -a.z}; }
__device__ __forceinline__ d3 operator*(d3 a, d3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
__device__ __forceinline__ d3 operator*(d3 a, double t) { return {a.x * t, a.y * t, a.z * t}; }
__device__ __forceinline__ d3 operator*(double t, d3 a) { return {a.x * t, a.y * t, a.z * t}; }
// Contraction is OFF for the device build (-ffp-contract=off): every fma below is explicit, so
// an expression computes the same bits in every inlining context. The reference relies on
// that determinism: a sphere that is both a world object and a ConstantMedium boundary
// (main.rs:656-666) must yield the identical t from both tests, or constant_medium.rs:52-55
// draws an extra random number.
__device__ __forceinline__ double dot(d3 u, d3 v) {  // vec3.rs:167
  return fma(u.x, v.x, fma(u.y, v.y, u.z * v.z));
}
__device__ __forceinline__ d3 vfma(double t, d3 a, d3 b) {  // t*a + b
  return {fma(t, a.x, b.x), fma(t, a.y, b.y), fma(t, a.z, b.z)};
}
__device__ __forceinline__ d3 cross(d3 u, d3 v) {  // vec3.rs:171-177
  return {fma(u.y, v.z, -(u.z * v.y)), fma(u.z, v.x, -(u.x * v.z)), fma(u.x, v.y, -(u.y * v.x))};
}
// Geometry-side reciprocal and reciprocal square root: the hardware v_rcp_f64 / v_rsq_f64
// estimate plus two Newton-Raphson steps (quadratic convergence: full f64 accuracy, within an
// ulp of the IEEE quotient, at about half the instructions of the IEEE division / sqrt
// sequences). Used only where the operand is finite and non-zero by construction (quad
// denominators past the 1e-8 test, |d|^2, |v|^2 of non-degenerate vectors); radiance weights
// keep IEEE division so 0/0 stays NaN exactly as in the reference.
#ifdef RT_EXACT_PROBE
__device__ __forceinline__ double rcp_nr(double b) { return 1.0 / b; }
__device__ __forceinline__ double rcp_nr1(double b) { return 1.0 / b; }
__device__ __forceinline__ double div_nr(double a, double b) { return a / b; }
__device__ __forceinline__ double rsq_nr(double x) { return 1.0 / __builtin_sqrt(x); }
__device__ __forceinline__ double rcp_w(double b) { return 1.0 / b; }
__device__ __forceinline__ double sqrt_nr(double x) { return __builtin_sqrt(x); }
#else
__device__ __forceinline__ double rcp_nr(double b) {
  double r = __builtin_amdgcn_rcp(b);
  r = fma(fma(-b, r, 1.0), r, r);
  return fma(fma(-b, r, 1.0), r, r);
}
// The per-batch reciprocal of an axis-aligned quad test: one Newton step. The test's quotient
// is then corrected once more (t = t0 + (num - d t0) r, aquad_core), which is what bounds t to
// an ulp; the second step of rcp_nr would only refine r below that.
__device__ __forceinline__ double rcp_nr1(double b) {
  const double r = __builtin_amdgcn_rcp(b);
  return fma(fma(-b, r, 1.0), r, r);
}
__device__ __forceinline__ double div_nr(double a, double b) {
  double r = rcp_nr(b);
  double q = a * r;
  return fma(fma(-b, q, a), r, q);
}
__device__ __forceinline__ double rsq_nr(double x) {
  double y = __builtin_amdgcn_rsq(x);
  double h = 0.5 * x;
  y = y * fma(-h * y, y, 1.5);
  return y * fma(-h * y, y, 1.5);
}
// Radiance weights only (PDF values, scattering PDF, the throughput factor): 1/b by rcp + two
// Newton steps. Weights never steer a path (directions, hits and draws do), so their last-ulp
// rounding is free to differ from an IEEE quotient (the CPU oracle, which follows the recursive
// (atten*s_pdf*L)/pdf form, already differs there); 1/0 = inf and 1/inf = 0 are kept, so the
// reference's inf/NaN weights (render.rs:289-290) stay inf/NaN.
__device__ __forceinline__ double rcp_w(double b) {
  const double r0 = __builtin_amdgcn_rcp(b);
  double r = fma(fma(-b, r0, 1.0), r0, r0);
  r = fma(fma(-b, r, 1.0), r, r);
  return (r0 == 0.0 || __builtin_isinf(r0)) ? r0 : r;
}
// sqrt from v_rsq_f64 plus one Goldschmidt/Newton refinement of (s, h) = (sqrt x, 1/(2 sqrt x))
// and a final residual correction: within an ulp of the IEEE root (like rsq_nr / div_nr, the
// device's geometry rounding) at about half the library sequence. +-0 and +inf
// return themselves, negative and NaN inputs give NaN, as IEEE sqrt does. Inputs here are
// never subnormal (uniform draws are multiples of 2^-32; squared unit-scale cosines).
__device__ __forceinline__ double sqrt_nr(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  double s = x * y;
  double h = 0.5 * y;
  const double r = fma(-s, h, 0.5);
  s = fma(s, r, s);
  h = fma(h, r, h);
  const double e = fma(-s, s, x);
  s = fma(e, h, s);
  return __builtin_amdgcn_class(x, 0x260) ? x : s;  // +-0, +inf
}
#endif
__device__ __forceinline__ d3 unit_vector(d3 v) {  // vec3.rs:179-181
  return v * rsq_nr(dot(v, v));
}
__device__ __forceinline__ d3 reflect(d3 v, d3 n) {  // vec3.rs:219-221
  return vfma(-2.0 * dot(v, n), n, v);
}
__device__ __forceinline__ d3 refract(d3 uv, d3 n, double e) {  // vec3.rs:223-229
  double c = fmin(dot(-uv, n), 1.0);
  d3 perp = e * vfma(c, n, uv);
  return vfma(-sqrt_nr(fabs(1.0 - dot(perp, perp))), n, perp);
}

// ---------------------------------------------------------------- radiance weights
// Quantities that only weight radiance and never steer a path -- the throughput beta, a bounce's
// factor atten * s_pdf / pdf_val, emission, the background, PDF and scattering-PDF values, the
// light-list PDF after its f64 hit tests -- are computed in f32 (wt / w3). Every ray, hit,
// interval, Schlick / TIR test, random draw and every zero test that selects a branch stays f64,
// so a path takes the same bounces (op counts identical to the f64 oracle's); only the sample's
// radiance carries the f32 roundings (a few 2^-24 relative per bounce). v_fma_f64 issues at half
// the f32 rate, and v_rcp_f32 / v_rsq_f32 (1 ulp) replace f64 reciprocals and roots with their
// Newton steps. RT_F64W (A/B only): the same expressions in f64.
#ifdef RT_F64W
typedef double wt;
typedef d3 w3;
__device__ __forceinline__ w3 mkw(wt x, wt y, wt z) { return mk(x, y, z); }
__device__ __forceinline__ w3 to_w3(d3 v) { return v; }
__device__ __forceinline__ d3 to_d3(w3 v) { return v; }
__device__ __forceinline__ wt rcp_wt(wt b) { return rcp_w(b); }
__device__ __forceinline__ wt rsq_wt(wt x) { return rsq_nr(x); }
#else
typedef float wt;
struct w3 {
  float x, y, z;
};
__device__ __forceinline__ w3 mkw(wt x, wt y, wt z) { return {x, y, z}; }
__device__ __forceinline__ w3 operator*(w3 a, w3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
__device__ __forceinline__ w3 operator*(w3 a, wt t) { return {a.x * t, a.y * t, a.z * t}; }
__device__ __forceinline__ w3 to_w3(d3 v) { return {(float)v.x, (float)v.y, (float)v.z}; }
__device__ __forceinline__ d3 to_d3(w3 v) { return {(double)v.x, (double)v.y, (double)v.z}; }
// 1/b within an ulp; 1/+-0 = +-inf, 1/inf = 0 and NaN stay, as the reference's weights
__device__ __forceinline__ wt rcp_wt(wt b) { return __builtin_amdgcn_rcpf(b); }
__device__ __forceinline__ wt rsq_wt(wt x) { return __builtin_amdgcn_rsqf(x); }
#endif
constexpr wt kInvPiW = (wt)(1.0 / 3.14159265358979323846);

// x^5 correctly rounded, for Schlick's (1 - cos)^5 (material.rs:162 calls powf(5.), i.e. the
// platform pow). x^2 is formed exactly as a double-double (a + ae), squared and multiplied by x
// in double-double (relative error ~2^-104), then rounded once: the IEEE-rounded x^5 except
// for exact values within ~2^-104 of a rounding midpoint (dielectric bounces only).
__device__ __forceinline__ double pow5_cr(double x) {
  const double a = x * x, ae = fma(x, x, -a);
  const double b = a * a, be = fma(a, a, -b) + (2.0 * a) * ae;
  const double c = b * x, ce = fma(b, x, -c) + be * x;
  return c + ce;
}

// An f64 constant materialised at its point of use: two s_mov_b32 into an SGPR pair, which the
// fma reads directly. The compiler otherwise hoists literal constants out of the path loop into
// VGPR pairs and, short of registers, spills them (final_scene: 12 of the 24 spilled VGPRs were
// sincos2pi's coefficients); volatile asm is not hoisted.
template <uint64_t B>
__device__ __forceinline__ double kd_bits() {
  uint32_t lo, hi;
  asm volatile("s_mov_b32 %0, %1" : "=s"(lo) : "i"((uint32_t)B));
  asm volatile("s_mov_b32 %0, %1" : "=s"(hi) : "i"((uint32_t)(B >> 32)));
  return __builtin_bit_cast(double, (uint64_t)hi << 32 | lo);
}
#define KD(x) kd_bits<__builtin_bit_cast(uint64_t, (double)(x))>()

// fma(a, b, K) with the f64 constant K in an SGPR pair (v_fma_f64 reads it there): written
// in asm because the compiler otherwise forms v_fmac_f64, whose addend is tied to the
// destination, and copies each constant into a VGPR pair first (3 instructions per step).
template <uint64_t B>
__device__ __forceinline__ double fma_k(double a, double b) {
  double r;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(__builtin_bit_cast(double, B)));
  return r;
}

// sin(2*pi*u), cos(2*pi*u) for u in [0, 1) (vec3.rs:244, object.rs:127: phi = 2*pi*r1).
// Exact reduction to a quarter-turn fraction r in [-1/2, 1/2], then near-minimax polynomials of
// theta = r*pi/2 (|theta| <= pi/4) evaluated with fused Horner steps: sin = th + th^3 P(th^2)
// (degree 13), cos = 1 - th^2/2 + th^4 Q(th^2) (degree 14). Relative least-squares fits in 200-bit
// arithmetic, coefficients rounded to f64 (tools_gpu/fit_sincos.py): measured max error 0.70 ulp
// (sin) and 0.83 ulp (cos) against the exact values, like the libm result within an ulp, at
// 15 f64 operations instead of the 40 of an unfused Taylor series; none of the large-argument
// machinery of the general sincos.
__device__ __forceinline__ void sincos2pi(double u, double* so, double* co) {
  double t = 4.0 * u;
  double k = floor(t + 0.5);
  double th = (t - k) * (0.5 * kPi);
  double x2 = th * th;
  double s = 0x1.5e0a1f55525f5p-33;
  s = fma_k<__builtin_bit_cast(uint64_t, (double)(-0x1.ae6007fd13afdp-26))>(s, x2);
  s = fma_k<__builtin_bit_cast(uint64_t, (double)(0x1.71de379346184p-19))>(s, x2);
  s = fma_k<__builtin_bit_cast(uint64_t, (double)(-0x1.a01a019e80c94p-13))>(s, x2);
  s = fma_k<__builtin_bit_cast(uint64_t, (double)(0x1.1111111110ba4p-7))>(s, x2);
  s = fma_k<__builtin_bit_cast(uint64_t, (double)(-0x1.5555555555555p-3))>(s, x2);
  s = fma(th * x2, s, th);
  double c = -0x1.907cfe8bc9784p-37;
  c = fma_k<__builtin_bit_cast(uint64_t, (double)(0x1.1eeb67eadb724p-29))>(c, x2);
  c = fma_k<__builtin_bit_cast(uint64_t, (double)(-0x1.27e4fa16c73f4p-22))>(c, x2);
  c = fma_k<__builtin_bit_cast(uint64_t, (double)(0x1.a01a019f4dbdbp-16))>(c, x2);
  c = fma_k<__builtin_bit_cast(uint64_t, (double)(-0x1.6c16c16c16962p-10))>(c, x2);
  c = fma_k<__builtin_bit_cast(uint64_t, (double)(0x1.5555555555555p-5))>(c, x2);
  c = fma(c, x2, -0.5);
  c = fma(c, x2, 1.0);
  // quadrant q: (sin, cos) = (s, c), (c, -s), (-s, -c), (-c, s); selects and sign-bit flips
  const int q = ((int)k) & 3;
  const bool sw = (q & 1) != 0;
  const uint64_t ms = (uint64_t)((q & 2) != 0) << 63, mc = (uint64_t)(((q + 1) & 2) != 0) << 63;
  *so = __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, sw ? c : s) ^ ms);
  *co = __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, sw ? s : c) ^ mc);
}

// log(x) of a uniform draw x = k * 2^-32, k in [0, 2^32) (random_double, utils.rs:5-7), for
// ConstantMedium's free-flight distance (constant_medium.rs:75). fdlibm's reduction: x = 2^e m,
// m in [sqrt(1/2), sqrt(2)), f = m - 1, s = f / (2 + f), log(m) = f - hfsq + s (hfsq + R(s^2)),
// with R a near-minimax polynomial of degree 7 fitted in 200-bit arithmetic (tools_gpu/
// fit_log.py: 0.77 ulp worst case over the draws, like the libm result within an ulp) and ln 2
// split so that e * ln2_hi is exact. About 30 f64 operations against the 95 of the general
// double-double library log; log(0) = -inf as in the reference (hit distance +inf: no scatter).
__device__ __forceinline__ double log_u01(double x) {
  double m = __builtin_amdgcn_frexp_mant(x);  // [0.5, 1)
  int e = __builtin_amdgcn_frexp_exp(x);
  const bool low = m < 0x1.6a09e667f3bcdp-1;  // sqrt(1/2)
  m = low ? m * 2.0 : m;
  e = low ? e - 1 : e;
  const double f = m - 1.0;
  const double hfsq = 0.5 * f * f;
  const double s = div_nr(f, 2.0 + f);
  const double z = s * s;
  double r = 0x1.2b5726b357134p-3;
  r = fma_k<__builtin_bit_cast(uint64_t, 0x1.39fe7a28d6e94p-3)>(r, z);
  r = fma_k<__builtin_bit_cast(uint64_t, 0x1.7462b3d0fabd6p-3)>(r, z);
  r = fma_k<__builtin_bit_cast(uint64_t, 0x1.c71c62e8d3992p-3)>(r, z);
  r = fma_k<__builtin_bit_cast(uint64_t, 0x1.2492492dee5a0p-2)>(r, z);
  r = fma_k<__builtin_bit_cast(uint64_t, 0x1.9999999995300p-2)>(r, z);
  r = fma_k<__builtin_bit_cast(uint64_t, 0x1.5555555555558p-1)>(r, z);
  const double R = r * z;
  const double dk = (double)e;
  const double t = fma(s, hfsq + R, dk * 0x1.be8e7bcd5e4f2p-27);  // ln2_lo
  const double v = dk * 0x1.62e42f8000000p-1 - ((hfsq - t) - f);  // ln2_hi
  return x == 0.0 ? -kInf : v;
}

// Perlin tables staged per workgroup (dynamic LDS of the TEX kernels: n_perlin_lds tables)
constexpr uint32_t kPerlinLds = 4;
// Scenes whose node/material/texture/light tables (+ Perlin tables) fit this many bytes are
// staged in LDS whole: 4 workgroups per CU x 24 KiB stay well inside the CU's 160 KiB.
constexpr size_t kStageScene = 24u << 10;
extern __shared__ __attribute__((aligned(16))) uint8_t rt_lds[];

// Table pointers for per-lane (divergent) reads: TP = lptr for the workgroup's LDS copy of a
// small scene (ds_read, 32-bit addresses: one SGPR per table), gptr for the global tables.
template <class TP>
struct TabsT {
  TP nodes, mats, texs, lights, loffs;
  const uint8_t* perlin;  // LDS: the staged Perlin tables
};

struct TraceParams {
  const uint32_t* __restrict__ nodes;
  const uint32_t* __restrict__ mats;
  const uint32_t* __restrict__ texs;
  const uint8_t* __restrict__ perlin;
  const uint32_t* __restrict__ lights;
  const uint32_t* __restrict__ light_offs;
  const uint8_t* __restrict__ texels;
  // f64 RGB outputs of the launch (rt_reduce sums them), 64 values (one per pixel of the tile)
  // per slot: the row totals of the row pairs [0, n_pairs_r) (slot = pair), the block partials
  // of the segment pairs [n_pairs_r, n_pairs_a) (slot = n_pairs_r + (pair - n_pairs_r) * n_blk +
  // blk), then the per-sample values of the tail pairs (slot = n_pairs_r + (n_pairs_a -
  // n_pairs_r) * n_blk + (pair - n_pairs_a) * sqrt_spp + s_i). A row or segment pool's id is
  // its slot.
  double* __restrict__ part;
  unsigned long long* __restrict__ ops;
  unsigned int* __restrict__ queue;  // next unclaimed pool (zeroed before each launch)
  int n_pools;    // pools of this launch: n_pairs_r + (pairs - n_pairs_r) * n_blk
  int n_pairs_r;  // (tile, s_j) pairs rendered as row items (one item per pixel, all s_i)
  int n_pairs_a;  // pairs [n_pairs_r, n_pairs_a): segment items; the rest one item per sample
  int n_blk;      // s_i blocks (segments) per pair: ceil(sqrt_spp / kPoolSi)
  uint32_t root, n_lights, lights_is_list, flags;
  uint32_t lights_nested;  // some light entry is a nested HittableList (RTL_LLIST)
  int sphere_light0;    // index of the first SPHERE light record, -1 if none
  double inv_n_lights;  // 1.0 / n_lights (host IEEE division, hittable.rs:116)
  uint32_t n_perlin_lds;  // Perlin tables readable from LDS (TEX kernels)
  // LDS staging (rt_trace prologue): stage_bytes of the scene allocation starting at stage_src.
  // stage_scene = 1: the whole small-table prefix [nodes .. Perlin] is copied, and per-lane
  // (divergent) reads of nodes / materials / textures / lights use the copy; 0: only the first
  // n_perlin_lds Perlin tables are copied. Offsets are bytes from the start of the allocation.
  const uint8_t* stage_src;
  uint32_t stage_bytes, stage_scene;
  // BVH region (rt_layout.h): node words [0, bvh_words) are BVH records; the first bvh_lds_words
  // of them are in LDS at byte offset bvh_lds_off (staged by the prologue unless stage_scene
  // already copied the node array)
  uint32_t bvh_words, bvh_lds_words, bvh_lds_off;
  // compact ordered BVHs (rt_layout.h CBVH) staged in LDS for cbvh_walk: cbvh_bytes from
  // cbvh_src at LDS byte offset cbvh_lds_off (~0u: not staged, the OBVH streams are walked from
  // global memory), and the walk's per-lane u16 stacks at stack_lds_off
  const uint8_t* cbvh_src;
  uint32_t cbvh_bytes, cbvh_lds_off, stack_lds_off;
  // BVH kernels: the row items' per-lane f64 row totals (3 x blockDim doubles) at this dynamic
  // LDS byte offset (row pools only when the plan placed them: n_pairs_r = 0 otherwise)
  uint32_t row_lds_off;
  uint32_t o_mats, o_texs, o_lights, o_loffs, o_perl;
  double center[3], p00[3], du[3], dv[3], ddu[3], ddv[3], bg[3];
  double rs;
  int defocus;
  int W, n_rows, row_begin, row_step, sqrt_spp, sj0, n_sj, max_depth;
  uint32_t seed_lo, seed_hi;
  int tiles_x;
};

// The kernel's only argument sits at offset 0 of the kernarg segment. Camera constants are read
// through this pointer at their point of use; the empty asm makes the pointer opaque so the loads
// are not hoisted out of the path loop, where ~40 loop-invariant SGPRs would spill to VGPR lanes.
typedef const __attribute__((address_space(4))) TraceParams* kparams_t;
__device__ __forceinline__ kparams_t kparams() {
  kparams_t p = (kparams_t)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return p;
}
__device__ __forceinline__ d3 karr3(const __attribute__((address_space(4))) double* a) {
  return {a[0], a[1], a[2]};
}

// ---------------------------------------------------------------- loads
// Two pointer kinds reach the same node records:
//  gptr: per-lane (divergent) node index -> vector loads (global_load_dwordx4 through L1/L2)
//  kptr: wave-uniform node index (no BVH: every lane walks the same node sequence) -> the
//        constant address space lets hipcc use scalar loads (s_load_dwordx*, K$), so node
//        data lands in SGPRs and costs neither VGPRs nor vector-memory latency.
typedef const uint32_t* gptr;
typedef const __attribute__((address_space(4))) uint32_t* kptr;
typedef const __attribute__((address_space(4))) double* kdptr;
//  lptr: the LDS copy of a staged small scene (per-lane reads as ds_read)
typedef const __attribute__((address_space(3))) uint32_t* lptr;
typedef const __attribute__((address_space(3))) double* ldptr;
typedef double v2d __attribute__((ext_vector_type(2)));
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(3))) v2d* ld2ptr;
typedef const __attribute__((address_space(3))) v4u* lu4ptr;

__device__ __forceinline__ d3 ld3(gptr X, int k) {  // f64 triple at payload double index k
  const double* d = reinterpret_cast<const double*>(X + 4) + k;
  if ((k & 1) == 0) {
    double2 a = *reinterpret_cast<const double2*>(d);
    return mk(a.x, a.y, d[2]);
  }
  double2 b = *reinterpret_cast<const double2*>(d + 1);
  return mk(d[0], b.x, b.y);
}
__device__ __forceinline__ d3 ld3(kptr X, int k) {
  kdptr d = reinterpret_cast<kdptr>(X + 4) + k;
  return mk(d[0], d[1], d[2]);
}
__device__ __forceinline__ double ldd(gptr X, int k) {
  return reinterpret_cast<const double*>(X + 4)[k];
}
__device__ __forceinline__ double ldd(kptr X, int k) { return reinterpret_cast<kdptr>(X + 4)[k]; }
__device__ __forceinline__ uint4 ld4u(gptr p) { return *reinterpret_cast<const uint4*>(p); }
__device__ __forceinline__ d3 ld3(lptr X, int k) {
  ldptr d = reinterpret_cast<ldptr>(X + 4) + k;
  if ((k & 1) == 0) {
    const v2d a = *reinterpret_cast<ld2ptr>(d);
    return mk(a.x, a.y, d[2]);
  }
  const v2d b = *reinterpret_cast<ld2ptr>(d + 1);
  return mk(d[0], b.x, b.y);
}
__device__ __forceinline__ double ldd(lptr X, int k) { return reinterpret_cast<ldptr>(X + 4)[k]; }
__device__ __forceinline__ uint4 ld4u(lptr p) {
  const v4u v = *reinterpret_cast<lu4ptr>(p);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint4 ld4u(kptr p) { return make_uint4(p[0], p[1], p[2], p[3]); }
// first 64 bytes of a node record: four independent 16-byte loads, one memory round trip
template <class Ptr>
__device__ __forceinline__ void ld64(Ptr p, uint4& a, uint4& b, uint4& c, uint4& e) {
  a = ld4u(p);
  b = ld4u(p + 4);
  c = ld4u(p + 8);
  e = ld4u(p + 12);
}
__device__ __forceinline__ d3 arr3(const double* a) { return mk(a[0], a[1], a[2]); }

// ---------------------------------------------------------------- op counters (COUNT build)
template <bool COUNT>
struct Ctr {
  __device__ __forceinline__ void inc(int) {}
  __device__ __forceinline__ void inc_if(int, bool) {}
  __device__ __forceinline__ void flush(unsigned int*) {}
};
template <>
struct Ctr<true> {
  uint32_t c[RT_OP_COUNT];
  __device__ Ctr() {
#pragma unroll
    for (int k = 0; k < RT_OP_COUNT; ++k) c[k] = 0;
  }
  __device__ __forceinline__ void inc(int k) { c[k]++; }
  __device__ __forceinline__ void inc_if(int k, bool b) { c[k] += b ? 1u : 0u; }
  __device__ void flush(unsigned int* sh) {
#pragma unroll
    for (int k = 0; k < RT_OP_COUNT; ++k)
      if (c[k]) atomicAdd(&sh[k], c[k]);
  }
};

// ---------------------------------------------------------------- primitives
// Quad::hit object.rs:453-490; inclusive interval (Interval::contains interval.rs:21-23).
// Branch-free: every lane evaluates the whole test and the outcome is a predicate, so a wave
// walks the quad in one straight-line block (no exec-mask churn, loads of the next node can be
// hoisted). Rejections follow the reference's order and NaN behaviour exactly:
// |n.d| < 1e-8 -> miss; !(tmin <= t <= tmax) -> miss; a < 0 || 1 < a || b < 0 || 1 < b -> miss.
template <bool COUNT, class Ptr>
__device__ __forceinline__ bool quad_test(Ptr q, d3 o, d3 d, double tmin, double tmax,
                                          double& t_out, Ctr<COUNT>& C) {
  C.inc(RT_OP_QUAD_TESTS);
  d3 n = ld3(q, 0);
  double denom = dot(n, d);
  double t = div_nr(ldd(q, 3) - dot(n, o), denom);
  d3 pq = vfma(t, d, o) - ld3(q, 4);
  double a = dot(pq, ld3(q, 8));
  double b = dot(pq, ld3(q, 12));
  const bool plane = !(fabs(denom) < 1e-8);
  const bool range = plane & (tmin <= t) & (t <= tmax);
  // IEEE minNum/maxNum: a NaN coordinate drops out, and the reference's comparisons accept it
  const double lo = __builtin_fmin(a, b), hi = __builtin_fmax(a, b);
  const bool hit = range & !(lo < 0.0) & !(1.0 < hi);
  C.inc_if(RT_OP_QUAD_PLANE, plane);
  C.inc_if(RT_OP_QUAD_INTERVAL, range);
  C.inc_if(RT_OP_QUAD_HITS, hit);
  t_out = hit ? t : t_out;
  return hit;
}

// The same test for an axis-aligned quad (rt_layout.h RTL_QUAD_AXIS): bit-identical results,
// with r = rcp_nr(d) computed once per batch instead of once per quad.
template <int K>
struct ic {  // an int as a type (compile-time axis of a generic lambda's argument)
  static constexpr int value = K;
};
template <int K>
__device__ __forceinline__ double comp(d3 v) {
  return K == 0 ? v.x : (K == 1 ? v.y : v.z);
}
__device__ __forceinline__ double hilo(uint32_t lo, uint32_t hi) {
  return __hiloint2double((int)hi, (int)lo);
}
struct AQuad {  // the first 64 bytes of a world QUAD record
  uint32_t h0;
  double qk, lo0, lo1, hi0, hi1;  // accepted hit-point coordinates per in-plane axis (rt_layout.h)
};
template <class Ptr>
__device__ __forceinline__ AQuad load_aquad(Ptr Q) {
  const uint4 a = ld4u(Q), b = ld4u(Q + 4), c = ld4u(Q + 8), e = ld4u(Q + 12);
  return {a.x, hilo(b.x, b.y), hilo(b.z, b.w), hilo(c.x, c.y), hilo(c.z, c.w), hilo(e.x, e.y)};
}
// t of an axis-aligned quad and whether its planar coordinates a, b lie in [0, 1] (shared by
// the test below and the one-walk ConstantMedium boundary). a = fl(fl(y - q) C) is monotone in
// the hit point's coordinate y, so the accept test !(a < 0) & !(1 < a) (NaN accepts, object.rs:473)
// is y in the record's [y0, y1] or NaN, compared directly (rt_layout.h; four compares instead of
// two subtractions, two products, min/max and two compares).
template <int K>
__device__ __forceinline__ void aquad_core(const AQuad& q, d3 o, d3 d, d3 r, double& t, bool& inr) {
  constexpr int LO = K == 0 ? 1 : 0, HI = K == 2 ? 1 : 2;
  const double dk = comp<K>(d), rk = comp<K>(r);
  const double num = q.qk - comp<K>(o);
  const double t0 = num * rk;
  t = fma(fma(-dk, t0, num), rk, t0);  // div_nr(num, dk)
  const double ya = fma(t, comp<LO>(d), comp<LO>(o)), yb = fma(t, comp<HI>(d), comp<HI>(o));
  inr = !(ya < q.lo0) & !(q.lo1 < ya) & !(yb < q.hi0) & !(q.hi1 < yb);
}
template <bool COUNT, int K>
__device__ __forceinline__ bool aquad_test(const AQuad& q, d3 o, d3 d, d3 r, double tmin,
                                           double tmax, double& t_out, Ctr<COUNT>& C) {
  C.inc(RT_OP_QUAD_TESTS);
  const double dk = comp<K>(d);
  double t;
  bool inr;
  aquad_core<K>(q, o, d, r, t, inr);
  // straight-line predicate
  const bool plane = !(fabs(dk) < 1e-8);
  const bool range = plane & (tmin <= t) & (t <= tmax);
  const bool hit = range & inr;
  C.inc_if(RT_OP_QUAD_PLANE, plane);
  C.inc_if(RT_OP_QUAD_INTERVAL, range);
  C.inc_if(RT_OP_QUAD_HITS, hit);
  t_out = hit ? t : t_out;
  return hit;
}
// A world QUAD record (batch member or single): branch on its axis code (wave-uniform in UNI
// traversal); r = rcp_nr(d) of the current frame.
template <bool COUNT, class Ptr>
__device__ __forceinline__ bool world_quad_test(Ptr Q, d3 o, d3 d, d3 r, double tmin, double tmax,
                                                double& t_out, Ctr<COUNT>& C) {
  const AQuad q = load_aquad(Q);
  switch (RTL_QUAD_AXIS(q.h0)) {
    case 1u: return aquad_test<COUNT, 0>(q, o, d, r, tmin, tmax, t_out, C);
    case 2u: return aquad_test<COUNT, 1>(q, o, d, r, tmin, tmax, t_out, C);
    case 3u: return aquad_test<COUNT, 2>(q, o, d, r, tmin, tmax, t_out, C);
    default: return quad_test<COUNT>(Q + RTL_QUAD_GEN, o, d, tmin, tmax, t_out, C);
  }
}

// world_quad_test on an axis-aligned form already in registers (Q = the record, for the
// general payload of a non-axis-aligned quad).
template <bool COUNT, class Ptr>
__device__ __forceinline__ bool aquad_dispatch(const AQuad& q, Ptr Q, d3 o, d3 d, d3 r,
                                               double tmin, double tmax, double& t_out,
                                               Ctr<COUNT>& C) {
  switch (RTL_QUAD_AXIS(q.h0)) {
    case 1u: return aquad_test<COUNT, 0>(q, o, d, r, tmin, tmax, t_out, C);
    case 2u: return aquad_test<COUNT, 1>(q, o, d, r, tmin, tmax, t_out, C);
    case 3u: return aquad_test<COUNT, 2>(q, o, d, r, tmin, tmax, t_out, C);
    default: return quad_test<COUNT>(Q + RTL_QUAD_GEN, o, d, tmin, tmax, t_out, C);
  }
}

template <bool COUNT>
__device__ __forceinline__ bool sphere_test_v(d3 center, double r, d3 o, d3 d, double tmin,
                                              double tmax, double& t_out, Ctr<COUNT>& C);
// Sphere::hit object.rs:145-184; strict interval (Interval::surrounds interval.rs:25-27).
template <bool COUNT, class Ptr>
__device__ __forceinline__ bool sphere_test(Ptr s, d3 o, d3 d, double tm, double tmin,
                                            double tmax, double& t_out, Ctr<COUNT>& C) {
  d3 center = ld3(s, 0);
  if (s[0] & RTL_SPHERE_MOVING) center = vfma(tm, ld3(s, 4), center);  // Sphere::center(time) object.rs:107-112
  return sphere_test_v<COUNT>(center, ldd(s, 3), o, d, tmin, tmax, t_out, C);
}
// sphere_test on a center (at the ray's time) and radius already in registers; the generated
// scene walkers (rt_jit.cpp) pass them as literals.
template <bool COUNT>
__device__ __forceinline__ bool sphere_test_v(d3 center, double r, d3 o, d3 d, double tmin,
                                              double tmax, double& t_out, Ctr<COUNT>& C) {
  C.inc(RT_OP_SPHERE_TESTS);
  d3 oc = o - center;
  double a = dot(d, d);
  double half_b = dot(oc, d);
  double c = dot(oc, oc) - r * r;
  double disc = fma(half_b, half_b, -(a * c));
  // straight-line: both roots are formed and the predicate selects (object.rs:157-166); a
  // negative discriminant gives NaN roots, which the predicate never reads
  const bool real = !(disc < 0.0);
  C.inc_if(RT_OP_SPHERE_ROOTS, real);
  const double sqrtd = sqrt_nr(disc);
  const double ra = rcp_nr(a);
  const double near = (-half_b - sqrtd) * ra;
  const double far = (sqrtd - half_b) * ra;
  const bool in_near = (tmin < near) & (near < tmax);
  const bool in_far = (tmin < far) & (far < tmax);
  const bool hit = real & (in_near | in_far);
  C.inc_if(RT_OP_SPHERE_HITS, hit);
  t_out = hit ? (in_near ? near : far) : t_out;
  return hit;
}

// Aabb::hit object.rs:340-370 on bounds already in registers (the LANE walker's 64-byte node
// fetch), with inv_d = 1/d computed once per ray frame.
__device__ __forceinline__ bool aabb_hit(const double (&mn)[3], const double (&mx)[3], d3 o,
                                         d3 inv, double tmin, double tmax) {
  const double oo[3] = {o.x, o.y, o.z}, id[3] = {inv.x, inv.y, inv.z};
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    double t0 = (mn[a] - oo[a]) * id[a];
    double t1 = (mx[a] - oo[a]) * id[a];
    if (id[a] < 0.0) {
      double tt = t0;
      t0 = t1;
      t1 = tt;
    }
    if (t0 > tmin) tmin = t0;
    if (t1 < tmax) tmax = t1;
    if (tmax <= tmin) return false;
  }
  return true;
}

// The same test without branches: tmin only grows and tmax only shrinks, so one final
// comparison answers the reference's per-axis early exit, and max/min (IEEE maxNum/minNum:
// a NaN slab bound, (min - o) * inf with o on the slab plane, leaves the interval alone) are
// the reference's `if t0 > tmin { tmin = t0 }` / `if t1 < tmax { tmax = t1 }` (ties differ
// at most in the sign of a zero, which no comparison sees).
__device__ __forceinline__ bool aabb_hit_bf(const double (&mn)[3], const double (&mx)[3], d3 o,
                                            d3 inv, double tmin, double tmax) {
  const double oo[3] = {o.x, o.y, o.z}, id[3] = {inv.x, inv.y, inv.z};
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const double t0 = (mn[a] - oo[a]) * id[a];
    const double t1 = (mx[a] - oo[a]) * id[a];
    const bool neg = id[a] < 0.0;
    tmin = __builtin_fmax(tmin, neg ? t1 : t0);
    tmax = __builtin_fmin(tmax, neg ? t0 : t1);
  }
  return tmin < tmax;
}

// Translate/RotateY ray into object space (transform.rs:59, 86-107).
__device__ __forceinline__ void translate_in(d3 off, d3& o) { o = o - off; }
__device__ __forceinline__ void rotate_y_in(double s, double c, d3& o, d3& d) {
  o = mk(fma(c, o.x, -(s * o.z)), o.y, fma(s, o.x, c * o.z));
  d = mk(fma(c, d.x, -(s * d.z)), d.y, fma(s, d.x, c * d.z));
}
template <class Ptr>
__device__ __forceinline__ void xform_in(Ptr X, d3& o, d3& d) {
  if ((X[0] & 0xffu) == RTL_TRANSLATE) {
    translate_in(ld3(X, 2), o);
  } else {
    rotate_y_in(ldd(X, 2), ldd(X, 3), o, d);
  }
}
// Hit record back to the parent space (transform.rs:65, 114-130).
template <class Ptr>
__device__ __forceinline__ void xform_out(Ptr X, d3& p, d3& n) {
  if ((X[0] & 0xffu) == RTL_TRANSLATE) {
    p = p + ld3(X, 2);
  } else {
    double s = ldd(X, 2), c = ldd(X, 3);
    p = mk(fma(c, p.x, s * p.z), p.y, fma(-s, p.x, c * p.z));
    n = mk(fma(c, n.x, s * n.z), n.y, fma(-s, n.x, c * n.z));
  }
}
// xform_out on constants already in registers (generated frame code, rt_jit.cpp)
__device__ __forceinline__ void translate_out(d3 off, d3& p) { p = p + off; }
__device__ __forceinline__ void rotate_y_out(double s, double c, d3& p, d3& n) {
  p = mk(fma(c, p.x, s * p.z), p.y, fma(-s, p.x, c * p.z));
  n = mk(fma(c, n.x, s * n.z), n.y, fma(-s, n.x, c * n.z));
}
// Local ray of `frame` = the world ray pushed through its transform chain, root first.
template <class Ptr>
__device__ __forceinline__ void frame_ray(Ptr N, int frame, d3 wo, d3 wd, d3& o, d3& d) {
  o = wo;
  d = wd;
  if (frame < 0) return;
  uint4 h = ld4u(N + frame);
  uint4 ch = ld4u(N + frame + 4);
  if (h.x & RTL_XFORM_LONG) {  // chain in the appended table (rt_layout.h)
    for (uint32_t k = 0; k < h.z; ++k) xform_in(N + N[ch.x + k], o, d);
    return;
  }
  const uint32_t c4[4] = {ch.x, ch.y, ch.z, ch.w};
#pragma unroll
  for (int k = 0; k < RTL_MAX_CHAIN; ++k)
    if ((uint32_t)k < h.z) xform_in(N + c4[k], o, d);
}
// A hit point and normal of `frame` back to world space, innermost transform first.
template <class Ptr>
__device__ __forceinline__ void frame_out(Ptr N, int frame, d3& p, d3& n) {
  if (frame < 0) return;
  const uint4 fh = ld4u(N + frame);
  const uint4 ch = ld4u(N + frame + 4);
  if (fh.x & RTL_XFORM_LONG) {
    for (uint32_t k = fh.z; k-- > 0;) xform_out(N + N[ch.x + k], p, n);
    return;
  }
  const uint32_t c4[4] = {ch.x, ch.y, ch.z, ch.w};
#pragma unroll
  for (int k = RTL_MAX_CHAIN - 1; k >= 0; --k)
    if ((uint32_t)k < fh.z) xform_out(N + c4[k], p, n);
}

// ConstantMedium::hit's two boundary queries (constant_medium.rs:46-55) in ONE wave-uniform walk
// of a boundary flagged RTL_VOLF_* by the flattener: rec1 = boundary.hit(r, (-inf, inf)),
// rec2 = boundary.hit(r, [rec1.t + 1e-4, inf)). With closest-hit updates over one primitive (or
// a list of quads), rec1.t is the smallest candidate and rec2.t the smallest candidate >= tmin2
// = rec1.t + 1e-4, where a candidate is a root inside the strict interval (sphere) or a quad
// hit whose planar coordinates are inside (the quads' interval is inclusive). The walk keeps
// the two smallest quad candidates (with multiplicity); when both lie below tmin2 the lane
// needs the third and reports `fallback` (the caller reruns the second query for it). The
// arithmetic of every candidate is the sphere_test / aquad_test arithmetic, so t1 and t2 are
// the two-pass values bit for bit. Not used by the op-counting build.
__device__ bool volume_two_hits(const TraceParams& P, uint32_t node, uint32_t kind, d3 o, d3 d,
                                double tm, double& t1, double& t2, bool& fallback) {
  const kptr N = (kptr)P.nodes;
  fallback = false;
  for (;;) {  // the instance chain in front of the primitive(s)
    const uint32_t ty = N[node] & 0xffu;
    if (ty != RTL_TRANSLATE && ty != RTL_ROTATE_Y) break;
    xform_in(N + node, o, d);
    node = N[node + 3];
  }
  const kptr X = N + node;
  if (kind == RTL_VOLF_SPHERE) {  // sphere_test's roots once, both strict intervals
    d3 center = ld3(X, 0);
    const double r = ldd(X, 3);
    if (X[0] & RTL_SPHERE_MOVING) center = vfma(tm, ld3(X, 4), center);
    const d3 oc = o - center;
    const double a = dot(d, d);
    const double half_b = dot(oc, d);
    const double c = dot(oc, oc) - r * r;
    const double disc = fma(half_b, half_b, -(a * c));
    const bool real = !(disc < 0.0);
    const double sqrtd = sqrt_nr(disc);
    const double ra = rcp_nr(a);
    const double near = (-half_b - sqrtd) * ra;
    const double far = (sqrtd - half_b) * ra;
    const bool n1 = (-kInf < near) & (near < kInf), f1 = (-kInf < far) & (far < kInf);
    t1 = n1 ? near : far;
    const double tmin2 = t1 + 0.0001;
    const bool n2 = (tmin2 < near) & (near < kInf), f2 = (tmin2 < far) & (far < kInf);
    t2 = n2 ? near : far;
    return real & (n1 | f1) & (n2 | f2);
  }
  // axis-aligned quads: one QUAD record or a QUADS batch
  const bool batch = (X[0] & 0xffu) == RTL_QUADS;
  const uint32_t cnt = batch ? (X[0] >> 8) : 1u;
  kptr Q = batch ? X + 4 : X;
  const d3 r = mk(rcp_nr1(d.x), rcp_nr1(d.y), rcp_nr1(d.z));
  // the two smallest candidates with multiplicity, +inf = none: min/max updates (a candidate's t
  // is finite: |q_k - o_k| < 2^1023 and |d_k| >= 1e-8)
  double m1 = kInf, m2 = kInf;
  for (uint32_t k = 0; k < cnt; ++k, Q += RTL_QUAD_WORDS) {
    const AQuad q = load_aquad(Q);
    double t;
    double dk;
    bool inr;
    switch (RTL_QUAD_AXIS(q.h0)) {
      case 1u: aquad_core<0>(q, o, d, r, t, inr); dk = d.x; break;
      case 2u: aquad_core<1>(q, o, d, r, t, inr); dk = d.y; break;
      default: aquad_core<2>(q, o, d, r, t, inr); dk = d.z; break;
    }
    // aquad_test's predicate without the interval, plus t >= -inf (not NaN)
    const bool v = !(fabs(dk) < 1e-8) & (-kInf <= t) & inr;
    const double te = v ? t : kInf;
    m2 = __builtin_fmin(m2, __builtin_fmax(m1, te));
    m1 = __builtin_fmin(m1, te);
  }
  const bool have1 = m1 < kInf, have2 = m2 < kInf;
  t1 = m1;
  const double tmin2 = m1 + 0.0001;
  bool hit2;
  if (m1 >= tmin2) {  // only when m1 + 1e-4 rounds back to m1
    t2 = m1;
    hit2 = true;
  } else if (have2 && m2 >= tmin2) {
    t2 = m2;
    hit2 = true;
  } else {
    t2 = 0.0;
    hit2 = false;
    fallback = have2;  // two candidates inside [t1, tmin2): the answer is a third one
  }
  return have1 & (hit2 | fallback);
}
// The one-walk boundary query of the interpreter; scene-specialised kernels (rt_jit.cpp) pass
// a generated policy per ConstantMedium record with the same arithmetic.
struct VolTwoInterp {
  static __device__ __forceinline__ bool two_hits(const TraceParams& P, uint32_t node,
                                                  uint32_t kind, d3 o, d3 d, double tm,
                                                  double& t1, double& t2, bool& fallback) {
    return volume_two_hits(P, node, kind, o, d, tm, t1, t2, fallback);
  }
};

#ifdef RT_PROF
// profiling build: per-lane LANE-walker step counts and per-workgroup traversal counters
// (flushed to P.ops[10..17] at kernel exit; tools_gpu/prof_sections.py)
__shared__ uint32_t prof_steps[kBlockBvh];
__shared__ unsigned long long prof_trav[16];
__shared__ uint32_t prof_wmax[kBlockBvh / 64];
__shared__ unsigned long long prof_wt[kBlockBvh / 64];
__device__ __forceinline__ bool prof_first_lane() {
  const unsigned long long m = __ballot(1);
  return (threadIdx.x & 63) == (unsigned)(__builtin_ctzll(m));
}
// wave-level section timer of the LANE walker: cycles since the wave's last checkpoint go to
// section k (prof_trav[8 + k]), and cnt counts the checkpoint (prof_trav[12 + k])
#define PFW(k, cnt)                                                      \
  do {                                                                   \
    const unsigned long long now_ = __builtin_readcyclecounter();       \
    if (prof_first_lane()) {                                             \
      const int w_ = threadIdx.x >> 6;                                   \
      if ((k) >= 0) atomicAdd(&prof_trav[8 + (k)], now_ - prof_wt[w_]); \
      prof_wt[w_] = now_;                                                \
      if (cnt) atomicAdd(&prof_trav[12 + ((k) < 0 ? 0 : (k))], 1ull);   \
    }                                                                    \
  } while (0)
#endif

// ---------------------------------------------------------------- traversal
// Threaded walk of the flattened scene (rt_layout.h). MAIN: the world (records the hit node and
// its frame, handles ConstantMedium when VOL). !MAIN: a volume boundary (closest t only).
//
// Two walkers share this body:
//  UNI  (wave-uniform): outside BVH subtrees the node sequence does not depend on the ray (lists,
//       transforms, volumes and primitives are visited in a fixed order), so the node index is
//       readfirstlane'd and node records arrive by scalar loads (K$, SGPRs, no VGPRs). Used for
//       every scene's top level.
//  LANE (per-lane): inside a BVH subtree each lane follows its own skip links. Each node's first
//       64 bytes (header + bbox, or header + axis-aligned quad form) are fetched by four
//       independent 16-byte vector loads, so one memory round trip serves a BVH node. The UNI
//       walker hands a BVH subtree [root, skip) to the LANE walker with the current closest-hit
//       state and resumes at its skip once every lane has finished it (BVH = the scene has one).
// VOLB: some ConstantMedium lies inside a BVH subtree (the per-lane walker then needs its volume
// branch, a nested walker; without it the LANE instantiation leaves that code out).
// VOLI: some ConstantMedium boundary may need the interpreter's two walks (not one-walk, or one-
// walk quads whose third candidate can be needed); without it only volume_two_hits is compiled.
// VN: ConstantMedium records nested inside volume boundaries are handled this many levels deep
// (constant_medium.rs:46-55 queries `boundary.hit`, which may be another ConstantMedium).
template <bool MAIN, bool COUNT, bool VOL, bool UNI, bool BVH, bool VOLB = VOL, bool VOLI = true,
          int VN = 0>
__device__ bool traverse(const TraceParams& P, uint32_t node, uint32_t stop, d3 wo, d3 wd,
                         double tm, d3 o, d3 d, int frame, double tmin, double tmax,
                         double& t_out, uint32_t& hit_node, int& hit_frame, Rng& g,
                         Ctr<COUNT>& C);
// ConstantMedium::hit constant_medium.rs:41-95 for the VOLUME record at `node` (header h) in the
// current frame (o, d): true when the free-flight distance ends inside the boundary before
// `closest`, with the hit t in t_hit. Shared by the interpreter walker and the generated
// walkers of rt_jit.cpp.
template <bool COUNT, bool UNI, bool BVH, bool VOLI, class VT = VolTwoInterp, int VN = 0>
__device__ __forceinline__ bool volume_hit(const TraceParams& P, uint32_t node, uint4 h, d3 wo,
                                           d3 wd, double tm, d3 o, d3 d, int frame, double tmin,
                                           double closest, double& t_hit, Rng& g, Ctr<COUNT>& C,
                                           const double* ray_len = nullptr) {
  // ray_len: |d| computed once by a generated walker for all the volumes of one frame (the same
  // sqrt_nr(dot(d, d)) of the same d)
  typedef typename cond<UNI, kptr, gptr>::type Ptr;
  const Ptr X = (Ptr)P.nodes + node;
  C.inc(RT_OP_VOLUME_TESTS);
  // rec1 = boundary.hit(r, (-inf, inf)), rec2 = boundary.hit(r, [rec1.t + 1e-4, inf)):
  // one rolled loop, so the boundary walker is instantiated once
  double t1 = 0.0, t2 = 0.0;
  bool both = true;
  const uint32_t fuse = h.x & (RTL_VOLF_SPHERE | RTL_VOLF_QUADS);
  if constexpr (UNI && !COUNT && !VOLI) {  // every boundary is a one-walk sphere
    bool fb;
    both = VT::two_hits(P, h.w, fuse, o, d, tm, t1, t2, fb);
  } else if (UNI && !COUNT && fuse) {
    bool fb;
    both = VT::two_hits(P, h.w, fuse, o, d, tm, t1, t2, fb);
    if (__ballot(fb) != 0ull) {  // rare: rerun the second query for those lanes
      double tb;
      uint32_t dn;
      int df;
      const bool b2 = traverse<false, COUNT, false, UNI, BVH>(P, h.w, ~0u, wo, wd, tm, o, d,
                                                              frame, t1 + 0.0001, kInf, tb,
                                                              dn, df, g, C);
      if (fb) {
        both = b2;
        t2 = tb;
      }
    }
  } else {
#pragma unroll 1
    for (int pass = 0; pass < 2 && both; ++pass) {
      double tb;
      uint32_t dn;
      int df;
      // a boundary holding ConstantMedium records (VN > 0) walks them too: their hits (and
      // random draws) are part of `boundary.hit`, in the reference's order
      both = traverse<false, COUNT, (VN > 0), UNI, BVH, false, true, VN>(P, h.w, ~0u, wo, wd, tm,
                                                                         o, d, frame,
                                                                         pass ? t1 + 0.0001 : -kInf,
                                                                         kInf, tb, dn, df, g, C);
      if (pass) t2 = tb; else t1 = tb;
    }
  }
  if (both) {
    if (t1 < tmin) t1 = tmin;
    if (t2 > closest) t2 = closest;
    if (t1 < t2) {
      if (t1 < 0.0) t1 = 0.0;
      const double ray_length = ray_len ? *ray_len : sqrt_nr(dot(d, d));
      double dist_inside = (t2 - t1) * ray_length;
      C.inc(RT_OP_VOLUME_DRAWS);
      double hit_distance = ldd(X, 0) * log_u01(rnd(g));
      if (!(hit_distance > dist_inside)) {
        t_hit = t1 + div_nr(hit_distance, ray_length);
        return true;
      }
    }
  }
  return false;
}

// A BVH subtree [node, stop) walked per lane: its ordered BVH when it has one (obvh != 0),
// otherwise (and always in the op-counting build) the reference tree in the reference order.
template <bool MAIN, bool COUNT, bool VOLB, bool BVH>
__device__ bool bvh_subtree(const TraceParams& P, uint32_t node, uint32_t stop, uint32_t obvh,
                            d3 wo, d3 wd, double tm, d3 o, d3 d, int frame, double tmin,
                            double tmax, double& t_out, uint32_t& hit_node, int& hit_frame,
                            Rng& g, Ctr<COUNT>& C);

template <bool MAIN, bool COUNT, bool VOL, bool UNI, bool BVH, bool VOLB, bool VOLI, int VN>
__device__ bool traverse(const TraceParams& P, uint32_t node, uint32_t stop, d3 wo, d3 wd,
                         double tm, d3 o, d3 d, int frame, double tmin, double tmax,
                         double& t_out, uint32_t& hit_node, int& hit_frame, Rng& g,
                         Ctr<COUNT>& C) {
  typedef typename cond<UNI, kptr, gptr>::type Ptr;
  const Ptr N = (Ptr)P.nodes;
  double closest = tmax;
  bool hit = false;
  // 1/d of the lane's ray in the current frame (Aabb::hit object.rs:347 divides per test; the
  // quotient is the same value every time, so the LANE walker forms it once per frame, by
  // rcp_w: within an ulp, and 1/+-0 = +-inf as the slab test needs)
  d3 inv = mk(0., 0., 0.);
  if (!UNI) inv = mk(rcp_w(d.x), rcp_w(d.y), rcp_w(d.z));
#ifdef RT_PROF
  if (!UNI) PFW(-1, 0);
#endif
  for (;;) {
    uint4 h, q1, q2, q3;
#ifdef RT_PROF
    if (!UNI) PFW(0, 1);
#endif
    if (UNI) {
      node = __builtin_amdgcn_readfirstlane(node);
      frame = __builtin_amdgcn_readfirstlane(frame);
      h = ld4u(N + node);
    } else {
      if (node == stop) break;
      // while-while: a lane steps through BVH nodes until it reaches a leaf (or the subtree's
      // end); lanes that got there first wait at the loop exit, so the leaf bodies below run
      // with every lane that has a leaf instead of interleaving with the AABB steps. BVH records
      // live in the BVH region [0, bvh_words) (rt_layout.h), so the index alone says "BVH node"
      // and no header is read; the region's first bvh_lds_words words are staged in LDS.
      const kparams_t KP = kparams();
      const uint32_t bvh_words = KP->bvh_words, bvh_lds = KP->bvh_lds_words;
      const uint4* LB = reinterpret_cast<const uint4*>(rt_lds + KP->bvh_lds_off);
      auto step = [&](uint4 bh, uint4 b1, uint4 b2, uint4 b3) {
        C.inc(RT_OP_AABB_TESTS);
#ifdef RT_PROF
        prof_steps[threadIdx.x] += 1;
        if (prof_first_lane()) atomicAdd(&prof_trav[13], 1ull);
#endif
        const double mn[3] = {hilo(b1.x, b1.y), hilo(b2.x, b2.y), hilo(b3.x, b3.y)};
        const double mx[3] = {hilo(b1.z, b1.w), hilo(b2.z, b2.w), hilo(b3.z, b3.w)};
        node = aabb_hit_bf(mn, mx, o, inv, tmin, closest) ? bh.z : bh.y;  // first child : skip
      };
      if (bvh_lds == bvh_words) {  // the whole region is in LDS
        while (node < bvh_words) {
          const uint4* L = LB + (node >> 2);
          step(L[0], L[1], L[2], L[3]);
          if (node == stop) break;
        }
      } else {
        while (node < bvh_words) {
          uint4 bh, b1, b2, b3;
          if (node < bvh_lds) {
            const uint4* L = LB + (node >> 2);
            bh = L[0], b1 = L[1], b2 = L[2], b3 = L[3];
          } else {
            ld64(N + node, bh, b1, b2, b3);
          }
          step(bh, b1, b2, b3);
          if (node == stop) break;
        }
      }
#ifdef RT_PROF
      PFW(1, 0);
#endif
      if (node == stop) break;
      ld64(N + node, h, q1, q2, q3);  // a leaf record (the node array is padded past its END)
#ifdef RT_PROF
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      PFW(2, 1);
#endif
    }
    const Ptr X = N + node;
    uint32_t type = h.x & 0xffu;
    if (type == RTL_QUAD) {
      double t = closest;
      const d3 r = mk(rcp_nr1(d.x), rcp_nr1(d.y), rcp_nr1(d.z));
      bool hq;
      if (UNI) {
        hq = world_quad_test<COUNT>(X, o, d, r, tmin, closest, t, C);
      } else {
        const AQuad q = {h.x, hilo(q1.x, q1.y), hilo(q1.z, q1.w), hilo(q2.x, q2.y),
                         hilo(q2.z, q2.w), hilo(q3.x, q3.y)};
        hq = aquad_dispatch<COUNT>(q, X, o, d, r, tmin, closest, t, C);
      }
      closest = t;  // t_out is only written on a hit (t started as closest)
      hit = hit | hq;
      if (MAIN) {
        hit_node = hq ? node : hit_node;
        hit_frame = hq ? frame : hit_frame;
      }
      node = h.w;
    } else if (type == RTL_QUADS) {
      // batch of sibling quads: the same sequential closest-hit updates as the list
      const uint32_t cnt = h.x >> 8;
      Ptr Q = X + 4;
      const d3 r = mk(rcp_nr1(d.x), rcp_nr1(d.y), rcp_nr1(d.z));
      uint4 a0, a1, a2, a3;  // LANE: the next quad's axis form is in flight during this test
      if (!UNI) ld64(Q, a0, a1, a2, a3);
      // the batch's winner is tracked as an index: one select per quad instead of three
      uint32_t hk = ~0u;
      for (uint32_t k = 0; k < cnt; ++k, Q += RTL_QUAD_WORDS) {
        double t = closest;
        bool hq;
        if (UNI) {  // scalar loads at the point of use (prefetching them raised SGPR pressure)
          hq = world_quad_test<COUNT>(Q, o, d, r, tmin, closest, t, C);
        } else {
          const AQuad q = {a0.x, hilo(a1.x, a1.y), hilo(a1.z, a1.w), hilo(a2.x, a2.y),
                           hilo(a2.z, a2.w), hilo(a3.x, a3.y)};
          ld64(Q + RTL_QUAD_WORDS, a0, a1, a2, a3);  // past the batch: the next node (padded)
          hq = aquad_dispatch<COUNT>(q, Q, o, d, r, tmin, closest, t, C);
        }
        // selects, not a branch: the closest-hit update stays in the straight-line block
        closest = t;  // t_out is only written on a hit (t started as closest)
        hk = hq ? k : hk;
      }
      const bool hb = hk != ~0u;
      hit = hit | hb;
      if (MAIN) {
        hit_node = hb ? (uint32_t)(node + 4 + hk * RTL_QUAD_WORDS) : hit_node;
        hit_frame = hb ? frame : hit_frame;
      }
      node = h.y;
#ifdef RT_PROF
      if (!UNI) PFW(3, 1);
#endif
    } else if (type == RTL_SPHERE) {
      double t = closest;
      const bool hs = sphere_test<COUNT>(X, o, d, tm, tmin, closest, t, C);
      closest = t;
      hit = hit | hs;
      if (MAIN) {
        hit_node = hs ? node : hit_node;
        hit_frame = hs ? frame : hit_frame;
      }
      node = h.w;
    } else if (type == RTL_BVH) {
      if (UNI) {
        if (BVH) {  // the subtree [node, skip) per lane, continuing this walk's closest hit
          double t;
          uint32_t hn;
          int hf;
#ifdef RT_PROF
          const unsigned long long pt0 = __builtin_readcyclecounter();
          prof_steps[threadIdx.x] = 0u;
#endif
          const bool sub = bvh_subtree<MAIN, COUNT, VOLB, BVH>(P, node, h.y, h.w, wo, wd, tm, o,
                                                             d, frame, tmin, closest, t, hn, hf,
                                                             g, C);
#ifdef RT_PROF
          {
            const unsigned long long dt = __builtin_readcyclecounter() - pt0;
            const uint32_t st = prof_steps[threadIdx.x];
            const int wv = threadIdx.x >> 6;
            atomicMax(&prof_wmax[wv], st);
            const uint32_t mx = prof_wmax[wv];
            const int which = MAIN ? (frame < 0 ? 0 : 1) : 2;
            if (prof_first_lane()) {
              prof_wmax[wv] = 0u;
              atomicAdd(&prof_trav[which], dt);
              atomicAdd(&prof_trav[3 + (which > 0 ? 1 : 0)], (unsigned long long)mx);
            }
            atomicAdd(&prof_trav[5 + (which > 0 ? 1 : 0)], (unsigned long long)st);
            if (prof_first_lane()) atomicAdd(&prof_trav[7], 1ull);
          }
#endif
          if (sub) {
            closest = t;
            hit = true;
            if (MAIN) {
              hit_node = hn;
              hit_frame = hf;
            }
          }
        }
        node = h.y;
      }  // LANE: BVH nodes never get here (the while-while step above consumes them)
    } else if (type == RTL_TRANSLATE || type == RTL_ROTATE_Y) {
      C.inc(type == RTL_TRANSLATE ? RT_OP_TRANSLATE : RT_OP_ROTATE_Y);
      xform_in(X, o, d);
      if (!UNI && type == RTL_ROTATE_Y) inv = mk(rcp_w(d.x), rcp_w(d.y), rcp_w(d.z));
      frame = (int)node;
      node = h.w;  // the instance's child
    } else if (type == RTL_EXIT) {
      frame = (int)h.z;
      frame_ray(N, frame, wo, wd, o, d);
      if (!UNI) inv = mk(rcp_w(d.x), rcp_w(d.y), rcp_w(d.z));
      node = h.w;
    } else if ((MAIN || VN > 0) && VOL && type == RTL_VOLUME) {
      double tv;
      if (volume_hit<COUNT, UNI, BVH, VOLI, VolTwoInterp, (MAIN ? VN : (VN > 0 ? VN - 1 : 0))>(
              P, node, h, wo, wd, tm, o, d, frame, tmin, closest, tv, g, C)) {
        closest = tv;
        hit = true;
        if (MAIN) {
          hit_node = node;
          hit_frame = frame;
        }
      }
      node = h.y;
    } else if (type == RTL_DUP) {
      node = COUNT ? h.w : h.y;
    } else if (type == RTL_END) {
      break;
    } else {
      node = h.y;
    }
  }
#ifdef RT_PROF
  if (!UNI) PFW(0, 0);
#endif
  t_out = closest;
  return hit;
}


// The ordered-BVH walk (rt_layout.h OBVH, rt_obvh.cpp) of one lane over the same leaf records as
// the reference subtree. Every candidate is computed with the reference walker's arithmetic
// (aquad_core / quad_test / sphere_test_v), but without the running upper bound: a quad's t
// (inclusive [tmin, inf)), a sphere's near root in (tmin, inf) else its far root. The closest
// candidate wins; away from ties that is the record the reference order returns. The lane is
// flagged (the caller re-walks the reference tree in the reference order) when its result could
// depend on the order: a candidate within kTieRel (relative) of the running closest t (which
// starts at the caller's tmax), or a winner within kTieRel of tmin. Boxes are padded bounds and
// the slab test keeps every box whose entry is <= closest * (1 + kTieRel), so no candidate the
// flag logic must see is culled.
constexpr double kTieRel = 0x1p-30;
typedef float f32x2 __attribute__((ext_vector_type(2)));
// The exact test of one ordered-BVH leaf record (QUAD, QUADS batch, SPHERE) with the reference
// walker's arithmetic; every candidate goes to cand(valid, t, record).
template <class F>
__device__ __forceinline__ void obvh_leaf(const gptr N, uint32_t rec, d3 o, d3 d, d3 r, double tm,
                                          double tmin, F& cand) {
  const bool box = (rec & RTL_LEAF_BOX) != 0u;
  rec &= ~RTL_LEAF_BOX;
  if (box && tmin >= 0.0) {
    // make_box's six sides (object.rs:509-560; rt_obvh.cpp make_box_batch): 0 z = max, 1 x = max,
    // 2 z = min, 3 x = min, 4 y = max, 5 y = min. The three sides the ray faces (the min side of
    // an axis where d >= 0) are tested in full with the batch's arithmetic. The other three are
    // candidates only at their plane's t (aquad_core's quotient, +inf where the plane test or the
    // interval rejects them), so when every such t lies beyond the facing sides' smallest
    // candidate by more than the tie window, none of them can win or come within 3 kTieRel of the
    // final closest (any closest <= that candidate), and their tests are skipped: the walk's result
    // and tie flag are the full batch's. Otherwise (no facing side hit, a grazing ray, an origin
    // inside the box) they are tested as well. The order of candidates only matters at exact ties,
    // which the tie flag sends to the reference-order walk.
    const gptr B = N + rec + 4;
    const uint32_t fx = d.x >= 0.0 ? 3u : 1u, fy = d.y >= 0.0 ? 5u : 4u, fz = d.z >= 0.0 ? 2u : 0u;
    const uint32_t gx = 4u - fx, gy = 9u - fy, gz = 2u - fz;  // the opposite sides
    double front = kInf;
    auto side = [&](const AQuad& q, uint32_t f, auto K) {
      double t;
      bool inr;
      aquad_core<decltype(K)::value>(q, o, d, r, t, inr);
      const double dk = comp<decltype(K)::value>(d);
      const bool v = !(fabs(dk) < 1e-8) & (tmin <= t) & inr;
      cand(v, t, rec + 4 + f * RTL_QUAD_WORDS);
      front = v ? fmin(front, t) : front;
    };
    // one side's 64-byte record in flight while the previous one is tested (as the batch loop)
    AQuad q = load_aquad(B + fx * RTL_QUAD_WORDS), qn = load_aquad(B + fy * RTL_QUAD_WORDS);
    side(q, fx, ic<0>());
    q = qn;
    qn = load_aquad(B + fz * RTL_QUAD_WORDS);
    side(q, fy, ic<1>());
    const double px = ldd(B + gx * RTL_QUAD_WORDS, 0), py = ldd(B + gy * RTL_QUAD_WORDS, 0),
                 pz = ldd(B + gz * RTL_QUAD_WORDS, 0);
    side(qn, fz, ic<2>());
    // the opposite sides' candidate t: the plane quotient of aquad_core
    auto plane = [&](double qk, auto K) {
      constexpr int k = decltype(K)::value;
      const double dk = comp<k>(d), rk = comp<k>(r);
      const double num = qk - comp<k>(o);
      const double t0 = num * rk;
      const double t = fma(fma(-dk, t0, num), rk, t0);
      return (!(fabs(dk) < 1e-8) & (tmin <= t)) ? t : kInf;
    };
    const double far = fmin(fmin(plane(px, ic<0>()), plane(py, ic<1>())), plane(pz, ic<2>()));
    if (!(front < kInf) || far <= front * (1.0 + 3.0 * kTieRel)) {
      side(load_aquad(B + gx * RTL_QUAD_WORDS), gx, ic<0>());
      side(load_aquad(B + gy * RTL_QUAD_WORDS), gy, ic<1>());
      side(load_aquad(B + gz * RTL_QUAD_WORDS), gz, ic<2>());
    }
    return;
  }
  const uint32_t ty = N[rec] & 0xffu;
  if (ty == RTL_SPHERE) {
    const gptr X = N + rec;
    d3 c = ld3(X, 0);
    if (X[0] & RTL_SPHERE_MOVING) c = vfma(tm, ld3(X, 4), c);
    const double rad = ldd(X, 3);
    const d3 oc = o - c;
    const double a = dot(d, d);
    const double half_b = dot(oc, d);
    const double cc = dot(oc, oc) - rad * rad;
    const double disc = fma(half_b, half_b, -(a * cc));
    const bool real = !(disc < 0.0);
    const double sqrtd = sqrt_nr(disc);
    const double ra = rcp_nr(a);
    const double nr = (-half_b - sqrtd) * ra;
    const double fr = (sqrtd - half_b) * ra;
    const bool in_n = (tmin < nr) & (nr < kInf), in_f = (tmin < fr) & (fr < kInf);
    cand(real & (in_n | in_f), in_n ? nr : fr, rec);
  } else {
    const bool batch = ty == RTL_QUADS;
    const uint32_t cnt = batch ? (N[rec] >> 8) : 1u;
    gptr Q = batch ? N + rec + 4 : N + rec;
    uint32_t qrec = batch ? rec + 4 : rec;
    // the next quad's axis-aligned form is loaded while this one is tested (past the batch's
    // last quad the load reads the following record or the allocation's 256-byte tail, unused;
    // C4 -1 %, profiles/r03_ab_c4_variants.log)
    // (Loading the record's first 80 bytes before its type is known, to start a sphere or a
    // batch in one round trip, measured no faster: profiles/r03_ab_c4_leaf_variants.log.)
    AQuad qn = load_aquad(Q);
    for (uint32_t k = 0; k < cnt; ++k, Q += RTL_QUAD_WORDS, qrec += RTL_QUAD_WORDS) {
      const AQuad q = qn;
      qn = load_aquad(Q + RTL_QUAD_WORDS);
      const uint32_t axis = RTL_QUAD_AXIS(q.h0);
      double t, dk;
      bool inr;
      if (axis == 1u) {
        aquad_core<0>(q, o, d, r, t, inr);
        dk = d.x;
      } else if (axis == 2u) {
        aquad_core<1>(q, o, d, r, t, inr);
        dk = d.y;
      } else if (axis == 3u) {
        aquad_core<2>(q, o, d, r, t, inr);
        dk = d.z;
      } else {  // quad_test's arithmetic (object.rs:453-490)
        const gptr G = Q + RTL_QUAD_GEN;
        const d3 n = ld3(G, 0);
        dk = dot(n, d);
        t = div_nr(ldd(G, 3) - dot(n, o), dk);
        const d3 pq = vfma(t, d, o) - ld3(G, 4);
        const double a = dot(pq, ld3(G, 8)), b = dot(pq, ld3(G, 12));
        const double lo = __builtin_fmin(a, b), hi = __builtin_fmax(a, b);
        inr = !(lo < 0.0) & !(1.0 < hi);
      }
      // (a t of +inf needs no test of its own: no walker's candidate logic can take it)
      cand(!(fabs(dk) < 1e-8) & (tmin <= t) & inr, t, qrec);
    }
  }
}

template <bool MAIN>
__device__ bool obvh_walk(const TraceParams& P, uint32_t ob, d3 o, d3 d, double tm, int frame,
                          double tmin, double tmax, double& t_out, uint32_t& hit_node,
                          int& hit_frame, bool& flag) {
  const gptr N = (gptr)P.nodes;
  const uint4 hd = ld4u(N + ob);  // n_entries, 0, 0, streams_off
  const d3 inv = mk(rcp_w(d.x), rcp_w(d.y), rcp_w(d.z));
  // octant by sign bit (1/-0 = -inf: the near bound of that axis is its max)
  const uint32_t oct = (inv.x < 0.0 ? 1u : 0u) | (inv.y < 0.0 ? 2u : 0u) | (inv.z < 0.0 ? 4u : 0u);
  const uint4* S = reinterpret_cast<const uint4*>(N + ob + hd.w) + (size_t)oct * hd.x * 2;
  const d3 r = mk(rcp_nr1(d.x), rcp_nr1(d.y), rcp_nr1(d.z));
  // Box steps in f32 (the bounds were rounded outwards with a 2^-18 (1 + |coord|) margin,
  // rt_obvh.cpp). Error budget of a slab time t_a = (bound - o_a) * inv_a: the f32 roundings
  // of o (2^-24 |o_a| <= 2^-24 (|bound| + |bound - o_a|): the first part is inside the margin,
  // the second is relative to t_a), of inv, of the difference and of the product: a few 2^-24
  // relative, so the interval is widened by kBoxRel = 2^-20 on both ends. Culling therefore
  // never drops a box holding a candidate <= closest * (1 + kTieRel).
  constexpr float kBoxRel = 0x1p-20f;
  const float ox = (float)o.x, oy = (float)o.y, oz = (float)o.z;
  const float ix = (float)inv.x, iy = (float)inv.y, iz = (float)inv.z;
  const f32x2 ox2 = {ox, ox}, oy2 = {oy, oy}, oz2 = {oz, oz};
  const f32x2 ix2 = {ix, ix}, iy2 = {iy, iy}, iz2 = {iz, iz};
  const float tmin_f = (float)(tmin - fabs(tmin) * 0x1p-20);
  double closest = tmax;
  float close_f = (float)(closest + closest * (2.0 * kTieRel));
  bool hit = false;
  double tie_at = -1.0;  // running closest at the latest near-tie (the winner's t or earlier)
  uint32_t hn = 0;
  uint32_t e = 0;
#ifdef RT_PROF  // profiling build: per-lane box steps / leaves, wave maxima, wave cycles
  uint32_t pf_box = 0, pf_leaf = 0;
  const unsigned long long pf_t0 = __builtin_readcyclecounter();
#endif
  // one candidate: a near-tie test against the running closest, then the strict-min update.
  // Interior faces of touching boxes tie with each other before the ordered walk reaches the
  // nearest hit; only a near-tie AT the final closest t can change the reference's record.
  auto cand = [&](bool valid, double t, uint32_t rec) {
    const bool nt = valid & (closest < kInf) & (fabs(t - closest) <= closest * kTieRel);
    tie_at = nt ? closest : tie_at;
    const bool win = valid & (t < closest);
    closest = win ? t : closest;
    hn = win ? rec : hn;
    hit = hit | win;
  };
  for (;;) {
    uint4 s = make_uint4(0u, 0u, 0u, 0u);
    // while-while: box steps until a leaf (or the end), then the leaves with every lane that has
    // one (as the reference-order LANE walker)
    while (e < hd.x) {
      s = S[2 * e];
      const uint4 s2 = S[2 * e + 1];
      // (near, far) bound pairs: one packed f32 subtract and multiply per axis (v_pk_add_f32,
      // v_pk_mul_f32), the same two roundings per slab time as the scalar form
      const f32x2 bx = {__uint_as_float(s.z), __uint_as_float(s.w)};
      const f32x2 by = {__uint_as_float(s2.x), __uint_as_float(s2.y)};
      const f32x2 bz = {__uint_as_float(s2.z), __uint_as_float(s2.w)};
      const f32x2 tx2 = (bx - ox2) * ix2, ty2 = (by - oy2) * iy2, tz2 = (bz - oz2) * iz2;
      const float tnx = tx2.x, tfx = tx2.y, tny = ty2.x, tfy = ty2.y, tnz = tz2.x, tfz = tz2.y;
      // fmaxf / fminf drop a NaN bound (o on the bound's plane with inv = +-inf): no constraint
      const float tn = fmaxf(fmaxf(tmin_f, tnx), fmaxf(tny, tnz));
      const float tf = fminf(fminf(close_f, tfx), fminf(tfy, tfz));
      const bool pass = fmaf(-fabsf(tn), kBoxRel, tn) <= fmaf(fabsf(tf), kBoxRel, tf);
      const bool leaf = (s.x & 0x80000000u) != 0u;
      if (leaf & pass) break;  // the leaf's own box is hit: test its record
      e = (pass | leaf) ? e + 1u : s.x;
#ifdef RT_PROF
      ++pf_box;
#endif
    }
    if (e >= hd.x) break;
    const uint32_t rec = s.y;
    const double closest_before = closest;
    obvh_leaf(N, rec, o, d, r, tm, tmin, cand);
    if (closest != closest_before) close_f = (float)(closest + closest * (2.0 * kTieRel));
    ++e;
#ifdef RT_PROF
    ++pf_leaf;
#endif
  }
  flag = ((tie_at >= 0.0) & (fabs(tie_at - closest) <= closest * (2.0 * kTieRel))) |
         (hit & (closest <= tmin * (1.0 + kTieRel)));
#ifdef RT_PROF
  {
    const unsigned long long dt = __builtin_readcyclecounter() - pf_t0;
    uint32_t mb = pf_box, ml = pf_leaf, sb = pf_box, sl = pf_leaf;  // wave max and sum
    for (int k = 32; k > 0; k >>= 1) {
      mb = max(mb, (uint32_t)__shfl_xor((int)mb, k));
      ml = max(ml, (uint32_t)__shfl_xor((int)ml, k));
      sb += (uint32_t)__shfl_xor((int)sb, k);
      sl += (uint32_t)__shfl_xor((int)sl, k);
    }
    // P.ops[40 + ...] (past the pool-queue word; rt_scene_prof_counters): per walk kind
    // (0: world frame, 1: instance frame) 6 counters
    unsigned long long* pc = P.ops + 40 + (frame < 0 ? 0 : 6);
    const unsigned long long fl = __popcll(__ballot(flag));
    if (prof_first_lane()) {
      atomicAdd(&pc[0], (unsigned long long)sb);
      atomicAdd(&pc[2], (unsigned long long)sl);
      atomicAdd(&pc[1], (unsigned long long)mb);
      atomicAdd(&pc[3], (unsigned long long)ml);
      atomicAdd(&pc[4], 1ull);
      atomicAdd(&pc[5], dt);
      atomicAdd(&P.ops[52], fl);  // lanes flagged for the reference-order re-walk
    }
  }
#endif
  if (hit) {
    t_out = closest;
    if (MAIN) {
      hit_node = hn;
      hit_frame = frame;
    }
  }
  return hit;
}

// The same walk over the tree's compact copy in LDS (rt_layout.h CBVH): a node holds both
// children's boxes, both are tested in one step, the nearer hit child is visited first and the
// other pushed on the lane's u16 stack in LDS. The box arithmetic (outward-rounded f32 bounds, the
// octant's near/far bound per axis, the kBoxRel widening), the candidates (obvh_leaf) and the
// tie flags are obvh_walk's, so the result is the same closest candidate and the same flag; only
// the order of the steps and where the nodes come from differ. The LDS copy turns the walk's
// dependent L2 round trips (~1 us each, the kernel waited on memory about half its cycles) into
// LDS reads, and a step covers two boxes.
// TPOS (tmin >= 0, every walk but a ConstantMedium boundary's): entry times are then >= 0 and a
// box passes when tn <= tf * kBoxPos, one product for box()'s two widenings. It keeps every box
// the widened test keeps: that test passing means tn (1 - 2^-20)(1 - u) <= tf (1 + 2^-20)(1 + u)
// (u = 2^-24, one rounding each), i.e. tn <= tf (1 + 2^-19 + 2u + ...) <= fl(tf * kBoxPos).
template <bool MAIN, bool TPOS>
__device__ bool cbvh_walk_t(const TraceParams& P, uint4 hd, d3 o, d3 d, double tm, int frame,
                          double tmin, double tmax, double& t_out, uint32_t& hit_node,
                          int& hit_frame, bool& flag) {
  typedef const __attribute__((address_space(3))) uint8_t* lb_t;
  typedef __attribute__((address_space(3))) uint8_t* lbw_t;
  typedef const __attribute__((address_space(3))) uint32_t* lw_t;
  const gptr N = (gptr)P.nodes;
  const uint32_t n_int = (hd.x - 1u) >> 1;  // n_entries = 2 n_leaf - 1
  const lb_t base = (lb_t)rt_lds + P.cbvh_lds_off + hd.y;
  const lw_t refs = reinterpret_cast<lw_t>(base + (size_t)n_int * 48u);
  const lw_t leaves = refs + n_int;
  // the lane's stack entries are blockDim.x u32 apart; sp is kept as a byte offset (a step adds
  // or subtracts sstep instead of multiplying an entry count by the stride). An entry holds the
  // pending child's reference (low 16 bits) and its box's entry time tn as bf16 (high 16 bits:
  // f32 truncated, which rounds a tn >= 0 down; a negative tn is stored as -inf), so that a pop
  // can drop a child whose box no longer passes against the CURRENT closest without reading its
  // node (see pop below).
  typedef __attribute__((address_space(3))) uint32_t* ls_t;
  const lbw_t stack_b = (lbw_t)rt_lds + P.stack_lds_off + 4u * threadIdx.x;
  const uint32_t sstep = 4u * blockDim.x;
  auto slot = [&](uint32_t off) { return reinterpret_cast<ls_t>(stack_b + off); };
  const d3 r = mk(rcp_nr1(d.x), rcp_nr1(d.y), rcp_nr1(d.z));
  // The f32 slab reciprocals from the leaves' f64 ones (rcp_nr1, within an ulp of 1/d, then
  // rounded to f32 like 1/d itself: inside the box test's 2^-18 budget). d_a = +-0 gives NaN
  // there (rcp_nr1's 0 * inf), and a NaN slab time constrains nothing: every box is kept on
  // that axis, never dropped. The octant is d's sign bit (-0: the d_a < 0 side, as 1/-0 = -inf).
  const bool nx = __builtin_signbit(d.x), ny = __builtin_signbit(d.y), nz = __builtin_signbit(d.z);
  const float ix = (float)r.x, iy = (float)r.y, iz = (float)r.z;
  constexpr float kBoxRel = 0x1p-20f;
  constexpr float kBoxPos = 1.0f + 0x1p-18f;
  const float ox = (float)o.x, oy = (float)o.y, oz = (float)o.z;
  // slab times as fma(bound, inv, -o inv): one packed fma per axis instead of a subtraction and
  // a product. The extra rounding of o inv is 2^-24 |o inv| <= 2^-24 (|bound| + |bound - o|) |inv|,
  // the same two parts as o's own rounding (obvh_walk's budget): inside the bounds' margin and
  // relative to t. A NaN slab time (0 * inf, inf - inf: d_a = 0) constrains nothing (fmaxf /
  // fminf drop it), so such boxes are kept, never dropped.
  const f32x2 ix2 = {ix, ix}, iy2 = {iy, iy}, iz2 = {iz, iz};
  const f32x2 nox2 = {-(ox * ix), -(ox * ix)}, noy2 = {-(oy * iy), -(oy * iy)},
              noz2 = {-(oz * iz), -(oz * iz)};
  const float tmin_f = (float)(tmin - fabs(tmin) * 0x1p-20);
  double closest = tmax;
  float close_f = (float)(closest + closest * (2.0 * kTieRel));
  bool hit = false;
  // The tie flag from the two smallest values of {tmax, every candidate}: `closest` is the
  // smallest, `second` the next. obvh_walk flags a lane when a candidate came within kTieRel of
  // the running closest and that closest is within 2 kTieRel of the final one; any such pair
  // (the running closest a, the candidate b) makes the two smallest values lie within
  // 2 kTieRel (+ roundings) of each other, so testing second <= closest (1 + 3 kTieRel) flags
  // every lane obvh_walk flags (and at most a few more, which re-walk in the reference order).
  // A candidate then costs a min, a max and the winner's selects, not the tie test's four.
  double second = kInf;
  uint32_t hn = 0;
  auto cand = [&](bool valid, double t, uint32_t rec) {
    const double te = valid ? t : kInf;
    second = fmin(second, fmax(closest, te));
    const bool win = te < closest;
    closest = win ? te : closest;
    hn = win ? rec : hn;
    hit = hit | win;
  };
  // slab test of one child box [lo_x hi_x lo_y hi_y lo_z hi_z]: the octant's near bound per axis
  // is hi where d_a < 0, as in the OBVH streams
  // A node stores each axis's bounds as [lo c0, lo c1, hi c0, hi c1] (rt_layout.h CBVH): the
  // lane reads its octant's near pair and far pair of both children with one 8-byte load each at
  // a per-lane byte offset, and forms both children's slab times of an axis with one packed fma
  // (no per-child select).
  typedef const __attribute__((address_space(3))) f32x2* lf2_t;
  const uint32_t onx = nx ? 8u : 0u, ony = ny ? 24u : 16u, onz = nz ? 40u : 32u;
  auto box = [&](float tnx, float tfx, float tny, float tfy, float tnz, float tfz, float& tn) {
    tn = fmaxf(fmaxf(tmin_f, tnx), fmaxf(tny, tnz));
    const float tf = fminf(fminf(close_f, tfx), fminf(tfy, tfz));
    if constexpr (TPOS) {
      return tn <= tf * kBoxPos;
    } else {
      return fmaf(-fabsf(tn), kBoxRel, tn) <= fmaf(fabsf(tf), kBoxRel, tf);
    }
  };
  constexpr uint32_t kDone = 0xffffu;
  uint32_t ref = hd.z & 0xffffu;
  uint32_t sp = 0;
  auto entry = [](uint32_t child, float tn) {
    return child | (tn < 0.0f ? 0xff800000u : (__float_as_uint(tn) & 0xffff0000u));
  };
  // Pop the next pending child, dropping those whose stored entry time tb fails box()'s test
  // against the current closest: tb <= tn, tf <= close_f, and both sides of the test are
  // monotone, so the child's box fails it, and so do its children's boxes (they lie inside it:
  // entry times no earlier, the same f32 outward-rounded bounds) and a leaf's candidates (the
  // margins that let box() cull a box keep every candidate <= closest (1 + kTieRel) inside its
  // box). The walk visits the same nodes and leaves as with a full step per entry.
  auto pop = [&]() -> uint32_t {
    const float cut = TPOS ? close_f * kBoxPos : fmaf(fabsf(close_f), kBoxRel, close_f);
    while (sp > 0) {
      sp -= sstep;
      const uint32_t e = *slot(sp);
      const float tb = __uint_as_float(e & 0xffff0000u);
      const bool drop = TPOS ? (tb > cut) : (fmaf(-fabsf(tb), kBoxRel, tb) > cut);
      if (!drop) return e & 0xffffu;
    }
    return kDone;
  };
#ifdef RT_PROF  // profiling build: per-lane box steps / leaves, wave maxima, wave cycles (walk, leaves)
  uint32_t pf_box = 0, pf_leaf = 0;
  unsigned long long pf_leaf_cyc = 0;
  const unsigned long long pf_t0 = __builtin_readcyclecounter();
#endif
#ifdef RT_ABL_BUDGET  // ablation build (wrong images): a top-level walk stops after RT_ABL_BUDGET
                      // box steps; the time is an upper bound for resumable walks
  uint32_t ab_steps = 0;
#endif
  for (;;) {
    // while-while: steps until the lane holds a leaf whose box was hit (or is done), then the
    // leaves with every lane that has one. (Postponing a lane's leaf and stepping on until every
    // lane holds one -- speculative while-while -- was 11 % slower at C4: more steps against an
    // older closest t.)
    while (ref < 0x8000u) {
#ifdef RT_ABL_BUDGET
      if (frame < 0 && ++ab_steps > RT_ABL_BUDGET) {
        ref = kDone;
        sp = 0;
        break;
      }
#endif
      const lb_t nb = base + ref * 48u;
      const f32x2 NX = *reinterpret_cast<lf2_t>(nb + onx), FX = *reinterpret_cast<lf2_t>(nb + (onx ^ 8u));
      const f32x2 NY = *reinterpret_cast<lf2_t>(nb + ony), FY = *reinterpret_cast<lf2_t>(nb + (ony ^ 8u));
      const f32x2 NZ = *reinterpret_cast<lf2_t>(nb + onz), FZ = *reinterpret_cast<lf2_t>(nb + (onz ^ 8u));
      const uint32_t rr = refs[ref];
      const f32x2 tnx = __builtin_elementwise_fma(NX, ix2, nox2), tfx = __builtin_elementwise_fma(FX, ix2, nox2);
      const f32x2 tny = __builtin_elementwise_fma(NY, iy2, noy2), tfy = __builtin_elementwise_fma(FY, iy2, noy2);
      const f32x2 tnz = __builtin_elementwise_fma(NZ, iz2, noz2), tfz = __builtin_elementwise_fma(FZ, iz2, noz2);
      float tn0, tn1;
      const bool h0 = box(tnx.x, tfx.x, tny.x, tfy.x, tnz.x, tfz.x, tn0);
      const bool h1 = box(tnx.y, tfx.y, tny.y, tfy.y, tnz.y, tfz.y, tn1);
      // Logical (not bitwise) operators on the hit flags: `h0 & h1` on bools is int arithmetic,
      // which the compiler kept as 0/1 values in VGPRs (two v_cndmask, two v_and and a v_cmp per
      // step); with && / || the flags stay lane masks in SGPRs (C4 -2.7 %, r04_ab16_c4_steps.log).
      const bool first0 = h0 && (!h1 || (tn0 <= tn1));
      const uint32_t r0 = rr & 0xffffu, r1 = rr >> 16;
      const bool any = h0 || h1;
      const uint32_t nref = first0 ? r0 : r1;
      // Both children hit: visit the nearer, push the other. The far entry is written to the
      // free slot every step and kept (sp advanced) only then: no branch around the store. The
      // slot is inside the lane's stack: at an internal node of depth k the stack holds at most
      // k - 1 entries (pending siblings of its ancestors) and holds depth-of-tree slots. (The
      // round-3 branch-free form also read the top speculatively: 3.5 % slower,
      // r03_ab_cbvh_branchfree_c4; this one -0.7 %, r04_ab15_c4_steps.log.)
      *slot(sp) = first0 ? entry(r1, tn1) : entry(r0, tn0);
      sp += (h0 && h1) ? sstep : 0u;
      ref = any ? nref : pop();
#ifdef RT_PROF
      ++pf_box;
#endif
    }
    if (ref == kDone) break;
#ifdef RT_PROF
    ++pf_leaf;
    const unsigned long long pf_l0 = __builtin_readcyclecounter();
#endif
#ifdef RT_ABL_LEAF2  // ablation build: every leaf tested twice (same result); the delta is their cost
    {
      double z = 0.0;
      asm volatile("" : "+v"(z));
      bool any = false;
      auto nop = [&](bool v, double t, uint32_t) { any = any | (v & (t > z)); };
      obvh_leaf(N, leaves[ref & 0x7fffu], o, d, r, tm, tmin + z, nop);
      asm volatile("" ::"v"(any));
    }
#endif
    const double closest_before = closest;
    obvh_leaf(N, leaves[ref & 0x7fffu], o, d, r, tm, tmin, cand);
    if (closest != closest_before) close_f = (float)(closest + closest * (2.0 * kTieRel));
#ifdef RT_PROF
    pf_leaf_cyc += __builtin_readcyclecounter() - pf_l0;
#endif
    ref = pop();
  }
  flag = ((second < kInf) & (second <= closest * (1.0 + 3.0 * kTieRel))) |
         (hit & (closest <= tmin * (1.0 + kTieRel)));
#ifdef RT_PROF
  {
    const unsigned long long dt = __builtin_readcyclecounter() - pf_t0;
    uint32_t mb = pf_box, ml = pf_leaf, sb = pf_box, sl = pf_leaf;  // wave max and sum
    for (int k = 32; k > 0; k >>= 1) {
      mb = max(mb, (uint32_t)__shfl_xor((int)mb, k));
      ml = max(ml, (uint32_t)__shfl_xor((int)ml, k));
      sb += (uint32_t)__shfl_xor((int)sb, k);
      sl += (uint32_t)__shfl_xor((int)sl, k);
    }
    unsigned long long* pc = P.ops + 40 + (frame < 0 ? 0 : 6);
    const unsigned long long fl = __popcll(__ballot(flag));
    if (prof_first_lane()) {
      atomicAdd(&pc[0], (unsigned long long)sb);
      atomicAdd(&pc[2], (unsigned long long)sl);
      atomicAdd(&pc[1], (unsigned long long)mb);
      atomicAdd(&pc[3], (unsigned long long)ml);
      atomicAdd(&pc[4], 1ull);
      atomicAdd(&pc[5], dt);
      atomicAdd(&P.ops[52], fl);
      atomicAdd(&P.ops[53 + (frame < 0 ? 0 : 1)], pf_leaf_cyc);  // lane 0's cycles in leaf tests
    }
  }
#endif
  if (hit) {
    t_out = closest;
    if (MAIN) {
      hit_node = hn;
      hit_frame = frame;
    }
  }
  return hit;
}
template <bool MAIN>
__device__ __forceinline__ bool cbvh_walk(const TraceParams& P, uint4 hd, d3 o, d3 d, double tm,
                                          int frame, double tmin, double tmax, double& t_out,
                                          uint32_t& hit_node, int& hit_frame, bool& flag) {
  return tmin >= 0.0 ? cbvh_walk_t<MAIN, true>(P, hd, o, d, tm, frame, tmin, tmax, t_out,
                                               hit_node, hit_frame, flag)
                     : cbvh_walk_t<MAIN, false>(P, hd, o, d, tm, frame, tmin, tmax, t_out,
                                                hit_node, hit_frame, flag);
}

template <bool MAIN, bool COUNT, bool VOLB, bool BVH>
__device__ bool bvh_subtree(const TraceParams& P, uint32_t node, uint32_t stop, uint32_t obvh,
                            d3 wo, d3 wd, double tm, d3 o, d3 d, int frame, double tmin,
                            double tmax, double& t_out, uint32_t& hit_node, int& hit_frame,
                            Rng& g, Ctr<COUNT>& C) {
#ifdef RT_ABL_TWICE_BVH  // ablation build: the top-level (1) / in-instance (2) ordered-BVH walk
                         // runs twice (same image); the time delta is one walk's cost
  if (!COUNT && obvh != 0u &&
      ((RT_ABL_TWICE_BVH == 1 && frame < 0) || (RT_ABL_TWICE_BVH == 2 && frame >= 0))) {
    double t2 = 0.0, z = 0.0;
    uint32_t hn2 = 0;
    int hf2 = -1;
    bool f2 = false;
    asm volatile("" : "+v"(z));
    const uint4 hd2 = ld4u((gptr)P.nodes + obvh);
    const bool h2 = (P.cbvh_lds_off != ~0u && hd2.y != ~0u)
                        ? cbvh_walk<MAIN>(P, hd2, o, d, tm, frame, tmin + z, tmax, t2, hn2, hf2, f2)
                        : obvh_walk<MAIN>(P, obvh, o, d, tm, frame, tmin + z, tmax, t2, hn2, hf2, f2);
    asm volatile("" ::"v"(t2), "v"(hn2), "v"(h2), "v"(f2));
  }
#endif
  if constexpr (!COUNT) {
    if (obvh != 0u && !(P.flags & RT_FLAG_REFERENCE_BVH)) {
      bool flag = false;
      const uint4 hd = ld4u((gptr)P.nodes + obvh);  // [n_entries][cbvh block][root ref][streams]
      bool h;
      if (P.cbvh_lds_off != ~0u && hd.y != ~0u)  // the compact copy in LDS
        h = cbvh_walk<MAIN>(P, hd, o, d, tm, frame, tmin, tmax, t_out, hit_node, hit_frame, flag);
      else
        h = obvh_walk<MAIN>(P, obvh, o, d, tm, frame, tmin, tmax, t_out, hit_node, hit_frame,
                            flag);
      if (__ballot(flag) != 0ull && flag)  // rare: the reference order decides
        h = traverse<MAIN, COUNT, VOLB, false, BVH>(P, node, stop, wo, wd, tm, o, d, frame, tmin,
                                                    tmax, t_out, hit_node, hit_frame, g, C);
      return h;
    }
  }
  return traverse<MAIN, COUNT, VOLB, false, BVH>(P, node, stop, wo, wd, tm, o, d, frame, tmin,
                                                 tmax, t_out, hit_node, hit_frame, g, C);
}

// ---------------------------------------------------------------- textures
// Rust `as i32` / `as u32` (truncation, saturation at the type's range, NaN -> 0) is exactly what
// v_cvt_i32_f64 / v_cvt_u32_f64 compute; C++ leaves out-of-range conversions undefined, so the
// instructions are issued directly (the compiler made each range check a branch; C4 -1.4 %,
// profiles/r06i_ab_noise_c4.log; tests/test_gpu_parity.py::test_saturating_texture_coordinates)
__device__ __forceinline__ int32_t f2i_sat(double f) {
  int32_t r;
  asm("v_cvt_i32_f64 %0, %1" : "=v"(r) : "v"(f));
  return r;
}
__device__ __forceinline__ uint32_t f2u_sat(double f) {
  uint32_t r;
  asm("v_cvt_u32_f64 %0, %1" : "=v"(r) : "v"(f));
  return r;
}

// Perlin::turb perlin.rs:56-72 over noise 30-54 + trilinear_interp 74-96. T = one table
// (RTL_PERLIN_BYTES: ranvec as 256 float4, then perm_x/y/z), normally the workgroup's LDS copy
// (rt_trace stages the scene's first kPerlinLds tables at launch). The turbulence only colours a
// noise texture (a weight, rt_kernel.h wt), so it is computed in f32 -- except the lattice cell
// and the offset in it: floor(p) and p - floor(p) are exact in f64 (p doubles per octave, also
// exact), so every lane reads the reference's eight corners; the offsets are then rounded to f32.
// The octave loop stays rolled and each octave reads the six permutation entries once, so the
// eight corner gathers (one 16-byte read each) are the only wide live values.
__device__ __forceinline__ float perlin_turb(const uint8_t* __restrict__ T, d3 p) {
  const float4* rv = reinterpret_cast<const float4*>(T);
  const uint8_t* px = T + 4096;
  const uint8_t* py = px + 256;
  const uint8_t* pz = py + 256;
  float accum = 0.0f, weight = 1.0f;
#pragma unroll 1
  for (int oct = 0; oct < 7; ++oct) {
    const double fx = floor(p.x), fy = floor(p.y), fz = floor(p.z);
    const float u = (float)(p.x - fx), v = (float)(p.y - fy), w = (float)(p.z - fz);
    const uint32_t i = (uint32_t)f2i_sat(fx), j = (uint32_t)f2i_sat(fy), k = (uint32_t)f2i_sat(fz);
    const uint32_t X[2] = {px[i & 255u], px[(i + 1u) & 255u]};
    const uint32_t Y[2] = {py[j & 255u], py[(j + 1u) & 255u]};
    const uint32_t Z[2] = {pz[k & 255u], pz[(k + 1u) & 255u]};
    const float uu = u * u * (3.0f - 2.0f * u);
    const float vv = v * v * (3.0f - 2.0f * v);
    const float ww = w * w * (3.0f - 2.0f * w);
    // trilinear_interp (perlin.rs:74-96): the sum over the eight corners of
    // (i uu + (1-i)(1-uu)) (j vv + (1-j)(1-vv)) (k ww + (1-k)(1-ww)) (c . (u-i, v-j, w-k)),
    // formed as nested lerps (the same polynomial; 7 lerps instead of 8 weight products, within
    // noise of them at C4: profiles/r06i_ab_noise_c4.log)
    float dd[2][2][2];
#pragma unroll
    for (int di = 0; di < 2; ++di)
#pragma unroll
      for (int dj = 0; dj < 2; ++dj)
#pragma unroll
        for (int dk = 0; dk < 2; ++dk) {
          const float4 c = rv[X[di] ^ Y[dj] ^ Z[dk]];
          dd[di][dj][dk] = fmaf(c.x, u - (float)di, fmaf(c.y, v - (float)dj, c.z * (w - (float)dk)));
        }
    auto lerp = [](float a, float b, float t) { return fmaf(t, b - a, a); };
    const float x0 = lerp(lerp(dd[0][0][0], dd[0][0][1], ww), lerp(dd[0][1][0], dd[0][1][1], ww), vv);
    const float x1 = lerp(lerp(dd[1][0][0], dd[1][0][1], ww), lerp(dd[1][1][0], dd[1][1][1], ww), vv);
    const float acc = lerp(x0, x1, uu);
    accum = fmaf(weight, acc, accum);
    weight *= 0.5f;
    p = p * 2.0;
  }
  return fabsf(accum);
}
// Tables past the LDS-staged ones (scenes with more than kPerlinLds noise textures): global.
__device__ __noinline__ float perlin_turb_global(const uint8_t* __restrict__ T, d3 p) {
  return perlin_turb(T, p);
}

template <bool COUNT, bool TEX, class TT>
__device__ d3 tex_value(const TraceParams& P, const TT& T, uint32_t id, double u, double v,
                        d3 p, Ctr<COUNT>& C) {
  if (!TEX) return ld3(T.texs + (size_t)id * RTL_TEX_WORDS, 0);
  for (int guard = 0; guard < 65; ++guard) {
    const auto t = T.texs + (size_t)id * RTL_TEX_WORDS;
    uint4 h = ld4u(t);
    if (h.x == RT_TEX_SOLID) return ld3(t, 0);
    if (h.x == RT_TEX_CHECKER) {  // texture.rs:71-81
      double is = ldd(t, 0);
      int32_t x = f2i_sat(floor(is * p.x));
      int32_t y = f2i_sat(floor(is * p.y));
      int32_t z = f2i_sat(floor(is * p.z));
      uint32_t sum = (uint32_t)x + (uint32_t)y + (uint32_t)z;
      id = (sum & 1u) == 0u ? h.y : h.z;
      continue;
    }
    if (h.x == RT_TEX_IMAGE) {  // texture.rs:95-107, rt_image.rs:37-46
      int W = (int)h.y, H = (int)h.z;
      if (H <= 0 || W <= 0) return mk(0., 1., 1.);
      double cu = u < 0.0 ? 0.0 : (u > 1.0 ? 1.0 : u);
      double cv = v < 0.0 ? 0.0 : (v > 1.0 ? 1.0 : v);
      uint32_t i = f2u_sat(cu * (double)W);
      uint32_t j = f2u_sat(cv * (double)H);
      uint32_t x = i < (uint32_t)(W - 1) ? i : (uint32_t)(W - 1);
      uint32_t y = (uint32_t)H - j - 1u;
      if (y > (uint32_t)(H - 1)) y = (uint32_t)(H - 1);
      const uint8_t* px = P.texels + h.w + ((size_t)y * W + x) * 3;
      const double cs = 1.0 / 255.0;
      return mk((double)px[0] * cs, (double)px[1] * cs, (double)px[2] * cs);
    }
    if (h.x == RT_TEX_NOISE) {  // texture.rs:127-130
      C.inc(RT_OP_NOISE_EVALS);
      d3 s = p * ldd(t, 0);
      const float turb = h.y < P.n_perlin_lds
                        ? perlin_turb(T.perlin + (size_t)h.y * RTL_PERLIN_BYTES, s)
                        : perlin_turb_global(P.perlin + (size_t)h.y * RTL_PERLIN_BYTES, s);
#ifdef RT_ABL_NOISE2  // ablation build: the turbulence evaluated twice (same result; its cost)
      {
        d3 s2 = s;
        asm volatile("" : "+v"(s2.x));
        const float t2 = perlin_turb(T.perlin + (size_t)h.y * RTL_PERLIN_BYTES, s2);
        asm volatile("" ::"v"(t2));
      }
#endif
      double k = 0.5 * (1.0 + sin(fma(10.0, (double)turb, s.z)));
      return mk(k, k, k);
    }
    break;
  }
  return mk(0., 0., 0.);
}

// get_sphere_uv object.rs:114-120 (out of line: only image-textured spheres need it; (u, v)
// come back in registers, not through a stack slot)
struct UV {
  double u, v;
};
__device__ __noinline__ UV sphere_uv_f(d3 p) {
  double theta = acos(-p.y);
  double phi = atan2(-p.z, p.x) + kPi;
  return {phi * (1.0 / kPi) * 0.5, theta * (1.0 / kPi)};
}
__device__ __forceinline__ void sphere_uv(d3 p, double& u, double& v) {
  const UV r = sphere_uv_f(p);
  u = r.u;
  v = r.v;
}

// ---------------------------------------------------------------- sampling
struct Onb {
  d3 u, v, w;
};
// onb.rs:24-26 evaluates a*u + b*v + c*w left to right, (a*u + b*v) + c*w: the same association
// here, each sum fused with its product
__device__ __forceinline__ d3 onb_local(const Onb& b, d3 a) {
  return vfma(a.z, b.w, vfma(a.x, b.u, b.v * a.y));
}
__device__ __forceinline__ d3 random_cosine_direction(Rng& g) {  // vec3.rs:240-250
  double r1 = rnd(g);
  double r2 = rnd(g);
  double s, c;
  sincos2pi(r1, &s, &c);
  double sq = sqrt_nr(r2);
  return mk(c * sq, s * sq, sqrt_nr(1.0 - r2));
}
__device__ __forceinline__ d3 random_unit_vector(Rng& g) {  // vec3.rs:215-217, 231-238
  for (;;) {
    double x = rnd_pm1(g);
    double y = rnd_pm1(g);
    double z = rnd_pm1(g);
    d3 p = mk(x, y, z);
    if (dot(p, p) < 1.0) return unit_vector(p);
  }
}

// Quad::pdf_value's weight after its f64 hit test (object.rs:492-501): dist2 / (cosine * area)
// with dist2 = t^2 |d|^2 and cosine = |d . n| / |d| (shared by the interpreter and the generated
// light-list PDF, rt_jit.cpp, so that both kernels compute the same bits)
__device__ __forceinline__ wt quad_light_w(d3 dir, double t, d3 n, double area) {
#ifdef RT_F64W
  const double len2 = dot(dir, dir);
  const double dist2 = (t * t) * len2;
  const double cosine = fabs(dot(dir, n)) * rsq_nr(len2);
  return dist2 * rcp_w(cosine * area);
#else
  const w3 d = to_w3(dir), nf = to_w3(n);
  const float len2 = fmaf(d.x, d.x, fmaf(d.y, d.y, d.z * d.z));
  const float tf = (float)t;
  const float cosine = fabsf(fmaf(d.x, nf.x, fmaf(d.y, nf.y, d.z * nf.z))) * rsq_wt(len2);
  return ((tf * tf) * len2) * rcp_wt(cosine * (float)area);
#endif
}
// Sphere::pdf_value's weight (object.rs:190-202): 1 / (2 pi (1 - cos_theta_max)); 1 - cos in f64
// (a small, distant sphere's cos_theta_max is within a few f32 ulps of 1)
__device__ __forceinline__ wt sphere_light_w(double cos_max) {
  return rcp_wt((wt)(2.0 * kPi) * (wt)(1.0 - cos_max));
}

// Light-list PDF value (HittablePDF::value pdf.rs:91-93 -> HittableList::pdf_value
// hittable.rs:115-124 -> Quad/Sphere::pdf_value object.rs:492-501, 190-202).
// cos_sl0: cos_theta_max of the first sphere light at `origin` (object.rs:196), computed once per
// bounce by the caller and shared with Sphere::random (the same expression, the same bits).
template <bool COUNT>
__device__ wt light_leaf_pdf(const TraceParams& P, uint32_t i, d3 origin, d3 dir,
                             double cos_sl0, Ctr<COUNT>& C) {
  const kptr L = (kptr)P.lights + ((kptr)P.light_offs)[i];
  uint32_t type = L[0] & 0xffu;
  wt pv = 0;
  if (type == RTL_QUAD) {
    C.inc(RT_OP_LIGHT_PDF_QUAD);
    double t = 0.0;
    bool hq;
    const uint32_t axis = RTL_QUAD_AXIS(L[0]);
    if (axis) {  // axis-aligned form at d24 (rt_layout.h): the world quads' bit-identical test
      const kdptr A = reinterpret_cast<kdptr>(L + 4) + RTL_LQUAD_AXIS_D;
      const AQuad q = {L[0], A[0], A[1], A[2], A[3], A[4]};
      if (axis == 1u) {
        hq = aquad_test<COUNT, 0>(q, origin, dir, mk(rcp_nr1(dir.x), 0., 0.), 0.001, kInf, t, C);
      } else if (axis == 2u) {
        hq = aquad_test<COUNT, 1>(q, origin, dir, mk(0., rcp_nr1(dir.y), 0.), 0.001, kInf, t, C);
      } else {
        hq = aquad_test<COUNT, 2>(q, origin, dir, mk(0., 0., rcp_nr1(dir.z)), 0.001, kInf, t, C);
      }
    } else {
      hq = quad_test<COUNT>(L, origin, dir, 0.001, kInf, t, C);
    }
    {
      const wt q = quad_light_w(dir, t, ld3(L, 0), ldd(L, 7));
      pv = hq ? q : (wt)0;
    }
  } else if (type == RTL_SPHERE) {
    C.inc(RT_OP_LIGHT_PDF_SPHERE);
    bool hs;
    if (COUNT) {
      double t = 0.0;
      hs = sphere_test<COUNT>(L, origin, dir, 0.0, 0.001, kInf, t, C);
    } else {
      // Only a weight depends on this test (a PDF value), so the product build asks the same
      // question without the root: some root of Sphere::hit lies in (0.001, inf) exactly when
      // the far root does, (sqrt(disc) - half_b) / a > 0.001, i.e. sqrt(disc) > c1 = 0.001 a +
      // half_b: true for c1 < 0, else disc > c1^2 (object.rs:145-166 at time 0, 193).
      const d3 oc = origin - ld3(L, 0);
      const double a = dot(dir, dir);
      const double half_b = dot(oc, dir);
      const double r = ldd(L, 3);
      const double c = dot(oc, oc) - r * r;
      const double disc = fma(half_b, half_b, -(a * c));
      const double c1 = fma(0.001, a, half_b);
      hs = !(disc < 0.0) & ((c1 < 0.0) | (disc > c1 * c1));
    }
    double cos_max = 0.0;
    if ((int)i == P.sphere_light0) {  // uniform: the shared value (straight-line)
      cos_max = cos_sl0;
    } else if (hs) {
      d3 cmo = ld3(L, 0) - origin;
      double r = ldd(L, 3);
      cos_max = sqrt_nr(1.0 - r * r / dot(cmo, cmo));
    }
    const wt q = sphere_light_w(cos_max);
    pv = hs ? q : (wt)0;
  }
  return pv;  // RTL_OTHER (Object::pdf_value's default arm, object.rs:306-311): 0
}
// A light entry: a leaf, or a HittableList nested inside the light list (RTL_LLIST, object.rs:66
// -> hittable.rs:115-124): the left fold of its children's values times 1/len. NEST bounds the
// nesting below this entry (the flattener rejects deeper light lists).
template <bool COUNT, int NEST>
__device__ wt light_entry_pdf(const TraceParams& P, uint32_t i, d3 origin, d3 dir,
                              double cos_sl0, Ctr<COUNT>& C) {
  const kptr L = (kptr)P.lights + ((kptr)P.light_offs)[i];
  if constexpr (NEST > 0) {
    if ((L[0] & 0xffu) == RTL_LLIST) {
      const uint32_t n = L[0] >> 8, first = L[1];
      wt sum = 0;
      for (uint32_t k = 0; k < n; ++k) {
        const wt pv = light_entry_pdf<COUNT, NEST - 1>(P, first + k, origin, dir, cos_sl0, C);
        sum = k == 0 ? pv : sum + pv;
      }
      return sum * (wt)ldd(L, 0);  // weight = 1 / len, the host's IEEE division
    }
  }
  return light_leaf_pdf<COUNT>(P, i, origin, dir, cos_sl0, C);
}
template <bool COUNT>
__device__ wt light_pdf(const TraceParams& P, d3 origin, d3 dir, double cos_sl0,
                        Ctr<COUNT>& C) {
  wt sum = 0;
  for (uint32_t i = 0; i < P.n_lights; ++i) {
    const wt pv = P.lights_nested
                          ? light_entry_pdf<COUNT, RTL_LIGHT_NEST>(P, i, origin, dir, cos_sl0, C)
                          : light_leaf_pdf<COUNT>(P, i, origin, dir, cos_sl0, C);
    sum = i == 0 ? pv : sum + pv;
  }
  return P.lights_is_list ? sum * (wt)P.inv_n_lights : sum;  // weight = 1/len (hittable.rs:116)
}

// The reference's special values (render.rs:287-292). ray_color returns
// (attenuation * scattering_pdf * L_sub) / pdf_val, recursively: a bounce whose mixture PDF value
// is 0 (or NaN) turns the whole sample into inf or NaN per channel, even when the sub-path
// returns 0 (0 / 0 = NaN) -- something the forward beta/L product cannot see, since nothing may
// be added after it. Such a bounce sets RT_XS_ON: from then on the lane traces the sub-path with
// a fresh beta = 1, L = 0, and a channel ends as
//   NaN  if its bit in RT_XS_NAN is set (c = atten * s_pdf is 0 or NaN there: 0 * x / 0, or the
//        prefix throughput is 0 or NaN: 0 * inf), or L_sub is 0 or NaN (0 / 0, NaN / 0);
//   +inf otherwise (x / 0 with x > 0; a later such bounce inside the sub-path resolves the same
//        way, and the finite radiance gathered before it is absorbed by the inf / NaN).
// Radiance is never negative (attenuations, emission and PDFs are >= 0), so no -inf arises.
constexpr uint32_t RT_XS_ON = 8u;
__device__ __forceinline__ uint32_t xs_nan_bits(w3 c, w3 beta) {
  const bool nx = !(c.x != 0.0) | !(beta.x != 0.0);  // 0 or NaN
  const bool ny = !(c.y != 0.0) | !(beta.y != 0.0);
  const bool nz = !(c.z != 0.0) | !(beta.z != 0.0);
  return (nx ? 1u : 0u) | (ny ? 2u : 0u) | (nz ? 4u : 0u);
}
__device__ __forceinline__ double xs_chan(double l, bool nan_bit) {
  const double qnan = __builtin_nan("");
  return (nan_bit | !(l != 0.0)) ? qnan : kInf;  // !(l != 0): 0 or NaN
}
__device__ __forceinline__ d3 xs_resolve(d3 L, uint32_t xs) {
  if (!(xs & RT_XS_ON)) return L;
  return mk(xs_chan(L.x, xs & 1u), xs_chan(L.y, xs & 2u), xs_chan(L.z, xs & 4u));
}

// ---------------------------------------------------------------- the path kernel
// VOL: scene has ConstantMedium nodes; TEX: some material reads a non-solid texture.
// The world query of ray_color (render.rs:267: world.hit(r, Interval(0.001 -> 1e-4, inf))), by
// the run-time interpreter of the flattened node sequence. Scene-specialised kernels (rt_jit.cpp)
// supply a generated policy with the same signature and the same arithmetic.
// VN > 0: the scene nests ConstantMedium records inside volume boundaries (that deep).
// What a scene can contain, as far as the path loop's shading needs to know (a walker's kScene):
// the interpreter walks any scene (every bit set, the run-time checks decide), a scene-specialised
// walker (rt_jit.cpp) clears the bits of what its scene lacks, so the compiler drops that code and
// the register copies its branches would cost. A cleared bit only removes a case that cannot occur.
constexpr uint32_t kScMetal = RTL_SC_METAL, kScDielectric = RTL_SC_DIELECTRIC,
                   kScLight = RTL_SC_LIGHT, kScLights = RTL_SC_LIGHTS, kScLList = RTL_SC_LLIST,
                   kScLSphere = RTL_SC_LSPHERE, kScLOther = RTL_SC_LOTHER, kScAny = RTL_SC_ANY;
template <int VN>
struct TravInterpN {
  static constexpr uint32_t kScene = kScAny;
  template <bool COUNT, bool VOL, bool BVH, bool VOLB, bool VOLI>
  static __device__ __forceinline__ bool world(const TraceParams& P, d3& ro, d3& rd, double tm,
                                               double& t, uint32_t& hn, int& hf, Rng& g,
                                               Ctr<COUNT>& C) {
    return traverse<true, COUNT, VOL, true, BVH, VOLB, VOLI, VN>(P, P.root, ~0u, ro, rd, tm, ro,
                                                                 rd, -1, 0.0001, kInf, t, hn, hf,
                                                                 g, C);
  }
  // the mixture's light-list PDF value (pdf.rs:91-93)
  template <bool COUNT>
  static __device__ __forceinline__ wt lights_pdf(const TraceParams& P, d3 origin, d3 dir,
                                                  double cos_sl0, Ctr<COUNT>& C) {
    return light_pdf<COUNT>(P, origin, dir, cos_sl0, C);
  }
  // the hit record's frame (transform.rs:57-135): the world ray into the winner's frame, and its
  // hit point / normal back out
  template <class TP>
  static __device__ __forceinline__ void frame_in(TP N, int hf, d3 wo, d3 wd, d3& o, d3& d) {
    frame_ray(N, hf, wo, wd, o, d);
  }
  template <class TP>
  static __device__ __forceinline__ void frame_out(TP N, int hf, d3& p, d3& n) {
    rtk::frame_out(N, hf, p, n);
  }
};
typedef TravInterpN<0> TravInterp;

// The path kernel body; instantiated by rt_device.hip (interpreter) and by scene-specialised
// JIT kernels. Its __global__ wrapper passes TraceParams as the only kernel argument (kparams()).
template <bool COUNT, bool VOL, bool TEX, bool BVH, bool STAGED, bool VOLB, bool VOLI, class Trav>
__device__ __forceinline__ void trace_body(const TraceParams& P) {
  // STAGED: the small-table prefix is in LDS (P.stage_scene) and per-lane table reads are
  // ds_reads through 32-bit LDS pointers; otherwise they read the global tables.
  typedef typename cond<STAGED, lptr, gptr>::type TP;
  __shared__ unsigned int sh_ops[COUNT ? RT_OP_COUNT : 1];
  if (COUNT) {
    for (int k = threadIdx.x; k < RT_OP_COUNT; k += blockDim.x) sh_ops[k] = 0u;
    __syncthreads();
  }
  if (P.stage_bytes || (BVH && !P.stage_scene && P.bvh_lds_words) ||
      (BVH && !COUNT && P.cbvh_lds_off != ~0u)) {
    // copy the small tables (or just the Perlin tables) into LDS, then the BVH region
    const uint4* src = reinterpret_cast<const uint4*>(P.stage_src);
    uint4* dst = reinterpret_cast<uint4*>(rt_lds);
    const uint32_t n16 = P.stage_bytes / 16;
    for (uint32_t k = threadIdx.x; k < n16; k += blockDim.x) dst[k] = src[k];
    if (BVH && !P.stage_scene) {
      const uint4* bsrc = reinterpret_cast<const uint4*>(P.nodes);
      uint4* bdst = reinterpret_cast<uint4*>(rt_lds + P.bvh_lds_off);
      const uint32_t b16 = P.bvh_lds_words / 4;
      for (uint32_t k = threadIdx.x; k < b16; k += blockDim.x) bdst[k] = bsrc[k];
    }
    if (BVH && !COUNT && P.cbvh_lds_off != ~0u) {
      const uint4* csrc = reinterpret_cast<const uint4*>(P.cbvh_src);
      uint4* cdst = reinterpret_cast<uint4*>(rt_lds + P.cbvh_lds_off);
      for (uint32_t k = threadIdx.x; k < P.cbvh_bytes / 16; k += blockDim.x) cdst[k] = csrc[k];
    }
    __syncthreads();
  }
  TabsT<TP> T;
  if constexpr (STAGED) {
    typedef const __attribute__((address_space(3))) uint8_t* lbptr;
    const lbptr b = (lbptr)rt_lds;
    T.nodes = reinterpret_cast<lptr>(b);
    T.mats = reinterpret_cast<lptr>(b + P.o_mats);
    T.texs = reinterpret_cast<lptr>(b + P.o_texs);
    T.lights = reinterpret_cast<lptr>(b + P.o_lights);
    T.loffs = reinterpret_cast<lptr>(b + P.o_loffs);
    T.perlin = rt_lds + P.o_perl;
  } else {
    const uint8_t* b = (const uint8_t*)P.nodes;
    T.nodes = reinterpret_cast<gptr>(b);
    T.mats = reinterpret_cast<gptr>(b + P.o_mats);
    T.texs = reinterpret_cast<gptr>(b + P.o_texs);
    T.lights = reinterpret_cast<gptr>(b + P.o_lights);
    T.loffs = reinterpret_cast<gptr>(b + P.o_loffs);
    T.perlin = rt_lds + (P.stage_scene ? P.o_perl : 0u);
  }
  Ctr<COUNT> C;
#ifdef RT_PROF
  if (threadIdx.x < 16) prof_trav[threadIdx.x] = 0ull;
  if (threadIdx.x < kBlockBvh / 64) prof_wmax[threadIdx.x] = 0u;
  __syncthreads();
#endif
#ifdef RT_PROF  // profiling build: wave cycles per loop section into P.ops[0..7] (not shipped)
  unsigned long long prof_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long prof_last = __builtin_readcyclecounter();
  int prof_sec = 0;
  unsigned long long prof_lanes = 0, prof_iters = 0;  // lanes entering traversal, wave-iterations
#define PROF(k)                                                  \
  do {                                                           \
    const unsigned long long now_ = __builtin_readcyclecounter(); \
    prof_acc[prof_sec] += now_ - prof_last;                      \
    prof_last = now_;                                            \
    prof_sec = (k);                                              \
  } while (0)
#else
#define PROF(k) \
  do {          \
  } while (0)
#endif
  // Persistent waves over a global pool queue. A pool is one 8x8 pixel tile x
  // one stratum row s_j (x one block of kPoolSi stratum columns s_i for segment and tail pools).
  // Per pixel and s_j the samples are summed in the reference's s_i order (render.rs:185-189)
  // as block partials p_b (a running sum over one block of kPoolSi samples, from 0) and the row
  // total R = ((p_0 + p_1) + p_2) + ..., whoever computes them:
  //  * row pools (pairs [0, n_pairs_r), non-BVH kernels): one item per pixel = all its samples
  //    of the row; the lane keeps p_b and R in LDS and writes ONE f64 RGB value, R;
  //  * segment pools (then up to n_pairs_a): one item per pixel = one block's samples; the lane
  //    writes p_b and rt_reduce forms R;
  //  * tail pools (the last pairs): one item per pixel-sample, written as f64 RGB to its own
  //    output value; rt_reduce forms p_b (the same running sum) and R.
  // Row items keep the workspace at one value per (pixel, s_j); the segment band after them
  // absorbs the rows' launch tail (a row is ~sqrt_spp paths) and the single-sample tail the
  // segments' one, so the launch ends within a path or two per lane.
  // Idle lanes claim the next item of the wave's pool (ballot + mbcnt), across pool boundaries,
  // so lanes only idle at the very end of the launch. Wave-uniform pool state:
  const int lane = threadIdx.x & 63;
  int q = 0, si0 = 0, tx = 0, ty = 0, tile_w = 1, nv = 1, pool = 0, s_jp = 0;
  bool tailp = false;  // the pool is a tail pool (one item per sample)
  bool rowp = false;   // the pool is a row pool (one item per pixel, every s_i)
  uint32_t obase = 0;  // the pool's first output value (slot * 64)
  bool more = true;    // the queue may still hold pools
  constexpr uint32_t SC = Trav::kScene;  // the scene's material kinds and light-list shape
  const bool have_lights = (SC & kScLights) && P.n_lights > 0;
  const bool iso_ref = (P.flags & RT_FLAG_SEMANTICS_REFERENCE) != 0;
  constexpr int NB = BlockOf<BVH>::value;
  // per-lane f64 running sum of the item in flight (the block's samples so far), and of a row
  // item the row total over its finished blocks: static LDS in non-BVH kernels; BVH kernels,
  // whose LDS holds the compact trees, keep the row totals at the end of the dynamic LDS
  // (TraceParams::row_lds_off) when the launch's plan has room for them, and otherwise render
  // no row items (n_pairs_r = 0)
  constexpr bool ROWS = true;
  __shared__ double sh_acc[3 * NB];
  __shared__ double sh_row_s[BVH ? 1 : 3 * NB];
  typedef __attribute__((address_space(3))) double* ldw_t;
  const ldw_t sh_row = BVH ? (ldw_t)(rt_lds + P.row_lds_off) : (ldw_t)sh_row_s;
  // Non-BVH kernels: a bounce's throughput factor and an ending path's radiance are set inside
  // the divergent shading branches and read after they join; held in registers across the join
  // they were spilled to scratch at five waves per SIMD (cornell_smoke: 30 VGPRs, three
  // serialised scratch reloads per bounce, 35x the workspace's write bytes). Per-lane LDS slots
  // take the exec-masked writes of the branches as they are. (The BVH kernels' LDS holds the
  // compact trees; they keep registers, and do not spill there.)
  constexpr bool LDSF = !BVH;
  __shared__ wt sh_f[LDSF ? 3 * NB : 1];
  __shared__ wt sh_le[LDSF ? 3 * NB : 1];
  const int tid = threadIdx.x;

  d3 ro = mk(0., 0., 0.), rd = ro;
  w3 beta = mkw(0, 0, 0);
  double tm = 0.;
  // remaining bounces (low 24 bits, render.rs:260) | special-value state RT_XS_* << 24
  int depth = 0;
  bool alive = false;  // a path is in flight
  bool fresh = false;  // the lane's next sample needs its camera ray (claimed item / next s_i)
  uint32_t xk = 0;     // x | row-in-call << 16 | tail item << 31
  uint32_t sij = 0;    // row item << 31 | s_j << 16 | s_i of the sample in flight
  uint32_t oslot = 0;  // the item's output value (TraceParams::part: slot * 64 + pixel in tile)
  int next = 0;        // pool items claimed so far (wave-uniform)
  // a valid (non-zero) xoroshiro64* state from the start: lanes without a path still run bounces on
  // stale rays at the end of a launch, and the rejection loops (random_unit_vector) must end
  Rng g = {0x9E3779B9u, 1u};
  // A sample's radiance is final: add it to the item's running sum. Inside a block the item
  // continues with its next s_i; at a block end a segment (or tail) item writes its f64 sum, a
  // row item adds it to its row total and goes on, writing the total after its last block.
  auto end_sample = [&](d3 L) {
    // launch constants through the opaque kernarg pointer: read at the point of use instead of
    // being held in SGPRs across the path loop (kparams())
    const kparams_t Q = kparams();
    L = xs_resolve(L, (uint32_t)depth >> 24);
    double a0 = sh_acc[tid] + L.x, a1 = sh_acc[NB + tid] + L.y, a2 = sh_acc[2 * NB + tid] + L.z;
    alive = false;
    const int s_n = (int)(sij & 0xffffu) + 1;
    if (!(xk >> 31) && (s_n & (kPoolSi - 1)) != 0 && s_n < Q->sqrt_spp) {
      sh_acc[tid] = a0, sh_acc[NB + tid] = a1, sh_acc[2 * NB + tid] = a2;
      sij += 1u;
      fresh = true;
    } else {
      bool done = true;
      if (ROWS && (sij >> 31)) {  // a row item's block ends: R = p_0, then R + p_b
        if (s_n > kPoolSi) {
          a0 = sh_row[tid] + a0, a1 = sh_row[NB + tid] + a1, a2 = sh_row[2 * NB + tid] + a2;
        }
        if (s_n < Q->sqrt_spp) {
          sh_row[tid] = a0, sh_row[NB + tid] = a1, sh_row[2 * NB + tid] = a2;
          sh_acc[tid] = 0.0, sh_acc[NB + tid] = 0.0, sh_acc[2 * NB + tid] = 0.0;
          sij += 1u;
          fresh = true;
          done = false;
        }
      }
      if (done) {
        double* o = Q->part + (size_t)oslot * 3;
        o[0] = a0, o[1] = a1, o[2] = a2;
      }
    }
  };

  for (;;) {
    PROF(0);
    // ---- pool scheduling: every idle lane claims the next unclaimed item (all 64 lanes are
    // active here: lanes only ever leave the loop together)
    const bool idle = !alive && !fresh;
    const unsigned long long want = __ballot(idle);
    if (want != 0ull && next >= pool && more) {  // current pool drained: take the next one
      const kparams_t Q = kparams();
      uint32_t id = 0u;
      if (lane == 0) id = atomicAdd(Q->queue, 1u);
      id = __builtin_amdgcn_readfirstlane(id);
      if ((int)id < Q->n_pools) {
        const int r = ROWS ? Q->n_pairs_r : 0, nb = Q->n_blk;
        int blk = 0;
        rowp = ROWS && (int)id < r;
        if (rowp) {
          q = (int)id;
        } else {
          const int j = (int)id - r, m = j / nb;
          blk = j - m * nb;
          q = r + m;
        }
        tailp = q >= Q->n_pairs_a;
        obase = tailp ? (uint32_t)(r + (Q->n_pairs_a - r) * nb + (q - Q->n_pairs_a) * Q->sqrt_spp) * 64u
                      : id * 64u;
        const int tile = q / Q->n_sj;
        tx = tile % Q->tiles_x;
        ty = tile / Q->tiles_x;
        tile_w = imin(kWaveTile, Q->W - tx * kWaveTile);
        nv = tile_w * imin(kWaveTile, Q->n_rows - ty * kWaveTile);
        si0 = blk * kPoolSi;
        pool = tailp ? nv * imin(kPoolSi, Q->sqrt_spp - si0) : nv;
        s_jp = Q->sj0 + (q - tile * Q->n_sj);
      } else {
        more = false;
        pool = 0;
      }
      next = 0;
    }
    if (idle) {
      const int rank = (int)__builtin_amdgcn_mbcnt_hi(
          (uint32_t)(want >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)want, 0u));
      const int k = next + rank;
      if (k < pool) {
        int pv, s_i;
        if (nv == kWaveTile * kWaveTile) {  // full tile (wave-uniform): shifts
          pv = k & (kWaveTile * kWaveTile - 1);
          s_i = si0 + (k >> 6);
        } else {
          pv = k % nv;
          s_i = si0 + k / nv;
        }
        if (!tailp) s_i = si0;
        int cx, cy;  // pixel of the tile
        if (tile_w == kWaveTile) {  // wave-uniform: every tile but the right-edge column
          cx = pv & (kWaveTile - 1);
          cy = pv >> 3;
        } else {
          cx = pv % tile_w;
          cy = pv / tile_w;
        }
        const int x = tx * kWaveTile + cx;
        const int kr = ty * kWaveTile + cy;
        xk = (uint32_t)x | (uint32_t)kr << 16 | (tailp ? 0x80000000u : 0u);
        sij = (rowp ? 0x80000000u : 0u) | (uint32_t)s_jp << 16 | (uint32_t)s_i;
        oslot = obase + (tailp ? (uint32_t)s_i * 64u : 0u) + (uint32_t)pv;
        sh_acc[tid] = 0.0, sh_acc[NB + tid] = 0.0, sh_acc[2 * NB + tid] = 0.0;
        fresh = true;
      }
    }
    next += __popcll(want);
#ifdef RT_ABL_FRESH2  // ablation build: a second, discarded camera ray per fresh lane (its cost)
    if (fresh) {
      const kparams_t Q = kparams();
      uint32_t xk2 = xk;
      asm volatile("" : "+v"(xk2));
      const int x = (int)(xk2 & 0xffffu);
      const int y = Q->row_begin + (int)((xk2 >> 16) & 0x7fffu) * Q->row_step;
      const int s_i = (int)(sij & 0xffffu), s_j = (int)((sij >> 16) & 0x7fffu);
      Rng g2 = rng_seed(Q->seed_lo, Q->seed_hi, (uint32_t)(y * Q->W + x),
                        (uint32_t)(s_j * Q->sqrt_spp + s_i));
      d3 pc = vfma((double)y, karr3(Q->dv), vfma((double)x, karr3(Q->du), karr3(Q->p00)));
      double px = fma(Q->rs, (double)s_i + rnd(g2), -0.5);
      double py = fma(Q->rs, (double)s_j + rnd(g2), -0.5);
      d3 ps = pc + vfma(px, karr3(Q->du), karr3(Q->dv) * py);
      const double t2 = rnd(g2);
      asm volatile("" ::"v"(ps.x), "v"(ps.y), "v"(ps.z), "v"(t2));
    }
#endif
    if (fresh) {
      const kparams_t Q = kparams();
      const int x = (int)(xk & 0xffffu);
      const int y = Q->row_begin + (int)((xk >> 16) & 0x7fffu) * Q->row_step;
      const int s_i = (int)(sij & 0xffffu), s_j = (int)((sij >> 16) & 0x7fffu);
      // get_ray render.rs:218-249 (stratum (s_i, s_j): 2 jitter draws, defocus disk, time)
      g = rng_seed(Q->seed_lo, Q->seed_hi, (uint32_t)(y * Q->W + x),
                   (uint32_t)(s_j * Q->sqrt_spp + s_i));
      C.inc(RT_OP_SAMPLES);
      d3 pc = vfma((double)y, karr3(Q->dv), vfma((double)x, karr3(Q->du), karr3(Q->p00)));
      double px = fma(Q->rs, (double)s_i + rnd(g), -0.5);
      double py = fma(Q->rs, (double)s_j + rnd(g), -0.5);
      d3 ps = pc + vfma(px, karr3(Q->du), karr3(Q->dv) * py);
      d3 origin = karr3(Q->center);
      if (Q->defocus) {
        for (;;) {
          double dx = rnd_pm1(g);
          double dy = rnd_pm1(g);
          if (fma(dx, dx, dy * dy) < 1.0) {
            const kparams_t R = kparams();
            origin = vfma(dy, karr3(R->ddv), vfma(dx, karr3(R->ddu), karr3(R->center)));
            break;
          }
        }
      }
      ro = origin;
      rd = ps - origin;
      tm = rnd(g);
      beta = mkw(1, 1, 1);
      depth = Q->max_depth;  // RT_XS_* cleared
      alive = true;
      fresh = false;
      if (Q->max_depth == 0) {  // uniform: ray_color's depth guard (render.rs:260-262) at once
        C.inc(RT_OP_DEPTH_CUTOFF);
        end_sample(mk(0., 0., 0.));
      }
    }
    // one back edge only (a `continue` here would give the loop header a second incoming state
    // and the compiler a full copy of it); a wave with no path in flight but more pools to
    // claim (a pool boundary) runs one bounce on stale rays, which the lanes then drop
    if (!more && __ballot(alive) == 0ull) break;
    // One bounce, run by EVERY lane of the wave (product kernels): a lane without a path (only
    // at the very end of a launch) traces its stale ray and its result is dropped below. The
    // scattered ray and throughput factor are committed unconditionally after the block, and
    // the lanes that ended (miss, light) leave them undefined: the path state then has no value
    // that survives the block on some lanes only, which would make the compiler copy the whole
    // state (24 VGPRs) into join registers on every bounce. `break` leaves the block; the ending
    // lanes then share ONE end_sample. ray_color's depth guard (render.rs:260-262) is applied
    // where the depth is decremented (a fresh path starts with max_depth >= 1; at max_depth 0
    // the camera-ray block ends every sample at once).
    // A path gathers radiance only where it ends (a miss adds beta * background, a light hit beta *
    // emission, render.rs:272, 292-309; every other bounce adds the zero emission of a non-light,
    // and a zero-pdf bounce restarts the sum at 0), so its radiance is 0 until that bounce and
    // then 0 + beta * X = beta * X exactly: no running radiance is carried across bounces.
    bool term = false, emit_end = false;
    w3 Le;              // the ending lanes' radiance (undefined on the others)
    d3 p_next, d_next;  // the scattered ray
    w3 f_next;          // this bounce's throughput factor
    auto set_le = [&](w3 v) {
      if constexpr (LDSF) {
        sh_le[tid] = v.x, sh_le[NB + tid] = v.y, sh_le[2 * NB + tid] = v.z;
      } else {
        Le = v;
      }
    };
    auto set_f = [&](w3 v) {
      if constexpr (LDSF) {
        sh_f[tid] = v.x, sh_f[NB + tid] = v.y, sh_f[2 * NB + tid] = v.z;
      } else {
        f_next = v;
      }
    };
    const bool run = COUNT ? alive : true;
    if (!run) {
      term = alive;
      C.inc_if(RT_OP_DEPTH_CUTOFF, alive);
    } else do {
    C.inc(RT_OP_WORLD_QUERIES);
    PROF(1);
#ifdef RT_PROF
    prof_lanes += __popcll(__ballot(1));
    prof_iters += 1;
#endif
    double t;
    uint32_t hn = 0;
    int hf = -1;
#ifdef RT_ABL_TRAV2  // ablation build: the traversal runs twice (same result); the time delta
                     // is the traversal's cost
    {
      double z = 0.0;
      asm volatile("" : "+v"(z));
      double t2;
      uint32_t hn2;
      int hf2;
      Rng g2 = g;  // the world query of this kernel (generated or interpreted), on a copy of g
      d3 ro2 = ro;
      ro2.x += z;
      Trav::template world<COUNT, VOL, BVH, VOLB, VOLI>(P, ro2, rd, tm, t2, hn2, hf2, g2, C);
      asm volatile("" ::"v"(t2), "v"(hn2), "v"(hf2), "v"(g2.s0));
    }
#endif
    if (!Trav::template world<COUNT, VOL, BVH, VOLB, VOLI>(P, ro, rd, tm, t, hn, hf, g, C)) {
      C.inc(RT_OP_MISSES);  // background render.rs:298-309
      set_le(beta * to_w3(karr3(kparams()->bg)));
      term = emit_end = true;
      break;
    }
    // ---- hit record of the winning primitive, recomputed in its own frame (deferred)
    PROF(2);
    const TP X = T.nodes + hn;
    uint32_t type = X[0] & 0xffu;
    d3 o, d;
    Trav::frame_in(T.nodes, hf, ro, rd, o, d);
#ifdef RT_ABL_HIT2  // ablation build: the hit record's frame recomputed (transform chain) twice
    {
      d3 o2, d2, ro2 = ro;
      asm volatile("" : "+v"(ro2.x));
      frame_ray(T.nodes, hf, ro2, rd, o2, d2);
      asm volatile("" ::"v"(o2.x), "v"(o2.y), "v"(o2.z), "v"(d2.x), "v"(d2.y), "v"(d2.z));
    }
#endif
    d3 p = vfma(t, d, o);
    d3 normal;
    bool front = true;
    double u = 0., v = 0.;
    const TP M = T.mats + (size_t)X[2] * RTL_MAT_WORDS;
    uint4 mh = ld4u(M);
    const bool needs_uv = TEX && (mh.x & RTL_MATF_NEEDS_UV) != 0u;
    // the primitive's outward normal per type, then ONE set_face_normal (hittable.rs:22-37) for
    // every lane; a ConstantMedium hit has normal (1, 0, 0) and front_face true
    // (constant_medium.rs:82-90)
    d3 outward;
    if (type == RTL_QUAD) {
      const TP XG = X + RTL_QUAD_GEN;
      outward = ld3(XG, 0);
      if (needs_uv) {
        d3 pq = p - ld3(XG, 4);
        u = dot(pq, ld3(XG, 8));
        v = dot(pq, ld3(XG, 12));
      }
    } else if (type == RTL_SPHERE) {
      d3 c = ld3(X, 0);
      if (X[0] & RTL_SPHERE_MOVING) c = vfma(tm, ld3(X, 4), c);
      // (p - c) / radius (object.rs:169): q = x (1/r) with the host's IEEE reciprocal, then one
      // residual step q + fma(-q, r, x) (1/r), which is the correctly rounded quotient
      // (Markstein: 1/r correctly rounded, q within an ulp), i.e. the reference's division
      const d3 pc = p - c;
      const double ir = ldd(X, 7), rad = ldd(X, 3);
      const d3 q0 = pc * ir;
      outward = mk(fma(fma(-q0.x, rad, pc.x), ir, q0.x), fma(fma(-q0.y, rad, pc.y), ir, q0.y),
                   fma(fma(-q0.z, rad, pc.z), ir, q0.z));
      if (needs_uv) sphere_uv(outward, u, v);
    } else {
      outward = mk(1., 0., 0.);
    }
    front = (type != RTL_QUAD && type != RTL_SPHERE) | (dot(d, outward) < 0.0);
    normal = front ? outward : -outward;
    Trav::frame_out(T.nodes, hf, p, normal);  // back to world space
    const uint32_t kind = mh.x & 0xffu;
    PROF(3);
    if ((SC & kScLight) && kind == RT_MAT_DIFFUSE_LIGHT) {  // material.rs:210-222
      C.inc(RT_OP_EMISSIVE_HITS);
      set_le(front ? beta * to_w3(tex_value<COUNT, TEX>(P, T, mh.y, u, v, p, C)) : mkw(0, 0, 0));
      term = emit_end = true;
      break;
    }
    if ((SC & kScMetal) && kind == RT_MAT_METAL) {  // material.rs:124-134
      C.inc(RT_OP_METAL);
      d3 reflected = reflect(unit_vector(rd), normal);
      d3 ruv = random_unit_vector(g);
      p_next = p;
      d_next = vfma(ldd(M, 3), ruv, unit_vector(reflected));
      set_f(to_w3(ld3(M, 0)));
      break;
    }
    // Dielectric (material.rs:166-191), Lambertian and Isotropic (the mixture-PDF branch,
    // render.rs:278-292) run as ONE block: a wave holding both kinds of lanes shares the unit
    // vector, the first sqrt, the first uniform draw and the throughput update instead of
    // running two exclusive branches. Per lane the arithmetic and the draw order are exactly
    // those of the separate branches.
    PROF(4);
    const bool diel = (SC & kScDielectric) && kind == RT_MAT_DIELECTRIC;
    const bool iso = VOL && kind == RT_MAT_ISOTROPIC;  // VOL kernels: volumes or Isotropic
    C.inc(diel ? RT_OP_DIELECTRIC : (iso ? RT_OP_ISOTROPIC : RT_OP_LAMBERTIAN));
    // unit(r_in.direction) (material.rs:170) or CosinePDF's w = unit(normal) (pdf.rs:58-62)
    const d3 uu = unit_vector(diel ? rd : normal);
    const double ratio = front ? ldd(M, 4) : ldd(M, 3);  // dielectric: 1/ir : ir
    const double cos_t = fmin(dot(-uu, normal), 1.0);     // material.rs:172
    // first sqrt: the dielectric's sin(theta) (material.rs:173) or cos_theta_max of the first
    // sphere light at p (object.rs:196, 205-207), shared by Sphere::random and pdf_value
    double sq_in = fma(-cos_t, cos_t, 1.0);
    if ((SC & kScLSphere) && P.sphere_light0 >= 0) {
      const TP S0 = T.lights + T.loffs[P.sphere_light0];
      const d3 cmo = ld3(S0, 0) - p;
      const double r0 = ldd(S0, 3);
      const double arg = 1.0 - div_nr(r0 * r0, dot(cmo, cmo));
      sq_in = diel ? sq_in : arg;
    }
    const double sq = sqrt_nr(sq_in);
    const double cos_sl0 = sq;
    const bool tir = diel && ratio * sq > 1.0;  // cannot_refract (material.rs:175)
    // first uniform: the Schlick test, drawn only when not TIR (material.rs:180), or the
    // mixture coin (pdf.rs:120-126)
    double u0 = 0.0;
    if (diel ? !tir : have_lights) u0 = rnd(g);
    const double r0s = front ? ldd(M, 5) : ldd(M, 6);  // Schlick r0 of `ratio` (host-derived)
    // reflectance r0 + (1 - r0) * (1 - cos)^5 in the reference's operation order (material.rs:
    // 156-163: a product, then a sum), with the power correctly rounded (pow5_cr). The test
    // against u0 is decided from x^5 by three products (within 4.5 ulps of the correctly rounded
    // power, so the reflectance is within 6.5 ulps of the exact one) unless u0 lies within 32
    // ulps of it (a window of ~4e-15 relative, so about one draw in 10^14); those lanes take
    // pow5_cr, and the decision is the exact one everywhere. (Kernels without a BVH only: C2
    // -0.61 %, while the BVH kernel measured +0.51 %; profiles/r06l_ab_schlick_c{2,4}.log.)
    const double sx = 1.0 - cos_t, omr = 1.0 - r0s;
    bool refl_u;
    if constexpr (!BVH) {
      const double sx2 = sx * sx;
      const double refl_f = r0s + omr * ((sx2 * sx2) * sx);
      refl_u = refl_f > u0;
      const bool near_u = fabs(refl_f - u0) <= refl_f * 0x1p-48;
      if (__ballot(near_u) != 0ull && near_u) refl_u = r0s + omr * pow5_cr(sx) > u0;
    } else {
      refl_u = r0s + omr * pow5_cr(sx) > u0;
    }
    const bool refl = tir || refl_u;
    const bool light_branch = !diel && have_lights && u0 < 0.5;
    d3 dir;     // set on both arms below
    w3 factor;
    double cos_sl = cos_sl0;
    if (!diel) {
      const w3 atten = to_w3(tex_value<COUNT, TEX>(P, T, mh.y, u, v, p, C));
      // Draw order as the reference: mixture coin (above), then light index
      // (hittable.rs:126-129) or nothing, then the two uniforms of whichever generator runs.
      uint32_t ltype = 0, li = 0;
      TP L = T.lights;
      if (light_branch) {
        C.inc(RT_OP_LIGHT_GEN);
        li = P.lights_is_list ? rnd_index(g, P.n_lights) : 0u;
        L = T.lights + T.loffs[li];
        ltype = L[0] & 0xffu;
        while ((SC & kScLList) && ltype == RTL_LLIST) {  // a nested HittableList: random_int pick (hittable.rs:126-129)
          li = L[1] + rnd_index(g, L[0] >> 8);
          L = T.lights + T.loffs[li];
          ltype = L[0] & 0xffu;
        }
      } else {
        C.inc(RT_OP_COSINE_GEN);
      }
      const d3 un = uu;
      if (iso && !light_branch) {
        dir = random_unit_vector(g);  // SpherePDF::generate pdf.rs:51-53
#ifdef RT_ABL_RUV2  // ablation build: the isotropic rejection loop run twice on a copy of the
                    // RNG (same image; its cost)
        {
          Rng g2 = g;
          asm volatile("" : "+v"(g2.s0));
          const d3 d2 = random_unit_vector(g2);
          asm volatile("" ::"v"(d2.x), "v"(g2.s1));
        }
#endif
      } else if ((SC & kScLOther) && light_branch && ltype != RTL_QUAD && ltype != RTL_SPHERE) {
        dir = mk(1., 0., 0.);  // Object::random default arm (object.rs:300)
      } else {
        // Quad::random (object.rs:503-506), Sphere::random / random_to_sphere (204-212, 122-132)
        // and CosinePDF::generate (pdf.rs:75-77, vec3.rs:240-250) share one straight-line block:
        // one ONB, one sincos, selects instead of divergent branches.
        const double r1 = rnd(g), r2 = rnd(g);
        const bool lq = light_branch && ltype == RTL_QUAD;
        const bool ls = (SC & kScLSphere) && light_branch && ltype == RTL_SPHERE;
        d3 c = ls ? ld3(L, 0) : p;
        d3 wdir = c - p;  // Sphere::random direction (object.rs:205)
        d3 w = ls ? unit_vector(wdir) : un;
        d3 aa = fabs(w.x) > 0.9 ? mk(0., 1., 0.) : mk(1., 0., 0.);
        Onb b;
        b.v = unit_vector(cross(w, aa));
        b.u = cross(w, b.v);
        b.w = w;
        double sn, cs;
        sincos2pi(r1, &sn, &cs);
        // random_to_sphere (object.rs:122-132) / random_cosine_direction (vec3.rs:240-250): one
        // sqrt serves rho of both, so a wave with both kinds of lanes runs two sqrt, not three
        double z;
        if (ls) {
          double cm;
          if ((int)li == P.sphere_light0) {
            cm = cos_sl0;
          } else {
            const double rad = ldd(L, 3);
            cm = sqrt_nr(1.0 - rad * rad / dot(wdir, wdir));
          }
          z = fma(r2, cm - 1.0, 1.0);
        } else {
          z = sqrt_nr(1.0 - r2);
        }
        const double rho = sqrt_nr(ls ? fma(-z, z, 1.0) : r2);
        d3 local = onb_local(b, mk(cs * rho, sn * rho, z));
        if (lq) {
          local = vfma(r2, ld3(L, 20), vfma(r1, ld3(L, 16), ld3(L, 4))) - p;
        }
        dir = local;
      }
      wt mat_pdf, s_pdf;
      if (iso) {
        mat_pdf = (wt)(1.0 / (4.0 * kPi));                      // SpherePDF::value pdf.rs:47-49
        s_pdf = iso_ref ? (wt)0 : (wt)(1.0 / (4.0 * kPi));      // semantics S2 (material.rs:70-72)
      } else {
        // CosinePDF::value (pdf.rs:69-73) and Lambertian::scattering_pdf (material.rs:100-108):
        // the cosines of unit(dir) with w = unit(normal) and with the normal. Their zero tests
        // take the signs of the f64 dot products with dir (1/|dir| > 0 keeps a sign); the values
        // are weights: the f32 dots scaled by 1/|dir|.
        const double dw = dot(dir, un), dn = dot(normal, dir);
        const wt irs = rsq_wt((wt)dot(dir, dir)) * kInvPiW;
        mat_pdf = dw > 0.0 ? (wt)dw * irs : (wt)0;
        s_pdf = dn < 0.0 ? (wt)0 : (wt)dn * irs;
      }
      wt pdf_val = mat_pdf;
      PROF(5);
#ifndef RT_ABL_NOLPDF  // ablation build: no light-PDF evaluation (weights only; same paths)
      if (have_lights)  // pdf.rs:116
        pdf_val = fma((wt)0.5, Trav::template lights_pdf<COUNT>(P, p, dir, cos_sl, C), (wt)0.5 * mat_pdf);
#ifdef RT_ABL_LPDF2  // ablation build: the light PDF evaluated twice (same result)
      if (have_lights) {
        d3 p2 = p;
        asm volatile("" : "+v"(p2.x));
        const wt lp2 = Trav::template lights_pdf<COUNT>(P, p2, dir, cos_sl, C);
        asm volatile("" ::"v"(lp2));
      }
#endif
#endif
      PROF(6);
      factor = atten * (s_pdf * rcp_wt(pdf_val));
#ifndef RT_ABL_NOXS  // ablation build: no special-value tracking (cost of RT_XS_*)
      if (!(pdf_val != (wt)0)) {  // pdf_val 0 or NaN: the sample becomes inf / NaN (RT_XS_ON)
        depth |= (int)((RT_XS_ON | xs_nan_bits(atten * s_pdf, beta)) << 24);
        beta = mkw(1, 1, 1);
        factor = beta;
      }
#endif
    } else {
      // reflect (vec3.rs:219-221) or refract (vec3.rs:223-229; its cos_theta is cos_t)
      const d3 perp = ratio * vfma(cos_t, normal, uu);
      const d3 refr = vfma(-sqrt_nr(fabs(1.0 - dot(perp, perp))), normal, perp);
      dir = refl ? reflect(uu, normal) : refr;
      factor = to_w3(ld3(M, 0));  // attenuation = tint
    }
    p_next = p;
    d_next = dir;
    set_f(factor);
    } while (false);
    if (run) {  // wave-uniform: commit the bounce (garbage on ending lanes, never read)
      ro = p_next;
      rd = d_next;
      if constexpr (LDSF) f_next = mkw(sh_f[tid], sh_f[NB + tid], sh_f[2 * NB + tid]);
      beta = beta * f_next;
      // the product is formed here: left to itself the compiler sinks it to beta's next use (the
      // following bounce, past the pool scheduling and the camera-ray block), which keeps the
      // three factors live across the loop's back edge and spills them (ROCm 7.2: scratch
      // stores and three serialised reloads per bounce at C3 and C4)
      asm volatile("" : "+v"(beta.x), "+v"(beta.y), "+v"(beta.z));
      --depth;  // ending lanes had depth >= 1: the RT_XS_* bits above it are untouched
      const bool cut = !term && (depth & 0xffffff) == 0;
      C.inc_if(RT_OP_DEPTH_CUTOFF, cut);
      term |= cut;
    }
    if (term & alive) {
      if constexpr (LDSF) {
        if (emit_end) Le = mkw(sh_le[tid], sh_le[NB + tid], sh_le[2 * NB + tid]);
      }
      end_sample(emit_end ? to_d3(Le) : mk(0., 0., 0.));
    }
  }
#ifdef RT_PROF
  PROF(7);
  if ((threadIdx.x & 63) == 0)
    for (int k = 0; k < 8; ++k) atomicAdd(&P.ops[k], prof_acc[k]);
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(&P.ops[8], prof_lanes);
    atomicAdd(&P.ops[9], prof_iters);
  }
  __syncthreads();
  if (threadIdx.x < 16) atomicAdd(&P.ops[10 + threadIdx.x], prof_trav[threadIdx.x]);
#endif
#undef PROF
  if (COUNT) {
    C.flush(sh_ops);
    __syncthreads();
    for (int k = threadIdx.x; k < RT_OP_COUNT; k += blockDim.x)
      if (sh_ops[k]) atomicAdd(&P.ops[k], (unsigned long long)sh_ops[k]);
  }
}

}  // namespace rtk
