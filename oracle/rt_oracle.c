/*
 * rt_oracle.c — TEST INFRASTRUCTURE. CPU restatement of the reference per-pixel render loop.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library;
 * it is the checker, never the product. The product path is the HIP library
 * (surely-raytracing_amd/csrc/rt_device.hip), which never links or calls this file.
 *
 * Parity status: the Rust reference cannot be built here (no rustc/cargo, crates not vendored)
 * and is unseeded (rand::thread_rng, utils.rs:5-15), so no golden pixel vectors exist upstream.
 * This restatement is pinned by (a) analytic known-answer tests derived from the reference
 * formulas (tests/test_oracle_kat.py) and (b) statistics of the reference's own renders
 * final_images/{book3,mixed_pdf,cornell_smoke,book2}.png (tests/golden/final_images_stats.json,
 * tests/test_oracle_render.py).
 *
 * Structure follows the reference function by function, RECURSIVELY (not the threaded GPU
 * traversal), so that it independently checks the device's flattening:
 *   render loop        render.rs:171-197 (3-row chunks over a thread pool, s_j outer, s_i inner)
 *   get_ray            render.rs:218-249
 *   ray_color          render.rs:251-311 (recursion kept)
 *   HittableList::hit  hittable.rs:88-109     BvhNode::hit hittable.rs:216-236
 *   Sphere::hit        object.rs:145-184      Quad::hit object.rs:453-490
 *   Aabb::hit          object.rs:340-370      Translate/RotateY::hit transform.rs:57-135
 *   ConstantMedium::hit constant_medium.rs:41-95
 *   materials          material.rs:92-248     PDFs pdf.rs:44-127     Onb onb.rs:24-47
 *   textures           texture.rs:17-131      Perlin perlin.rs:30-96 RtImage::pixel_data rt_image.rs:37-46
 *
 * Two builds (ORACLE_F64 = 0/1):
 *   f64: the parity oracle. Reference precision (the reference is all f64) and the reference's
 *        own operation order, expression by expression: no contraction (-ffp-contract=off), the
 *        association Rust's left-to-right evaluation gives (a*u + b*v) + c*w, IEEE / and sqrt
 *        where the reference divides or takes a root, libm transcendentals. Also the CPU
 *        baseline ("port") of bench.py.
 *   f32: a precision study only (tests/test_oracle_render.py shows why the device is f64):
 *        the same algorithm in float, with fma and polynomial transcendentals.
 * Deliberate deviations from the reference's arithmetic: the RNG (SURVEY App. A
 * S4: a seeded counter stream instead of unseeded ChaCha12, 32-bit uniforms) and the semantics
 * register S1-S3 (S1 empty lights -> material PDF alone; S2 Isotropic scattering_pdf =
 * 1/(4pi); RT_FLAG_SEMANTICS_REFERENCE restores the reference behaviour); nothing else.
 * Both builds draw the same per-sample RNG stream.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/rt_mi355x.h"

#ifndef ORACLE_F64
#define ORACLE_F64 0
#endif

#if ORACLE_F64
typedef double real;
#define R(x) ((double)(x))
#define FMA(a, b, c) ((a) * (b) + (c))
#define SQRT sqrt
#define FABS fabs
#define FLOOR floor
#else
typedef float real;
#define R(x) ((float)(x))
#define FMA(a, b, c) fmaf((a), (b), (c))
#define SQRT sqrtf
#define FABS fabsf
#define FLOOR floorf
#endif

#define EXPORT __attribute__((visibility("default")))

static const double PI_D = 3.14159265358979323846;

/* =============================================================== fp32 math kernels (spec §4.3)
 * Built only from IEEE + - * / sqrt fma, identical on gfx950 (rt_fmath.h). */
static inline uint32_t f_bits(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
}
static inline float f_from(uint32_t u) {
  float f;
  memcpy(&f, &u, 4);
  return f;
}

/* sin(2*pi*u), cos(2*pi*u) for u in [0,1): exact reduction to a quarter-turn fraction. */
static void f32_sincos2pi(float u, float* s_out, float* c_out) {
  float t = u * 4.0f;
  float k = floorf(t + 0.5f);
  float r = t - k;
  float r2 = r * r;
  float s = fmaf(fmaf(fmaf(fmaf(0x1.4bc238p-13f, r2, -0x1.32ca84p-8f), r2, 0x1.466bbap-4f), r2,
                      -0x1.4abbcep-1f), r2, 0x1.921fb6p+0f) * r;
  float c = fmaf(fmaf(fmaf(fmaf(fmaf(-0x1.a0d88ap-16f, r2, 0x1.e1e760p-11f), r2, -0x1.55d3bap-6f),
                           r2, 0x1.03c1f0p-2f), r2, -0x1.3bd3ccp+0f), r2, 1.0f);
  int q = ((int)k) & 3;
  float so = q == 0 ? s : (q == 1 ? c : (q == 2 ? -s : -c));
  float co = q == 0 ? c : (q == 1 ? -s : (q == 2 ? -c : s));
  *s_out = so;
  *c_out = co;
}

/* natural log: fdlibm-style reduction m in [sqrt(1/2), sqrt(2)), s = f/(2+f) series. */
static float f32_log(float x) {
  if (x != x || x < 0.0f) return f_from(0x7fc00000u);
  if (x == 0.0f) return -INFINITY;
  if (x == INFINITY) return x;
  uint32_t ix = f_bits(x);
  int e = 0;
  if (ix < 0x00800000u) { /* denormal */
    x = x * 0x1p23f;
    ix = f_bits(x);
    e = -23;
  }
  e += (int)(ix >> 23) - 127;
  uint32_t mb = (ix & 0x007fffffu) | 0x3f800000u;
  if (mb > 0x3fb504f3u) { /* m > sqrt(2): halve */
    mb -= 0x00800000u;
    e += 1;
  }
  float f = f_from(mb) - 1.0f;
  float s = f / (2.0f + f);
  float z = s * s;
  float w = z * z;
  float t1 = w * (0x1.999c26p-2f + w * 0x1.f13c4cp-3f);
  float t2 = z * (0x1.555554p-1f + w * 0x1.23d3dcp-2f);
  float Rr = t2 + t1;
  float hfsq = 0.5f * f * f;
  float dk = (float)e;
  return dk * 0x1.62e300p-1f - ((hfsq - (s * (hfsq + Rr) + dk * 0x1.2fefa2p-17f)) - f);
}

/* sin(x) for moderate |x| (Cody-Waite with fma, 3-part pi/2). */
static float f32_sin(float x) {
  if (x != x || x == INFINITY || x == -INFINITY) return f_from(0x7fc00000u);
  float k = floorf(fmaf(x, 0x1.45f306p-1f, 0.5f));
  float r = fmaf(-k, 0x1.921fb6p+0f, x);
  r = fmaf(-k, -0x1.777a5cp-25f, r);
  r = fmaf(-k, -0x1.ee59dap-50f, r);
  float r2 = r * r;
  float s = fmaf(fmaf(fmaf(fmaf(0x1.6cb088p-19f, r2, -0x1.a00ec6p-13f), r2, 0x1.111108p-7f), r2,
                      -0x1.555556p-3f), r2, 1.0f) * r;
  float c = fmaf(fmaf(fmaf(fmaf(fmaf(-0x1.23b6aep-22f, r2, 0x1.a00e3ap-16f), r2, -0x1.6c16b2p-10f),
                           r2, 0x1.555556p-5f), r2, -0.5f), r2, 1.0f);
  int q = ((int)k) & 3;
  return q == 0 ? s : (q == 1 ? c : (q == 2 ? -s : -c));
}

static float f32_atan01(float t) { /* t in [0, 1] */
  const float T12 = 0x1.126146p-2f; /* 2 - sqrt(3) */
  int big = t > T12;
  float u = big ? (t * 0x1.bb67aep+0f - 1.0f) / (t + 0x1.bb67aep+0f) : t;
  float u2 = u * u;
  float p = fmaf(fmaf(fmaf(fmaf(fmaf(-0x1.37bc16p-4f, u2, 0x1.c26556p-4f), u2, -0x1.247c38p-3f), u2,
                           0x1.99993cp-3f), u2, -0x1.555556p-2f), u2, 1.0f) * u;
  return big ? p + 0x1.0c1524p-1f /* pi/6 */ : p;
}

static float f32_atan2(float y, float x) {
  if (x != x || y != y) return f_from(0x7fc00000u);
  float ax = fabsf(x), ay = fabsf(y);
  float mx = ax > ay ? ax : ay, mn = ax > ay ? ay : ax;
  float a = mx == 0.0f ? 0.0f : f32_atan01(mn / mx);
  if (ay > ax) a = 0x1.921fb6p+0f - a;
  if (x < 0.0f) a = 0x1.921fb6p+1f - a;
  return y < 0.0f ? -a : a;
}

static float f32_asin_half(float x) { /* |x| <= 1/2 */
  float x2 = x * x;
  float p = fmaf(fmaf(fmaf(fmaf(fmaf(fmaf(0x1.354c4ep-5f, x2, 0x1.d27f90p-7f), x2, 0x1.051bd2p-5f),
                                x2, 0x1.6c991ap-5f), x2, 0x1.333952p-4f), x2, 0x1.555548p-3f), x2,
                 1.0f);
  return p * x;
}

static float f32_acos(float x) {
  if (x != x || x > 1.0f || x < -1.0f) return f_from(0x7fc00000u);
  if (fabsf(x) <= 0.5f) return 0x1.921fb6p+0f - f32_asin_half(x);
  if (x > 0.0f) return 2.0f * f32_asin_half(sqrtf((1.0f - x) * 0.5f));
  return 0x1.921fb6p+1f - 2.0f * f32_asin_half(sqrtf((1.0f + x) * 0.5f));
}

#if ORACLE_F64
#define LOG log
#define POW pow /* f64::powf */
#define SIN sin
#define ACOS acos
#define ATAN2 atan2
static void sincos2pi(double u, double* s, double* c) {
  double phi = 2. * PI_D * u; /* vec3.rs:244 */
  *s = sin(phi);
  *c = cos(phi);
}
#else
#define LOG f32_log
#define POW powf
#define SIN f32_sin
#define ACOS f32_acos
#define ATAN2 f32_atan2
#define sincos2pi f32_sincos2pi
#endif

/* =============================================================== RNG
 * Per pixel-sample stream: pcg2d(pixel, sample) with seed-keyed increments seeds xoroshiro64*
 * (Blackman and Vigna; 64 bits of state, 32-bit outputs), the device's generator
 * (csrc/rt_rng.h rng_seed / rng_step). Round 5 keyed xoroshiro64** with pcg4d(pixel, sample,
 * seed_lo, seed_hi); rounds 1-4 used xoshiro128**. */
typedef struct { uint32_t s[2]; } rng_t;

static inline uint32_t rotl32(uint32_t x, int k) { return (x << k) | (x >> (32 - k)); }
static void rng_seed(rng_t* g, uint64_t seed, uint32_t pixel, uint32_t sample) {
  const uint32_t k0 = ((uint32_t)seed ^ 0x85EBCA6Bu) * 0x9E3779B9u + 1013904223u;
  const uint32_t k1 = ((uint32_t)(seed >> 32) ^ 0xC2B2AE35u) * 0x9E3779B9u + (k0 ^ 0x27D4EB2Fu);
  uint32_t v0 = pixel * 1664525u + k0, v1 = sample * 1664525u + k1;
  v0 += v1 * 1664525u;
  v1 += v0 * 1664525u;
  v0 ^= v0 >> 16;
  v1 ^= v1 >> 16;
  v0 += v1 * 1664525u;
  v1 += v0 * 1664525u;
  v0 ^= v0 >> 16;
  v1 ^= v1 >> 16;
  if ((v0 | v1) == 0) v0 = 0x9E3779B9u;
  g->s[0] = v0;
  g->s[1] = v1;
}
static inline uint32_t rng_u32(rng_t* g) { /* xoroshiro64* */
  uint32_t* s = g->s;
  const uint32_t s0 = s[0];
  uint32_t s1 = s[1];
  const uint32_t result = s0 * 0x9E3779BBu;
  s1 ^= s0;
  s[0] = rotl32(s0, 26) ^ s1 ^ (s1 << 9);
  s[1] = rotl32(s1, 13);
  return result;
}
/* random_double (utils.rs:5-7): f64 build (= the device path): 32-bit uniform in [0,1), exact
 * in double; f32 precision-study build: 24-bit uniform (representable in float). */
#if ORACLE_F64
static inline real rnd(rng_t* g) { return (double)rng_u32(g) * 0x1p-32; }
#else
static inline real rnd(rng_t* g) { return (float)(rng_u32(g) >> 8) * 0x1p-24f; }
#endif
/* random_range(min,max) (utils.rs:9-11) */
static inline real rnd_range(rng_t* g, real a, real b) { return a + (b - a) * rnd(g); }
/* random_int(0, n-1) (utils.rs:13-15) */
static inline uint32_t rnd_index(rng_t* g, uint32_t n) {
  return (uint32_t)(((uint64_t)rng_u32(g) * n) >> 32);
}

/* =============================================================== vec3 (vec3.rs) */
typedef struct { real x, y, z; } vec3;
static inline vec3 v3(real x, real y, real z) { vec3 v = {x, y, z}; return v; }
static inline vec3 vadd(vec3 a, vec3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline vec3 vsub(vec3 a, vec3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline vec3 vneg(vec3 a) { return v3(-a.x, -a.y, -a.z); }
static inline vec3 vmul(vec3 a, vec3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline vec3 vscale(vec3 a, real t) { return v3(a.x * t, a.y * t, a.z * t); }
static inline vec3 vfma(real t, vec3 a, vec3 b) { /* t*a + b */
  return v3(FMA(t, a.x, b.x), FMA(t, a.y, b.y), FMA(t, a.z, b.z));
}
#if ORACLE_F64 && !ORACLE_FMA_DOT
/* vec3.rs:167-169 / 74-76: (x*x' + y*y') + z*z', evaluated left to right */
static inline real dot(vec3 a, vec3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
#elif ORACLE_F64
/* perturbation study only (liboracle_f64fma.so, tools/flip_study.py): the dot product fused as
 * the device evaluates it, every other operation as above. Differs from the reference order in
 * the last bits of each dot product; the study measures how often that alone changes a path. */
static inline real dot(vec3 a, vec3 b) { return fma(a.x, b.x, fma(a.y, b.y, a.z * b.z)); }
#else
static inline real dot(vec3 a, vec3 b) { return FMA(a.x, b.x, FMA(a.y, b.y, a.z * b.z)); }
#endif
static inline vec3 cross(vec3 u, vec3 v) {
  return v3(FMA(u.y, v.z, -(u.z * v.y)), FMA(u.z, v.x, -(u.x * v.z)), FMA(u.x, v.y, -(u.y * v.x)));
}
#if ORACLE_F64
static inline vec3 unit_vector(vec3 v) { /* vec3.rs:179-181: v / v.length() */
  real len = SQRT(dot(v, v));
  return v3(v.x / len, v.y / len, v.z / len);
}
#else
static inline vec3 unit_vector(vec3 v) { return vscale(v, R(1) / SQRT(dot(v, v))); }
#endif
static inline vec3 reflect(vec3 v, vec3 n) { return vfma(-(R(2) * dot(v, n)), n, v); }
static inline real min1(real x) { return x < R(1) ? x : R(1); } /* f64::min(x, 1.) */
static inline vec3 refract(vec3 uv, vec3 n, real e) {             /* vec3.rs:223-229 */
  real cos_theta = min1(dot(vneg(uv), n));
  vec3 perp = vscale(vfma(cos_theta, n, uv), e);
  real par = -SQRT(FABS(R(1) - dot(perp, perp)));
  return vfma(par, n, perp);
}

typedef struct { vec3 o, d; real tm; } ray_t;
static inline vec3 ray_at(const ray_t* r, real t) { return vfma(t, r->d, r->o); }

/* =============================================================== scene (parsed blob) */
typedef struct {
  int tag, mat, moving;
  vec3 c, cv;
  real radius;
  vec3 q, u, v, n, w;
  real d, area;
  vec3 off;
  real sin_t, cos_t, nid;
  real bbox[6];
  int first, count; /* list: child index range in `kids`; bvh: left/right in kids[first..+2] */
} onode;

typedef struct { int kind, tex; vec3 color; real fuzz, ir; } omat;
typedef struct { int kind; vec3 color; real inv_scale, scale; int even, odd, w, h, perlin; int64_t off; } otex;
typedef struct { vec3 ranvec[256]; int px[256], py[256], pz[256]; } operlin;

typedef struct {
  onode* nodes;
  int n_nodes, cap_nodes;
  int* kids;
  int n_kids, cap_kids;
  omat* mats;
  int n_mats;
  otex* texs;
  int n_texs;
  operlin* perlins;
  int n_perlins;
  const uint8_t* texels;
  int world, lights; /* node ids, lights = -1 if empty */
} oscene;

typedef struct { const uint64_t* s; uint64_t n, pos; int err; } cursor;
static int64_t ci(cursor* c) {
  if (c->pos >= c->n) { c->err = 1; return 0; }
  return (int64_t)c->s[c->pos++];
}
static double cf(cursor* c) {
  if (c->pos >= c->n) { c->err = 1; return 0; }
  double d;
  memcpy(&d, &c->s[c->pos++], 8);
  return d;
}
static vec3 cv3(cursor* c) {
  double x = cf(c), y = cf(c), z = cf(c);
  return v3(R(x), R(y), R(z));
}
static int new_node(oscene* sc) {
  if (sc->n_nodes == sc->cap_nodes) {
    sc->cap_nodes = sc->cap_nodes ? sc->cap_nodes * 2 : 256;
    sc->nodes = (onode*)realloc(sc->nodes, sizeof(onode) * sc->cap_nodes);
  }
  memset(&sc->nodes[sc->n_nodes], 0, sizeof(onode));
  return sc->n_nodes++;
}
static int alloc_kids(oscene* sc, int n) {
  if (sc->n_kids + n > sc->cap_kids) {
    while (sc->n_kids + n > sc->cap_kids) sc->cap_kids = sc->cap_kids ? sc->cap_kids * 2 : 256;
    sc->kids = (int*)realloc(sc->kids, sizeof(int) * sc->cap_kids);
  }
  int f = sc->n_kids;
  sc->n_kids += n;
  return f;
}
static void read_bbox(cursor* c, onode* n) {
  for (int i = 0; i < 6; ++i) n->bbox[i] = R(cf(c));
}
static int parse_obj(oscene* sc, cursor* c, int depth) {
  if (depth > 64 || c->err) { c->err = 1; return -1; }
  int id = new_node(sc);
  int tag = (int)ci(c);
  onode tmp;
  memset(&tmp, 0, sizeof(tmp));
  tmp.tag = tag;
  switch (tag) {
    case RT_OBJ_LIST: {
      int64_t n = ci(c);
      read_bbox(c, &tmp);
      if (n < 0 || n > (1 << 24)) { c->err = 1; return -1; }
      tmp.first = alloc_kids(sc, (int)n);
      tmp.count = (int)n;
      sc->nodes[id] = tmp;
      for (int i = 0; i < n; ++i) {
        int k = parse_obj(sc, c, depth + 1);
        sc->kids[tmp.first + i] = k;
      }
      return id;
    }
    case RT_OBJ_BVH: {
      read_bbox(c, &tmp);
      tmp.first = alloc_kids(sc, 2);
      tmp.count = 2;
      sc->nodes[id] = tmp;
      int l = parse_obj(sc, c, depth + 1);
      int r = parse_obj(sc, c, depth + 1);
      sc->kids[tmp.first] = l;
      sc->kids[tmp.first + 1] = r;
      return id;
    }
    case RT_OBJ_SPHERE:
      tmp.mat = (int)ci(c);
      tmp.moving = (int)ci(c);
      tmp.c = cv3(c);
      tmp.radius = R(cf(c));
      tmp.cv = cv3(c);
      read_bbox(c, &tmp);
      sc->nodes[id] = tmp;
      return id;
    case RT_OBJ_QUAD:
      tmp.mat = (int)ci(c);
      tmp.q = cv3(c);
      tmp.u = cv3(c);
      tmp.v = cv3(c);
      tmp.n = cv3(c);
      tmp.w = cv3(c);
      tmp.d = R(cf(c));
      tmp.area = R(cf(c));
      read_bbox(c, &tmp);
      sc->nodes[id] = tmp;
      return id;
    case RT_OBJ_TRANSLATE:
    case RT_OBJ_ROTATE_Y:
    case RT_OBJ_VOLUME: {
      if (tag == RT_OBJ_TRANSLATE) {
        tmp.off = cv3(c);
      } else if (tag == RT_OBJ_ROTATE_Y) {
        tmp.sin_t = R(cf(c));
        tmp.cos_t = R(cf(c));
      } else {
        tmp.mat = (int)ci(c);
        tmp.nid = R(cf(c));
      }
      read_bbox(c, &tmp);
      tmp.first = alloc_kids(sc, 1);
      tmp.count = 1;
      sc->nodes[id] = tmp;
      int k = parse_obj(sc, c, depth + 1);
      sc->kids[tmp.first] = k;
      return id;
    }
    default:
      c->err = 1;
      return -1;
  }
}

static void free_scene(oscene* sc) {
  free(sc->nodes);
  free(sc->kids);
  free(sc->mats);
  free(sc->texs);
  free(sc->perlins);
}

static int parse_scene(const rt_scene_blob* b, oscene* sc) {
  memset(sc, 0, sizeof(*sc));
  if (!b || !b->slots || b->n_slots < RT_BLOB_HEADER_SLOTS) return RT_ERR_BAD_BLOB;
  const uint64_t* s = b->slots;
  if (s[0] != RT_BLOB_MAGIC || s[1] != RT_BLOB_VERSION || s[2] != b->n_slots) return RT_ERR_BAD_BLOB;
  cursor c = {s, b->n_slots, 0, 0};
  sc->n_texs = (int)s[3];
  sc->texs = (otex*)calloc(sc->n_texs + 1, sizeof(otex));
  c.pos = s[4];
  for (int i = 0; i < sc->n_texs; ++i) {
    uint64_t base = c.pos;
    otex* t = &sc->texs[i];
    t->kind = (int)ci(&c);
    if (t->kind == RT_TEX_SOLID) t->color = cv3(&c);
    else if (t->kind == RT_TEX_CHECKER) {
      t->inv_scale = R(cf(&c));
      t->even = (int)ci(&c);
      t->odd = (int)ci(&c);
    } else if (t->kind == RT_TEX_IMAGE) {
      t->w = (int)ci(&c);
      t->h = (int)ci(&c);
      t->off = ci(&c);
    } else if (t->kind == RT_TEX_NOISE) {
      t->scale = R(cf(&c));
      t->perlin = (int)ci(&c);
    }
    c.pos = base + RT_TEX_SLOTS;
  }
  sc->n_mats = (int)s[5];
  sc->mats = (omat*)calloc(sc->n_mats + 1, sizeof(omat));
  c.pos = s[6];
  for (int i = 0; i < sc->n_mats; ++i) {
    uint64_t base = c.pos;
    omat* m = &sc->mats[i];
    m->kind = (int)ci(&c);
    if (m->kind == RT_MAT_METAL) {
      m->color = cv3(&c);
      m->fuzz = R(cf(&c));
    } else if (m->kind == RT_MAT_DIELECTRIC) {
      m->ir = R(cf(&c));
      m->color = cv3(&c);
    } else {
      m->tex = (int)ci(&c);
    }
    c.pos = base + RT_MAT_SLOTS;
  }
  sc->n_perlins = (int)s[7];
  sc->perlins = (operlin*)calloc(sc->n_perlins + 1, sizeof(operlin));
  c.pos = s[8];
  for (int i = 0; i < sc->n_perlins; ++i) {
    operlin* p = &sc->perlins[i];
    for (int k = 0; k < 256; ++k) p->ranvec[k] = cv3(&c);
    for (int k = 0; k < 256; ++k) p->px[k] = (int)ci(&c);
    for (int k = 0; k < 256; ++k) p->py[k] = (int)ci(&c);
    for (int k = 0; k < 256; ++k) p->pz[k] = (int)ci(&c);
  }
  sc->texels = b->texels;
  c.pos = s[9];
  sc->world = parse_obj(sc, &c, 0);
  sc->lights = -1;
  if ((int64_t)s[10] >= 0) {
    c.pos = s[10];
    sc->lights = parse_obj(sc, &c, 0);
    /* an empty HittableList of lights behaves like render_par's empty list (S1) */
    if (sc->lights >= 0 && sc->nodes[sc->lights].tag == RT_OBJ_LIST && sc->nodes[sc->lights].count == 0)
      sc->lights = -1;
  }
  if (c.err || sc->world < 0 || sc->nodes[sc->world].tag != RT_OBJ_LIST) {
    free_scene(sc);
    return RT_ERR_BAD_BLOB;
  }
  return RT_OK;
}

/* =============================================================== hit records & objects */
typedef struct {
  vec3 p, normal;
  real t, u, v;
  int front, mat, node; /* node: the primitive (for lazy sphere UV) */
  vec3 outward_local;   /* sphere outward normal (for get_sphere_uv) */
} hitrec;

typedef struct {
  const oscene* sc;
  uint64_t ops[RT_OP_COUNT];
  uint32_t flags;
} ctx_t;
#define CNT(cx, k) ((cx)->ops[k]++)

static void set_face_normal(hitrec* rec, const ray_t* r, vec3 outward) { /* hittable.rs:22-37 */
  rec->front = dot(r->d, outward) < R(0);
  rec->normal = rec->front ? outward : vneg(outward);
}

/* Aabb::hit object.rs:340-370 */
static int aabb_hit(ctx_t* cx, const real* bb, const ray_t* r, real tmin, real tmax) {
  CNT(cx, RT_OP_AABB_TESTS);
  const real o[3] = {r->o.x, r->o.y, r->o.z}, d[3] = {r->d.x, r->d.y, r->d.z};
  for (int a = 0; a < 3; ++a) {
    real inv_d = R(1) / d[a];
    real t0 = (bb[2 * a] - o[a]) * inv_d;
    real t1 = (bb[2 * a + 1] - o[a]) * inv_d;
    if (inv_d < R(0)) {
      real tt = t0;
      t0 = t1;
      t1 = tt;
    }
    if (t0 > tmin) tmin = t0;
    if (t1 < tmax) tmax = t1;
    if (tmax <= tmin) return 0;
  }
  return 1;
}

/* Quad::hit object.rs:453-490 (inclusive interval: Interval::contains) */
static int quad_hit(ctx_t* cx, const onode* q, const ray_t* r, real tmin, real tmax, hitrec* rec) {
  CNT(cx, RT_OP_QUAD_TESTS);
  real denom = dot(q->n, r->d);
  if (FABS(denom) < R(1e-8)) return 0;
  CNT(cx, RT_OP_QUAD_PLANE);
  real t = (q->d - dot(q->n, r->o)) / denom;
  if (!(tmin <= t && t <= tmax)) return 0;
  CNT(cx, RT_OP_QUAD_INTERVAL);
  vec3 p = ray_at(r, t);
  vec3 pq = vsub(p, q->q);
  real a = dot(q->w, cross(pq, q->v));
  real b = dot(q->w, cross(q->u, pq));
  if (a < R(0) || R(1) < a || b < R(0) || R(1) < b) return 0;
  CNT(cx, RT_OP_QUAD_HITS);
  rec->t = t;
  rec->p = p;
  rec->u = a;
  rec->v = b;
  rec->mat = q->mat;
  rec->node = -1;
  set_face_normal(rec, r, q->n);
  return 1;
}

/* Sphere::hit object.rs:145-184 (strict interval: Interval::surrounds) */
static int sphere_hit(ctx_t* cx, const onode* s, int node, const ray_t* r, real tmin, real tmax,
                      hitrec* rec) {
  CNT(cx, RT_OP_SPHERE_TESTS);
  vec3 center = s->moving ? vfma(r->tm, s->cv, s->c) : s->c; /* object.rs:107-112 */
  vec3 oc = vsub(r->o, center);
  real a = dot(r->d, r->d);
  real half_b = dot(oc, r->d);
  real c = dot(oc, oc) - s->radius * s->radius;
  real disc = FMA(half_b, half_b, -(a * c));
  if (disc < R(0)) return 0;
  CNT(cx, RT_OP_SPHERE_ROOTS);
  real sqrtd = SQRT(disc);
  real root = (-half_b - sqrtd) / a;
  if (!(tmin < root && root < tmax)) {
    root = (sqrtd - half_b) / a;
    if (!(tmin < root && root < tmax)) return 0;
  }
  CNT(cx, RT_OP_SPHERE_HITS);
  rec->t = root;
  rec->p = ray_at(r, root);
  /* (p - center) / radius, component by component (object.rs:169, Div<f64> vec3.rs:152-154) */
  vec3 pc = vsub(rec->p, center);
  vec3 outward = v3(pc.x / s->radius, pc.y / s->radius, pc.z / s->radius);
  rec->outward_local = outward;
  rec->u = R(0);
  rec->v = R(0);
  rec->mat = s->mat;
  rec->node = node;
  set_face_normal(rec, r, outward);
  return 1;
}

static int obj_hit(ctx_t* cx, int id, const ray_t* r, real tmin, real tmax, hitrec* rec);

/* ConstantMedium::hit constant_medium.rs:41-95 */
static int volume_hit(ctx_t* cx, const onode* v, const ray_t* r, real tmin, real tmax, hitrec* rec,
                      rng_t* g) {
  CNT(cx, RT_OP_VOLUME_TESTS);
  hitrec r1, r2;
  int b = cx->sc->kids[v->first];
  if (!obj_hit(cx, b, r, R(-INFINITY), R(INFINITY), &r1)) return 0;
  if (!obj_hit(cx, b, r, r1.t + R(0.0001), R(INFINITY), &r2)) return 0;
  real t1 = r1.t, t2 = r2.t;
  if (t1 < tmin) t1 = tmin;
  if (t2 > tmax) t2 = tmax;
  if (t1 >= t2) return 0;
  if (t1 < R(0)) t1 = R(0);
  real ray_length = SQRT(dot(r->d, r->d));
  real dist_inside = (t2 - t1) * ray_length;
  CNT(cx, RT_OP_VOLUME_DRAWS);
  real hit_distance = v->nid * LOG(rnd(g));
  if (hit_distance > dist_inside) return 0;
  real t = t1 + hit_distance / ray_length;
  rec->t = t;
  rec->p = ray_at(r, t);
  rec->normal = v3(R(1), R(0), R(0));
  rec->front = 1;
  rec->mat = v->mat;
  rec->u = R(0);
  rec->v = R(0);
  rec->node = -1;
  return 1;
}

static __thread rng_t* t_rng; /* stream of the sample being traced (volumes draw inside hit) */

/* Object::hit dispatch object.rs:28-39 */
static int obj_hit(ctx_t* cx, int id, const ray_t* r, real tmin, real tmax, hitrec* rec) {
  const oscene* sc = cx->sc;
  const onode* n = &sc->nodes[id];
  switch (n->tag) {
    case RT_OBJ_LIST: { /* hittable.rs:88-109 */
      int hit = 0;
      real closest = tmax;
      hitrec tr;
      for (int i = 0; i < n->count; ++i) {
        if (obj_hit(cx, sc->kids[n->first + i], r, tmin, closest, &tr)) {
          closest = tr.t;
          *rec = tr;
          hit = 1;
        }
      }
      return hit;
    }
    case RT_OBJ_BVH: { /* hittable.rs:216-236 */
      if (!aabb_hit(cx, n->bbox, r, tmin, tmax)) return 0;
      hitrec lr;
      if (obj_hit(cx, sc->kids[n->first], r, tmin, tmax, &lr)) {
        hitrec rr;
        if (obj_hit(cx, sc->kids[n->first + 1], r, tmin, lr.t, &rr)) *rec = rr;
        else *rec = lr;
        return 1;
      }
      return obj_hit(cx, sc->kids[n->first + 1], r, tmin, tmax, rec);
    }
    case RT_OBJ_SPHERE: return sphere_hit(cx, n, id, r, tmin, tmax, rec);
    case RT_OBJ_QUAD: return quad_hit(cx, n, r, tmin, tmax, rec);
    case RT_OBJ_TRANSLATE: { /* transform.rs:57-69 */
      CNT(cx, RT_OP_TRANSLATE);
      ray_t lr = {vsub(r->o, n->off), r->d, r->tm};
      if (!obj_hit(cx, sc->kids[n->first], &lr, tmin, tmax, rec)) return 0;
      rec->p = vadd(rec->p, n->off);
      return 1;
    }
    case RT_OBJ_ROTATE_Y: { /* transform.rs:84-135 */
      CNT(cx, RT_OP_ROTATE_Y);
      real c = n->cos_t, s = n->sin_t;
      ray_t lr;
      lr.o = v3(FMA(c, r->o.x, -(s * r->o.z)), r->o.y, FMA(s, r->o.x, c * r->o.z));
      lr.d = v3(FMA(c, r->d.x, -(s * r->d.z)), r->d.y, FMA(s, r->d.x, c * r->d.z));
      lr.tm = r->tm;
      if (!obj_hit(cx, sc->kids[n->first], &lr, tmin, tmax, rec)) return 0;
      vec3 p = rec->p, nn = rec->normal;
      rec->p = v3(FMA(c, p.x, s * p.z), p.y, FMA(-s, p.x, c * p.z));
      rec->normal = v3(FMA(c, nn.x, s * nn.z), nn.y, FMA(-s, nn.x, c * nn.z));
      return 1;
    }
    case RT_OBJ_VOLUME: return volume_hit(cx, n, r, tmin, tmax, rec, t_rng);
  }
  return 0;
}

/* =============================================================== textures */
static int32_t f2i_sat(real f) { /* Rust `as i32` */
  if (f != f) return 0;
  if (f >= R(2147483648.0)) return INT32_MAX;
  if (f <= R(-2147483648.0)) return INT32_MIN;
  return (int32_t)f;
}
static uint32_t f2u_sat(real f) { /* Rust `as u32` */
  if (f != f || f <= R(0)) return 0;
  if (f >= R(4294967296.0)) return UINT32_MAX;
  return (uint32_t)f;
}

/* Perlin::noise perlin.rs:30-54 + trilinear_interp 74-96 */
static real perlin_noise(ctx_t* cx, const operlin* pl, vec3 p) {
  (void)cx;
  real fx = FLOOR(p.x), fy = FLOOR(p.y), fz = FLOOR(p.z);
  real u = p.x - fx, v = p.y - fy, w = p.z - fz;
  int32_t i = f2i_sat(fx), j = f2i_sat(fy), k = f2i_sat(fz);
  real uu = (u * u) * (R(3) - R(2) * u);
  real vv = (v * v) * (R(3) - R(2) * v);
  real ww = (w * w) * (R(3) - R(2) * w);
  real accum = R(0);
  for (int di = 0; di < 2; ++di)
    for (int dj = 0; dj < 2; ++dj)
      for (int dk = 0; dk < 2; ++dk) {
        int idx = pl->px[(uint32_t)(i + di) & 255] ^ pl->py[(uint32_t)(j + dj) & 255] ^
                  pl->pz[(uint32_t)(k + dk) & 255];
        vec3 cvec = pl->ranvec[idx];
        real wi = di ? uu : R(1) - uu;
        real wj = dj ? vv : R(1) - vv;
        real wk = dk ? ww : R(1) - ww;
        vec3 wv = v3(u - R(di), v - R(dj), w - R(dk));
        accum = FMA((wi * wj) * wk, dot(cvec, wv), accum);
      }
  return accum;
}
static real perlin_turb(ctx_t* cx, const operlin* pl, vec3 p) { /* perlin.rs:56-72 */
  real accum = R(0), weight = R(1);
  vec3 tp = p;
  for (int i = 0; i < 7; ++i) {
    accum = FMA(weight, perlin_noise(cx, pl, tp), accum);
    weight = weight * R(0.5);
    tp = vscale(tp, R(2));
  }
  return FABS(accum);
}

static vec3 tex_value(ctx_t* cx, int id, real u, real v, vec3 p) { /* texture.rs:17-26 */
  const oscene* sc = cx->sc;
  for (int guard = 0; guard < 64; ++guard) {
    const otex* t = &sc->texs[id];
    switch (t->kind) {
      case RT_TEX_SOLID: return t->color;
      case RT_TEX_CHECKER: { /* texture.rs:71-81 */
        int32_t x = f2i_sat(FLOOR(t->inv_scale * p.x));
        int32_t y = f2i_sat(FLOOR(t->inv_scale * p.y));
        int32_t z = f2i_sat(FLOOR(t->inv_scale * p.z));
        uint32_t sum = (uint32_t)x + (uint32_t)y + (uint32_t)z;
        id = (sum & 1u) == 0 ? t->even : t->odd;
        continue;
      }
      case RT_TEX_IMAGE: { /* texture.rs:95-107, rt_image.rs:37-46 */
        if (t->h <= 0 || t->w <= 0) return v3(R(0), R(1), R(1));
        real cu = u < R(0) ? R(0) : (u > R(1) ? R(1) : u);
        real cvv = v < R(0) ? R(0) : (v > R(1) ? R(1) : v);
        uint32_t i = f2u_sat(cu * R(t->w));
        uint32_t j = f2u_sat(cvv * R(t->h));
        uint32_t x = i < (uint32_t)(t->w - 1) ? i : (uint32_t)(t->w - 1);
        uint32_t y = (uint32_t)t->h - j - 1u;
        if (y > (uint32_t)(t->h - 1)) y = (uint32_t)(t->h - 1);
        const uint8_t* px = sc->texels + t->off + ((size_t)y * t->w + x) * 3;
        const real cs = R(1.0 / 255.0);
        return v3(R(px[0]) * cs, R(px[1]) * cs, R(px[2]) * cs);
      }
      case RT_TEX_NOISE: { /* texture.rs:127-130 */
        CNT(cx, RT_OP_NOISE_EVALS);
        vec3 s = vscale(p, t->scale);
        real turb = perlin_turb(cx, &sc->perlins[t->perlin], s);
        real k = R(0.5) * (R(1) + SIN(FMA(R(10), turb, s.z)));
        return v3(k, k, k);
      }
    }
    break;
  }
  return v3(R(0), R(0), R(0));
}

static int tex_needs_uv(const oscene* sc, int id) {
  for (int guard = 0; guard < 64; ++guard) {
    const otex* t = &sc->texs[id];
    if (t->kind == RT_TEX_IMAGE) return t->w > 0 && t->h > 0;
    if (t->kind != RT_TEX_CHECKER) return 0;
    if (tex_needs_uv(sc, t->even)) return 1;
    id = t->odd;
  }
  return 0;
}

/* get_sphere_uv object.rs:114-120, evaluated only when a texture reads (u, v) */
static void sphere_uv(vec3 p, real* u, real* v) {
  real theta = ACOS(-p.y);
  real phi = ATAN2(-p.z, p.x) + R(PI_D);
  *u = (phi * R(1.0 / PI_D)) * R(0.5);
  *v = theta * R(1.0 / PI_D);
}

/* =============================================================== PDFs */
typedef struct { vec3 u, v, w; } onb_t;
static onb_t onb_from_w(vec3 w) { /* onb.rs:32-47 */
  onb_t b;
  vec3 unit_w = unit_vector(w);
  vec3 a = FABS(unit_w.x) > R(0.9) ? v3(R(0), R(1), R(0)) : v3(R(1), R(0), R(0));
  vec3 v = unit_vector(cross(unit_w, a));
  b.u = cross(unit_w, v);
  b.v = v;
  b.w = unit_w;
  return b;
}
static vec3 onb_local(const onb_t* b, vec3 a) { /* onb.rs:24-26: (a*u + b*v) + c*w */
  return vadd(vadd(vscale(b->u, a.x), vscale(b->v, a.y)), vscale(b->w, a.z));
}
static vec3 random_cosine_direction(rng_t* g) { /* vec3.rs:240-250 */
  real r1 = rnd(g), r2 = rnd(g);
  real s, c;
  sincos2pi(r1, &s, &c);
  real sq = SQRT(r2);
  return v3(c * sq, s * sq, SQRT(R(1) - r2));
}
static vec3 random_unit_vector(rng_t* g) { /* vec3.rs:215-217, 231-238 */
  for (;;) {
    real x = rnd_range(g, R(-1), R(1));
    real y = rnd_range(g, R(-1), R(1));
    real z = rnd_range(g, R(-1), R(1));
    vec3 p = v3(x, y, z);
    if (dot(p, p) < R(1)) return unit_vector(p);
  }
}

/* Hittable::pdf_value / random for the light object (object.rs:190-212, 492-506; hittable.rs:115-129) */
static real light_pdf_value(ctx_t* cx, int id, vec3 origin, vec3 dir) {
  const oscene* sc = cx->sc;
  const onode* n = &sc->nodes[id];
  ray_t r = {origin, dir, R(0)};
  hitrec rec;
  if (n->tag == RT_OBJ_QUAD) {
    CNT(cx, RT_OP_LIGHT_PDF_QUAD);
    if (!quad_hit(cx, n, &r, R(0.001), R(INFINITY), &rec)) return R(0);
    real len2 = dot(dir, dir);
    real dist2 = (rec.t * rec.t) * len2;
    real cosine = FABS(dot(dir, rec.normal) / SQRT(len2));
    return dist2 / (cosine * n->area);
  }
  if (n->tag == RT_OBJ_SPHERE) {
    CNT(cx, RT_OP_LIGHT_PDF_SPHERE);
    if (!sphere_hit(cx, n, id, &r, R(0.001), R(INFINITY), &rec)) return R(0);
    vec3 cmo = vsub(n->c, origin);
    real cos_max = SQRT(R(1) - (n->radius * n->radius) / dot(cmo, cmo));
    real solid = R(2 * PI_D) * (R(1) - cos_max);
    return R(1) / solid;
  }
  if (n->tag == RT_OBJ_LIST) {
    real weight = R(1) / R(n->count);
    real sum = R(0);
    for (int i = 0; i < n->count; ++i) {
      real pv = light_pdf_value(cx, sc->kids[n->first + i], origin, dir);
      sum = i == 0 ? pv : sum + pv; /* reduce(|x, y| x + y) */
    }
    return sum * weight;
  }
  return R(0);
}
static vec3 light_random(ctx_t* cx, int id, vec3 origin, rng_t* g) {
  const oscene* sc = cx->sc;
  const onode* n = &sc->nodes[id];
  if (n->tag == RT_OBJ_QUAD) {
    real a = rnd(g);
    real b = rnd(g);
    vec3 p = vfma(b, n->v, vfma(a, n->u, n->q));
    return vsub(p, origin);
  }
  if (n->tag == RT_OBJ_SPHERE) {
    vec3 direction = vsub(n->c, origin);
    real dist2 = dot(direction, direction);
    onb_t b = onb_from_w(direction);
    real r1 = rnd(g), r2 = rnd(g); /* random_to_sphere object.rs:122-132 */
    real k = SQRT(R(1) - (n->radius * n->radius) / dist2) - R(1);
    real z = FMA(r2, k, R(1));
    real s, c;
    sincos2pi(r1, &s, &c);
    real sq = SQRT(FMA(-z, z, R(1)));
    return onb_local(&b, v3(c * sq, s * sq, z));
  }
  if (n->tag == RT_OBJ_LIST) {
    if (n->count == 0) return v3(R(1), R(0), R(0)); /* reference panics (S1) */
    uint32_t i = rnd_index(g, (uint32_t)n->count);
    return light_random(cx, sc->kids[n->first + i], origin, g);
  }
  return v3(R(1), R(0), R(0));
}

/* =============================================================== ray_color (render.rs:251-311) */
typedef struct { vec3 bg; int max_depth; } camctx;

static vec3 ray_color(ctx_t* cx, const camctx* cc, const ray_t* r, int depth, rng_t* g) {
  const oscene* sc = cx->sc;
  if (depth <= 0) {
    CNT(cx, RT_OP_DEPTH_CUTOFF);
    return v3(R(0), R(0), R(0));
  }
  CNT(cx, RT_OP_WORLD_QUERIES);
  hitrec rec;
  if (!obj_hit(cx, sc->world, r, R(0.0001), R(INFINITY), &rec)) {
    CNT(cx, RT_OP_MISSES);
    return cc->bg;
  }
  const omat* m = &sc->mats[rec.mat];
  int mk = m->kind;
  /* texture (u,v): quads carry (a, b); spheres compute get_sphere_uv lazily */
  if ((mk == RT_MAT_LAMBERTIAN || mk == RT_MAT_DIFFUSE_LIGHT || mk == RT_MAT_ISOTROPIC) &&
      rec.node >= 0 && sc->nodes[rec.node].tag == RT_OBJ_SPHERE && tex_needs_uv(sc, m->tex))
    sphere_uv(rec.outward_local, &rec.u, &rec.v);

  if (mk == RT_MAT_DIFFUSE_LIGHT) { /* material.rs:210-222 */
    CNT(cx, RT_OP_EMISSIVE_HITS);
    return rec.front ? tex_value(cx, m->tex, rec.u, rec.v, rec.p) : v3(R(0), R(0), R(0));
  }
  if (mk == RT_MAT_METAL) { /* material.rs:124-134 */
    CNT(cx, RT_OP_METAL);
    vec3 reflected = reflect(unit_vector(r->d), rec.normal);
    vec3 ruv = random_unit_vector(g);
    reflected = vfma(m->fuzz, ruv, unit_vector(reflected));
    ray_t sr = {rec.p, reflected, r->tm};
    return vmul(m->color, ray_color(cx, cc, &sr, depth - 1, g));
  }
  if (mk == RT_MAT_DIELECTRIC) { /* material.rs:166-191 */
    CNT(cx, RT_OP_DIELECTRIC);
    real ratio = rec.front ? R(1) / m->ir : m->ir;
    vec3 ud = unit_vector(r->d);
    real cos_t = min1(dot(vneg(ud), rec.normal));
    real sin_t = SQRT(FMA(-cos_t, cos_t, R(1)));
    int cannot = ratio * sin_t > R(1);
    int refl = cannot;
    if (!cannot) {
      real r0 = (R(1) - ratio) / (R(1) + ratio); /* Dielectric::reflectance material.rs:156-163 */
      r0 = r0 * r0;
      real reflectance = r0 + (R(1) - r0) * POW(R(1) - cos_t, R(5));
      refl = reflectance > rnd(g);
    }
    vec3 dir = refl ? reflect(ud, rec.normal) : refract(ud, rec.normal, ratio);
    ray_t sr = {rec.p, dir, r->tm};
    return vmul(m->color, ray_color(cx, cc, &sr, depth - 1, g));
  }
  /* Lambertian / Isotropic: PdfPtr branch (render.rs:278-292) */
  int iso = mk == RT_MAT_ISOTROPIC;
  CNT(cx, iso ? RT_OP_ISOTROPIC : RT_OP_LAMBERTIAN);
  vec3 atten = tex_value(cx, m->tex, rec.u, rec.v, rec.p);
  onb_t uvw;
  if (!iso) uvw = onb_from_w(rec.normal); /* CosinePDF::new pdf.rs:58-62 */
  int have_lights = sc->lights >= 0;
  vec3 dir;
  real pdf_val;
  if (have_lights) {
    real mix = rnd(g); /* MixturePDF::generate pdf.rs:120-126 */
    if (mix < R(0.5)) {
      CNT(cx, RT_OP_LIGHT_GEN);
      dir = light_random(cx, sc->lights, rec.p, g);
    } else {
      CNT(cx, RT_OP_COSINE_GEN);
      dir = iso ? random_unit_vector(g) : onb_local(&uvw, random_cosine_direction(g));
    }
  } else {
    CNT(cx, RT_OP_COSINE_GEN);
    dir = iso ? random_unit_vector(g) : onb_local(&uvw, random_cosine_direction(g));
  }
  vec3 udir = unit_vector(dir);
  real mat_pdf;
  if (iso) {
    mat_pdf = R(1.0 / (4.0 * PI_D)); /* SpherePDF::value pdf.rs:47-49 */
  } else {
    real cth = dot(udir, uvw.w); /* CosinePDF::value pdf.rs:69-73: max(0, cos / PI) */
    real v = cth / R(PI_D);
    mat_pdf = v > R(0) ? v : R(0);
  }
  if (have_lights) {
    real lp = light_pdf_value(cx, sc->lights, rec.p, dir);
    pdf_val = FMA(R(0.5), lp, R(0.5) * mat_pdf);
  } else {
    pdf_val = mat_pdf;
  }
  real s_pdf;
  if (iso) {
    s_pdf = (cx->flags & RT_FLAG_SEMANTICS_REFERENCE) ? R(0) : R(1.0 / (4.0 * PI_D));
  } else {
    real cth = dot(rec.normal, udir); /* Lambertian::scattering_pdf material.rs:100-108 */
    s_pdf = cth < R(0) ? R(0) : cth / R(PI_D);
  }
  ray_t sr = {rec.p, dir, r->tm};
  vec3 L = ray_color(cx, cc, &sr, depth - 1, g);
  /* (attenuation * scattering_pdf * sample_color) / pdf_val  (render.rs:289-290) */
  vec3 cs = vmul(vscale(atten, s_pdf), L);
  return v3(cs.x / pdf_val, cs.y / pdf_val, cs.z / pdf_val); /* + emission (0 off lights) */
}

/* =============================================================== camera (render.rs:218-249) */
typedef struct {
  vec3 center, p00, du, dv, ddu, ddv;
  real rs, defocus;
  int W, H, sqrt_spp;
} ocam;

static ray_t get_ray(const ocam* c, int i, int j, int s_i, int s_j, rng_t* g) {
  vec3 pc = vfma(R(j), c->dv, vfma(R(i), c->du, c->p00));
  real px = FMA(c->rs, R(s_i) + rnd(g), R(-0.5));
  real py = FMA(c->rs, R(s_j) + rnd(g), R(-0.5));
  vec3 ps = vadd(pc, vfma(px, c->du, vscale(c->dv, py)));
  vec3 origin = c->center;
  if (c->defocus > R(0)) { /* defocus_disk_sample render.rs:238-241 */
    for (;;) {
      real x = rnd_range(g, R(-1), R(1));
      real y = rnd_range(g, R(-1), R(1));
      vec3 p = v3(x, y, R(0));
      if (dot(p, p) < R(1)) {
        origin = vfma(p.y, c->ddv, vfma(p.x, c->ddu, c->center));
        break;
      }
    }
  }
  ray_t r;
  r.o = origin;
  r.d = vsub(ps, origin);
  r.tm = rnd(g);
  return r;
}

/* =============================================================== render loop */
typedef struct {
  const oscene* sc;
  ocam cam;
  camctx cc;
  const rt_render_opts* opts;
  float* accum;
  int sj0, sj1;
  int n_chunks, chunk_rows;
  volatile int next_chunk;
  pthread_mutex_t mu;
  uint64_t ops[RT_OP_COUNT];
} job_t;

static void render_pixel(ctx_t* cx, job_t* jb, int x, int y, float* out) {
  const ocam* c = &jb->cam;
  uint32_t pixel = (uint32_t)(y * c->W + x);
  /* render.rs:185-189: one running sum per pixel over s_j (outer) and s_i (inner) */
  real tot[3] = {R(0), R(0), R(0)};
  for (int s_j = jb->sj0; s_j < jb->sj1; ++s_j) {
    for (int s_i = 0; s_i < c->sqrt_spp; ++s_i) {
      rng_t g;
      rng_seed(&g, jb->opts->seed, pixel, (uint32_t)(s_j * c->sqrt_spp + s_i));
      t_rng = &g;
      CNT(cx, RT_OP_SAMPLES);
      ray_t r = get_ray(c, x, y, s_i, s_j, &g);
      vec3 col = ray_color(cx, &jb->cc, &r, jb->cc.max_depth, &g);
      tot[0] += col.x;
      tot[1] += col.y;
      tot[2] += col.z;
    }
  }
  int ow = jb->opts->flags & RT_FLAG_OVERWRITE;
  for (int k = 0; k < 3; ++k) out[k] = ow ? (float)tot[k] : (float)((real)out[k] + tot[k]);
}

static void* worker(void* arg) {
  job_t* jb = (job_t*)arg;
  ctx_t cx;
  memset(&cx, 0, sizeof(cx));
  cx.sc = jb->sc;
  cx.flags = jb->opts->flags;
  int W = jb->cam.W;
  for (;;) {
    int ch = __atomic_fetch_add(&jb->next_chunk, 1, __ATOMIC_RELAXED);
    if (ch >= jb->n_chunks) break;
    int k0 = ch * jb->chunk_rows, k1 = k0 + jb->chunk_rows;
    if (k1 > jb->opts->n_rows) k1 = jb->opts->n_rows;
    for (int k = k0; k < k1; ++k) {
      int y = jb->opts->row_begin + k * jb->opts->row_step;
      for (int x = 0; x < W; ++x) render_pixel(&cx, jb, x, y, jb->accum + ((size_t)k * W + x) * 3);
    }
  }
  pthread_mutex_lock(&jb->mu);
  for (int k = 0; k < RT_OP_COUNT; ++k) jb->ops[k] += cx.ops[k];
  pthread_mutex_unlock(&jb->mu);
  return NULL;
}

static void load_cam(const rt_camera* c, ocam* o) {
#define L3(a) v3(R((a)[0]), R((a)[1]), R((a)[2]))
  o->center = L3(c->center);
  o->p00 = L3(c->pixel00_loc);
  o->du = L3(c->pixel_delta_u);
  o->dv = L3(c->pixel_delta_v);
  o->ddu = L3(c->defocus_disk_u);
  o->ddv = L3(c->defocus_disk_v);
#undef L3
  o->rs = R(c->recip_sqrt_spp);
  o->defocus = R(c->defocus_angle);
  o->W = c->image_width;
  o->H = c->image_height;
  o->sqrt_spp = c->sqrt_spp;
}

static int has_pdf_material(const oscene* sc) {
  for (int i = 0; i < sc->n_mats; ++i)
    if (sc->mats[i].kind == RT_MAT_LAMBERTIAN || sc->mats[i].kind == RT_MAT_ISOTROPIC) return 1;
  return 0;
}

EXPORT int oracle_precision_bits(void) { return ORACLE_F64 ? 64 : 32; }

/* Render rows [row_begin + k*row_step, k < n_rows] exactly as rt_render (same opts meaning). */
EXPORT int oracle_render(const rt_scene_blob* blob, const rt_camera* cam, const rt_render_opts* opts,
                         float* accum, uint64_t* ops_out, int n_threads) {
  if (!blob || !cam || !opts || !accum) return RT_ERR_INVALID_ARG;
  if (cam->sqrt_spp <= 0 || cam->image_width <= 0 || opts->n_rows < 0 || opts->row_step <= 0)
    return RT_ERR_INVALID_ARG;
  job_t jb;
  memset(&jb, 0, sizeof(jb));
  oscene sc;
  int rc = parse_scene(blob, &sc);
  if (rc) return rc;
  if (sc.lights < 0 && (opts->flags & RT_FLAG_SEMANTICS_REFERENCE) && has_pdf_material(&sc)) {
    free_scene(&sc);
    return RT_ERR_EMPTY_LIGHTS;
  }
  jb.sc = &sc;
  load_cam(cam, &jb.cam);
  jb.cc.bg = v3(R(cam->background[0]), R(cam->background[1]), R(cam->background[2]));
  jb.cc.max_depth = cam->max_depth;
  jb.opts = opts;
  jb.accum = accum;
  jb.sj0 = opts->sj_count > 0 ? opts->sj_begin : 0;
  jb.sj1 = opts->sj_count > 0 ? opts->sj_begin + opts->sj_count : cam->sqrt_spp;
  if (jb.sj0 < 0 || jb.sj1 > cam->sqrt_spp) {
    free_scene(&sc);
    return RT_ERR_INVALID_ARG;
  }
  jb.chunk_rows = 3; /* render.rs:171: chunk = 3 image rows */
  jb.n_chunks = (opts->n_rows + jb.chunk_rows - 1) / jb.chunk_rows;
  pthread_mutex_init(&jb.mu, NULL);
  if (n_threads < 1) n_threads = 1;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * n_threads);
  for (int i = 0; i < n_threads; ++i) pthread_create(&th[i], NULL, worker, &jb);
  for (int i = 0; i < n_threads; ++i) pthread_join(th[i], NULL);
  free(th);
  pthread_mutex_destroy(&jb.mu);
  if (ops_out)
    for (int k = 0; k < RT_OP_COUNT; ++k) ops_out[k] = jb.ops[k];
  free_scene(&sc);
  return RT_OK;
}

/* ---- unit entry points for known-answer tests ------------------------------------------ */
EXPORT void oracle_rng_draws(uint64_t seed, uint32_t pixel, uint32_t sample, int n, double* out) {
  rng_t g;
  rng_seed(&g, seed, pixel, sample);
  for (int i = 0; i < n; ++i) out[i] = (double)rnd(&g);
}
EXPORT void oracle_rng_u32(uint64_t seed, uint32_t pixel, uint32_t sample, int n, uint32_t* out) {
  rng_t g;
  rng_seed(&g, seed, pixel, sample);
  for (int i = 0; i < n; ++i) out[i] = rng_u32(&g);
}
/* get_sphere_uv (object.rs:114-120) at unit-sphere points p[3*i..] -> uv[2*i..] */
/* Perlin::turb (perlin.rs:56-72 over noise 30-54 and trilinear_interp 74-96) of one table:
 * ranvec 256 x 3 doubles, perms 3 x 256 (perm_x, perm_y, perm_z), n points. KAT entry. */
EXPORT void oracle_perlin_turb(const double* ranvec, const int* perms, const double* pts, int n,
                               double* out) {
  operlin pl;
  for (int k = 0; k < 256; ++k) {
    pl.ranvec[k] = v3(R(ranvec[3 * k]), R(ranvec[3 * k + 1]), R(ranvec[3 * k + 2]));
    pl.px[k] = perms[k];
    pl.py[k] = perms[256 + k];
    pl.pz[k] = perms[512 + k];
  }
  for (int i = 0; i < n; ++i)
    out[i] = (double)perlin_turb(NULL, &pl, v3(R(pts[3 * i]), R(pts[3 * i + 1]), R(pts[3 * i + 2])));
}
EXPORT void oracle_sphere_uv(const double* p, int n, double* uv) {
  for (int i = 0; i < n; ++i) {
    real u, v;
    sphere_uv(v3(R(p[3 * i]), R(p[3 * i + 1]), R(p[3 * i + 2])), &u, &v);
    uv[2 * i] = (double)u;
    uv[2 * i + 1] = (double)v;
  }
}
/* HittablePDF::value of the scene's light object at `origin` for n directions. */
EXPORT int oracle_light_pdf_batch(const rt_scene_blob* blob, const double* origin3, const double* dirs,
                                  int n, double* out) {
  oscene sc;
  if (parse_scene(blob, &sc)) return -1;
  if (sc.lights < 0) {
    free_scene(&sc);
    return -2;
  }
  ctx_t cx;
  memset(&cx, 0, sizeof(cx));
  cx.sc = &sc;
  vec3 o = v3(R(origin3[0]), R(origin3[1]), R(origin3[2]));
  for (int i = 0; i < n; ++i)
    out[i] = (double)light_pdf_value(&cx, sc.lights, o, v3(R(dirs[3 * i]), R(dirs[3 * i + 1]), R(dirs[3 * i + 2])));
  free_scene(&sc);
  return 0;
}
/* n light-PDF generate() draws at `origin` with the stream of (seed, 0, k): dirs[3*k..] */
EXPORT int oracle_light_generate(const rt_scene_blob* blob, const double* origin3, uint64_t seed, int n,
                                 double* dirs) {
  oscene sc;
  if (parse_scene(blob, &sc)) return -1;
  if (sc.lights < 0) {
    free_scene(&sc);
    return -2;
  }
  ctx_t cx;
  memset(&cx, 0, sizeof(cx));
  cx.sc = &sc;
  vec3 o = v3(R(origin3[0]), R(origin3[1]), R(origin3[2]));
  for (int k = 0; k < n; ++k) {
    rng_t g;
    rng_seed(&g, seed, 0, (uint32_t)k);
    vec3 d = light_random(&cx, sc.lights, o, &g);
    dirs[3 * k] = d.x, dirs[3 * k + 1] = d.y, dirs[3 * k + 2] = d.z;
  }
  free_scene(&sc);
  return 0;
}
/* n cosine-PDF directions about unit normal w (onb.rs + vec3.rs:240-250) */
EXPORT void oracle_cosine_dirs(const double* w3, uint64_t seed, int n, double* dirs) {
  onb_t b = onb_from_w(v3(R(w3[0]), R(w3[1]), R(w3[2])));
  for (int k = 0; k < n; ++k) {
    rng_t g;
    rng_seed(&g, seed, 1, (uint32_t)k);
    vec3 d = onb_local(&b, random_cosine_direction(&g));
    dirs[3 * k] = d.x, dirs[3 * k + 1] = d.y, dirs[3 * k + 2] = d.z;
  }
}
EXPORT void oracle_fmath(int fn, const float* x, const float* y, int n, float* out) {
  for (int i = 0; i < n; ++i) {
    float s, c;
    switch (fn) {
      case 0: f32_sincos2pi(x[i], &s, &c); out[i] = s; break;
      case 1: f32_sincos2pi(x[i], &s, &c); out[i] = c; break;
      case 2: out[i] = f32_log(x[i]); break;
      case 3: out[i] = f32_sin(x[i]); break;
      case 4: out[i] = f32_acos(x[i]); break;
      case 5: out[i] = f32_atan2(x[i], y[i]); break;
      default: out[i] = 0.f;
    }
  }
}
/* Camera ray for (i, j, s_i, s_j) with the sample's own stream: origin[3], dir[3], time. */
EXPORT void oracle_camera_ray(const rt_camera* cam, uint64_t seed, int i, int j, int s_i, int s_j,
                              double* out7) {
  ocam c;
  load_cam(cam, &c);
  rng_t g;
  rng_seed(&g, seed, (uint32_t)(j * cam->image_width + i), (uint32_t)(s_j * cam->sqrt_spp + s_i));
  ray_t r = get_ray(&c, i, j, s_i, s_j, &g);
  double v[7] = {r.o.x, r.o.y, r.o.z, r.d.x, r.d.y, r.d.z, r.tm};
  memcpy(out7, v, sizeof(v));
}
/* world.hit for one ray (t, p[3], normal[3], front, mat) — returns 1 on hit. */
EXPORT int oracle_world_hit(const rt_scene_blob* blob, const double* ray7, double tmin, double tmax,
                            double* out9) {
  oscene sc;
  if (parse_scene(blob, &sc)) return -1;
  ctx_t cx;
  memset(&cx, 0, sizeof(cx));
  cx.sc = &sc;
  rng_t g;
  rng_seed(&g, 0, 0, 0);
  t_rng = &g;
  ray_t r = {v3(R(ray7[0]), R(ray7[1]), R(ray7[2])), v3(R(ray7[3]), R(ray7[4]), R(ray7[5])), R(ray7[6])};
  hitrec rec;
  int h = obj_hit(&cx, sc.world, &r, R(tmin), R(tmax), &rec);
  if (h) {
    double v[9] = {rec.t, rec.p.x, rec.p.y, rec.p.z, rec.normal.x, rec.normal.y, rec.normal.z,
                   (double)rec.front, (double)rec.mat};
    memcpy(out9, v, sizeof(v));
  }
  free_scene(&sc);
  return h;
}
/* Light-PDF value and a generated direction at `origin` (pdf.rs:80-100): out = [pdf, dir3]. */
EXPORT int oracle_light_pdf(const rt_scene_blob* blob, const double* origin3, const double* dir3,
                            double* pdf_out) {
  oscene sc;
  if (parse_scene(blob, &sc)) return -1;
  if (sc.lights < 0) {
    free_scene(&sc);
    return -2;
  }
  ctx_t cx;
  memset(&cx, 0, sizeof(cx));
  cx.sc = &sc;
  *pdf_out = (double)light_pdf_value(&cx, sc.lights, v3(R(origin3[0]), R(origin3[1]), R(origin3[2])),
                                     v3(R(dir3[0]), R(dir3[1]), R(dir3[2])));
  free_scene(&sc);
  return 0;
}
