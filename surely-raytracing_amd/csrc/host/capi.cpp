// capi.cpp — C API (include/rt_host.h) over the C++ scene builder, plus the host output stage
// (color.rs write_color / linear_to_gamma / exposure, render.rs auto_expose + P3 header).
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../../include/rt_host.h"
#include "scene.hpp"

using namespace rt;

struct rth_scene {
  explicit rth_scene(uint64_t seed) : rng(seed) {}
  SceneRng rng;
  std::vector<TexturePtr> textures;
  std::vector<MaterialPtr> materials;
  std::vector<ObjectPtr> objects;
  std::vector<uint64_t> blob;
  std::vector<uint8_t> texels;
};

static thread_local std::string g_err;

static int32_t fail(const std::string& msg) {
  g_err = msg;
  return -1;
}

extern "C" const char* rth_last_error(void) { return g_err.c_str(); }

static Vec3 v3(const double* p) { return Vec3(p[0], p[1], p[2]); }

template <class T>
static int32_t push(std::vector<T>& vec, T v) {
  vec.push_back(std::move(v));
  return (int32_t)vec.size() - 1;
}

#define CHECK_S(s) \
  if (!(s)) return fail("null scene")
#define TEX(s, id) (((id) >= 0 && (size_t)(id) < (s)->textures.size()) ? (s)->textures[id] : nullptr)
#define MAT(s, id) (((id) >= 0 && (size_t)(id) < (s)->materials.size()) ? (s)->materials[id] : nullptr)
#define OBJ(s, id) (((id) >= 0 && (size_t)(id) < (s)->objects.size()) ? (s)->objects[id] : nullptr)

extern "C" {

rth_scene* rth_scene_new(uint64_t build_seed) { return new rth_scene(build_seed); }
void rth_scene_free(rth_scene* s) { delete s; }
double rth_random_double(rth_scene* s) { return s->rng.random_double(); }
double rth_random_range(rth_scene* s, double mn, double mx) { return s->rng.random_range(mn, mx); }
int64_t rth_random_int(rth_scene* s, int64_t mn, int64_t mx) { return s->rng.random_int(mn, mx); }

int32_t rth_solid_color(rth_scene* s, double r, double g, double b) {
  CHECK_S(s);
  return push(s->textures, SolidColor({r, g, b}));
}
int32_t rth_checker_texture(rth_scene* s, double scale, int32_t even, int32_t odd) {
  CHECK_S(s);
  auto e = TEX(s, even), o = TEX(s, odd);
  if (!e || !o) return fail("checker: bad texture id");
  return push(s->textures, CheckerTexture(scale, e, o));
}
int32_t rth_noise_texture(rth_scene* s, double scale) {
  CHECK_S(s);
  return push(s->textures, NoiseTexture(scale, s->rng));
}
int32_t rth_image_texture(rth_scene* s, int32_t w, int32_t h, const uint8_t* rgb8) {
  CHECK_S(s);
  if (w < 0 || h < 0) return fail("image: negative size");
  return push(s->textures, ImageTexture(w, h, rgb8));
}

static int32_t mat_with_tex(rth_scene* s, int32_t tex, MaterialPtr (*ctor)(TexturePtr)) {
  CHECK_S(s);
  auto t = TEX(s, tex);
  if (!t) return fail("bad texture id");
  return push(s->materials, ctor(t));
}
int32_t rth_lambertian(rth_scene* s, double r, double g, double b) {
  return mat_with_tex(s, rth_solid_color(s, r, g, b), Lambertian);
}
int32_t rth_lambertian_tex(rth_scene* s, int32_t tex) { return mat_with_tex(s, tex, Lambertian); }
int32_t rth_metal(rth_scene* s, double r, double g, double b, double fuzz) {
  CHECK_S(s);
  return push(s->materials, Metal({r, g, b}, fuzz));
}
int32_t rth_dielectric(rth_scene* s, double ir, double r, double g, double b) {
  CHECK_S(s);
  return push(s->materials, Dielectric(ir, {r, g, b}));
}
int32_t rth_diffuse_light(rth_scene* s, double r, double g, double b) {
  return mat_with_tex(s, rth_solid_color(s, r, g, b), DiffuseLight);
}
int32_t rth_diffuse_light_tex(rth_scene* s, int32_t tex) { return mat_with_tex(s, tex, DiffuseLight); }
int32_t rth_isotropic(rth_scene* s, double r, double g, double b) {
  return mat_with_tex(s, rth_solid_color(s, r, g, b), Isotropic);
}
int32_t rth_isotropic_tex(rth_scene* s, int32_t tex) { return mat_with_tex(s, tex, Isotropic); }

int32_t rth_sphere(rth_scene* s, const double c[3], double radius, int32_t mat) {
  CHECK_S(s);
  auto m = MAT(s, mat);
  if (!m) return fail("sphere: bad material id");
  return push(s->objects, Sphere(v3(c), radius, m));
}
int32_t rth_sphere_moving(rth_scene* s, const double c1[3], const double c2[3], double radius,
                          int32_t mat) {
  CHECK_S(s);
  auto m = MAT(s, mat);
  if (!m) return fail("sphere: bad material id");
  return push(s->objects, SphereMoving(v3(c1), v3(c2), radius, m));
}
int32_t rth_quad(rth_scene* s, const double q[3], const double u[3], const double v[3],
                 int32_t mat) {
  CHECK_S(s);
  auto m = MAT(s, mat);
  if (!m) return fail("quad: bad material id");
  return push(s->objects, Quad(v3(q), v3(u), v3(v), m));
}
int32_t rth_make_box(rth_scene* s, const double a[3], const double b[3], int32_t mat) {
  CHECK_S(s);
  auto m = MAT(s, mat);
  if (!m) return fail("make_box: bad material id");
  return push(s->objects, make_box(v3(a), v3(b), m));
}
int32_t rth_list_new(rth_scene* s) {
  CHECK_S(s);
  return push(s->objects, HittableList());
}
int32_t rth_list_add(rth_scene* s, int32_t list, int32_t obj) {
  CHECK_S(s);
  auto l = OBJ(s, list), o = OBJ(s, obj);
  if (!l || l->tag != RT_OBJ_LIST) return fail("list_add: not a list");
  if (!o) return fail("list_add: bad object id");
  if (o.get() == l.get()) return fail("list_add: a list cannot contain itself");
  list_add(l, o);
  return 0;
}
int32_t rth_list_create_bvh(rth_scene* s, int32_t list) {
  CHECK_S(s);
  auto l = OBJ(s, list);
  if (!l || l->tag != RT_OBJ_LIST) return fail("create_bvh: not a list");
  if (l->objects.empty()) return fail("create_bvh: empty list");  // reference indexes [0] and panics
  return push(s->objects, create_bvh(l, s->rng));
}
int32_t rth_list_len(rth_scene* s, int32_t list) {
  CHECK_S(s);
  auto l = OBJ(s, list);
  if (!l || l->tag != RT_OBJ_LIST) return fail("list_len: not a list");
  return (int32_t)l->objects.size();
}
int32_t rth_translate(rth_scene* s, int32_t obj, const double off[3]) {
  CHECK_S(s);
  auto o = OBJ(s, obj);
  if (!o) return fail("translate: bad object id");
  return push(s->objects, Translate(o, v3(off)));
}
int32_t rth_rotate_y(rth_scene* s, int32_t obj, double angle) {
  CHECK_S(s);
  auto o = OBJ(s, obj);
  if (!o) return fail("rotate_y: bad object id");
  return push(s->objects, RotateY(o, angle));
}
int32_t rth_constant_medium(rth_scene* s, int32_t boundary, double density, double r, double g,
                            double b) {
  return rth_constant_medium_tex(s, boundary, density, rth_solid_color(s, r, g, b));
}
int32_t rth_constant_medium_tex(rth_scene* s, int32_t boundary, double density, int32_t tex) {
  CHECK_S(s);
  auto o = OBJ(s, boundary);
  auto t = TEX(s, tex);
  if (!o || !t) return fail("constant_medium: bad id");
  return push(s->objects, ConstantMedium(o, density, t));
}
int rth_object_bbox(rth_scene* s, int32_t obj, double out6[6]) {
  CHECK_S(s);
  auto o = OBJ(s, obj);
  if (!o) return fail("bbox: bad object id");
  const Aabb& b = o->bbox;
  double v[6] = {b.x.min, b.x.max, b.y.min, b.y.max, b.z.min, b.z.max};
  std::memcpy(out6, v, sizeof(v));
  return 0;
}

int rth_serialize(rth_scene* s, int32_t world_list, int32_t lights, rt_scene_blob* out) {
  CHECK_S(s);
  auto w = OBJ(s, world_list);
  if (!w || w->tag != RT_OBJ_LIST) return fail("serialize: world must be a HittableList");
  ObjectPtr l;
  if (lights >= 0) {
    l = OBJ(s, lights);
    if (!l) return fail("serialize: bad lights id");
  }
  s->blob = serialize(w, l, &s->texels);
  out->slots = s->blob.data();
  out->n_slots = s->blob.size();
  out->texels = s->texels.empty() ? nullptr : s->texels.data();
  out->n_texels = s->texels.size();
  return 0;
}

int rth_camera_new(double aspect_ratio, int32_t image_width, int32_t spp, int32_t max_depth,
                   double vfov, const double lookfrom[3], const double lookat[3],
                   const double vup[3], double defocus_angle, double focus_dist,
                   const double background[3], rt_camera* out) {
  if (!out || image_width <= 0 || spp <= 0 || max_depth < 0 || !(aspect_ratio > 0))
    return fail("camera: invalid arguments");
  *out = camera_new(aspect_ratio, image_width, spp, max_depth, vfov, v3(lookfrom), v3(lookat),
                    v3(vup), defocus_angle, focus_dist, v3(background));
  return 0;
}

int rth_preset(rth_scene* s, const char* name, const char* variant, int32_t width, int32_t spp,
               int32_t depth, double aspect, int32_t* world_out, int32_t* lights_out,
               rt_camera* cam_out) {
  CHECK_S(s);
  Preset p;
  std::string err;
  if (!preset(name ? name : "", variant ? variant : "", s->rng, width, spp, depth, aspect, &p, &err))
    return fail(err);
  *world_out = push(s->objects, p.world);
  *lights_out = p.lights ? push(s->objects, p.lights) : -1;
  *cam_out = p.cam;
  return 0;
}

// ---------------------------------------------------------------- output stage (color.rs)
static double linear_to_gamma(double linear) {  // color.rs:53-59
  if (linear <= 0.0031308) return 12.92 * linear;
  return 1.055 * std::pow(linear, 1. / 2.4) - 0.055;
}
static double exposure(double linear, double v) {  // color.rs:37-39: 1 - E^(-v*linear)
  return 1. - std::pow(2.718281828459045, -v * linear);
}
// Rust `f64 as u8`: saturating, NaN -> 0.
static uint8_t as_u8(double x) {
  if (!(x == x)) return 0;
  if (x <= 0.) return 0;
  if (x >= 255.) return 255;
  return (uint8_t)x;
}

double rth_auto_expose(const float* accum, int64_t n, int32_t spp) {  // render.rs:325-339
  double medium_weight = 1. / (double)n;
  double medium_point = 0.;
  for (int64_t i = 0; i < n; ++i) {
    double lum = 0.2126 * accum[3 * i] + 0.71516 * accum[3 * i + 1] + 0.072169 * accum[3 * i + 2];
    medium_point = medium_point + medium_weight * (lum * lum);
  }
  medium_point = medium_point / (double)((int64_t)spp * spp);
  if (medium_point > 0.001) return -std::log(0.6) / std::sqrt(medium_point);
  return 1.;
}

int rth_write_color(const float* accum, int64_t n, double spp, int use_exposure, double ev,
                    uint8_t* out) {  // color.rs:8-33
  double scale = 1.0 / spp;
  for (int64_t i = 0; i < 3 * n; ++i) {
    double x = (double)accum[i] * scale;
    if (use_exposure) x = exposure(x, ev);
    x = linear_to_gamma(x);
    if (x < 0.) x = 0.;             // Interval{0, 0.999}.clamp (interval.rs:29-37)
    else if (x > 0.999) x = 0.999;  // NaN falls through both tests, as in the reference
    out[i] = as_u8(256. * x);
  }
  return 0;
}

int rth_write_ppm(const char* path, const uint8_t* rgb, int32_t w, int32_t h) {
  // Same text as render.rs:151 + write_color's "r g b\n" lines.
  FILE* f = std::fopen(path, "w");
  if (!f) return fail(std::string("cannot open ") + path);
  std::fprintf(f, "P3\n%d %d\n255\n", w, h);
  for (int64_t i = 0; i < (int64_t)w * h; ++i)
    std::fprintf(f, "%d %d %d\n", rgb[3 * i], rgb[3 * i + 1], rgb[3 * i + 2]);
  std::fclose(f);
  return 0;
}

}  // extern "C"
