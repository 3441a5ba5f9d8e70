// scene.hpp — host-side scene model: the reference's construction API restated in C++.
//
// The reference builds scenes with Rust constructors that precompute geometry in f64
// (Quad::new object.rs:427-446, Sphere::new/new_moving object.rs:83-105, RotateY::new
// transform.rs:143-186, Translate::new transform.rs:43-54, BvhNode::new hittable.rs:147-187,
// Perlin::new perlin.rs:15-28). This file keeps that vocabulary and arithmetic; Serializer
// flattens the resulting object graph into the rt_scene_blob format of include/rt_mi355x.h.
// Nothing here runs per sample: the per-pixel loop lives behind the C ABI.
#pragma once

#include <cmath>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "../../../include/rt_mi355x.h"

namespace rt {

struct Vec3 {
  double x = 0, y = 0, z = 0;
  Vec3() = default;
  Vec3(double a, double b, double c) : x(a), y(b), z(c) {}
  double dim(int n) const { return n == 0 ? x : (n == 1 ? y : z); }
  void set(int n, double v) { (n == 0 ? x : (n == 1 ? y : z)) = v; }
  double length_squared() const { return x * x + y * y + z * z; }  // vec3.rs:74-76
  double length() const { return std::sqrt(length_squared()); }
};
inline Vec3 operator+(Vec3 a, Vec3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline Vec3 operator-(Vec3 a, Vec3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline Vec3 operator-(Vec3 a) { return {-a.x, -a.y, -a.z}; }
inline Vec3 operator*(Vec3 a, double t) { return {a.x * t, a.y * t, a.z * t}; }
inline Vec3 operator*(double t, Vec3 a) { return a * t; }
inline Vec3 operator*(Vec3 a, Vec3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
inline Vec3 operator/(Vec3 a, double t) { return {a.x / t, a.y / t, a.z / t}; }
inline double dot(Vec3 u, Vec3 v) { return u.x * v.x + u.y * v.y + u.z * v.z; }  // vec3.rs:167
inline Vec3 cross(Vec3 u, Vec3 v) {                                                 // vec3.rs:171-177
  return {u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x};
}
inline Vec3 unit_vector(Vec3 v) { return v / v.length(); }  // vec3.rs:179-181

struct Interval {  // interval.rs:14-57
  double min = INFINITY, max = -INFINITY;
  double size() const { return max - min; }
  Interval expand(double delta) const { return {min - delta / 2., max + delta / 2.}; }
  static Interval hull(const Interval& a, const Interval& b) {
    return {std::fmin(a.min, b.min), std::fmax(a.max, b.max)};
  }
};

struct Aabb {  // object.rs:286-412
  Interval x, y, z;
  const Interval& axis(int n) const { return n == 0 ? x : (n == 1 ? y : z); }
  static Aabb from_points(Vec3 a, Vec3 b) {
    return {{std::fmin(a.x, b.x), std::fmax(a.x, b.x)},
            {std::fmin(a.y, b.y), std::fmax(a.y, b.y)},
            {std::fmin(a.z, b.z), std::fmax(a.z, b.z)}};
  }
  static Aabb from_boxes(const Aabb& a, const Aabb& b) {
    return {Interval::hull(a.x, b.x), Interval::hull(a.y, b.y), Interval::hull(a.z, b.z)};
  }
  Aabb pad() const {  // object.rs:372-391
    const double delta = 0.0001;
    return {x.size() >= delta ? x : x.expand(delta), y.size() >= delta ? y : y.expand(delta),
            z.size() >= delta ? z : z.expand(delta)};
  }
  Aabb operator+(Vec3 o) const {  // object.rs:394-412
    return {{x.min + o.x, x.max + o.x}, {y.min + o.y, y.max + o.y}, {z.min + o.z, z.max + o.z}};
  }
};

// Scene-build RNG (replaces rand::thread_rng in construction code).
// splitmix64; f64 uniforms carry 53 bits like rand's Standard distribution.
class SceneRng {
 public:
  explicit SceneRng(uint64_t seed) : s_(seed) {}
  uint64_t next_u64() {
    uint64_t z = (s_ += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  double random_double() { return (double)(next_u64() >> 11) * 0x1.0p-53; }
  double random_range(double a, double b) { return a + (b - a) * random_double(); }
  int64_t random_int(int64_t a, int64_t b) {  // inclusive, like gen_range(a..=b)
    uint64_t span = (uint64_t)(b - a) + 1u;
    return a + (int64_t)(((unsigned __int128)next_u64() * span) >> 64);
  }
  Vec3 random_vec3_range(double a, double b) {  // vec3.rs:197-203 (x, y, z draw order)
    double x = random_range(a, b), y = random_range(a, b), z = random_range(a, b);
    return {x, y, z};
  }

 private:
  uint64_t s_;
};

struct Perlin {  // perlin.rs:7-28
  Vec3 ranvec[RT_PERLIN_POINTS];
  int32_t perm_x[RT_PERLIN_POINTS], perm_y[RT_PERLIN_POINTS], perm_z[RT_PERLIN_POINTS];
  explicit Perlin(SceneRng& rng);
};

struct Texture {
  int kind = RT_TEX_SOLID;
  Vec3 color;                                 // SolidColor
  double inv_scale = 1;                       // CheckerTexture
  std::shared_ptr<Texture> even, odd;         //
  int32_t width = 0, height = 0;              // ImageTexture (RtImage)
  std::vector<uint8_t> rgb8;                  //
  double scale = 1;                           // NoiseTexture
  std::shared_ptr<Perlin> noise;              //
};
using TexturePtr = std::shared_ptr<Texture>;

struct Material {
  int kind = RT_MAT_LAMBERTIAN;
  TexturePtr tex;  // Lambertian albedo, DiffuseLight emit, Isotropic albedo
  Vec3 albedo;     // Metal
  double fuzz = 0; // Metal
  double ir = 1;   // Dielectric
  Vec3 tint{1, 1, 1};
};
using MaterialPtr = std::shared_ptr<Material>;

struct Object;
using ObjectPtr = std::shared_ptr<Object>;

struct Object {
  int tag = RT_OBJ_LIST;
  Aabb bbox;
  MaterialPtr mat;                       // Sphere, Quad, Volume (phase function)
  // Sphere (object.rs:73-105)
  Vec3 center, center_vec;
  bool moving = false;
  double radius = 0;
  // Quad (object.rs:414-446)
  Vec3 q, u, v, normal, w;
  double d = 0, area = 0;
  // HittableList (hittable.rs:55-80)
  std::vector<ObjectPtr> objects;
  // BvhNode (hittable.rs:135-187)
  ObjectPtr left, right;
  // Translate / RotateY (transform.rs) and ConstantMedium boundary (constant_medium.rs)
  ObjectPtr child;
  Vec3 offset;
  double sin_theta = 0, cos_theta = 1;
  double neg_inv_density = 0;
};

// ---- constructors (reference names) --------------------------------------------------------
TexturePtr SolidColor(Vec3 c);
TexturePtr CheckerTexture(double scale, TexturePtr even, TexturePtr odd);
TexturePtr NoiseTexture(double scale, SceneRng& rng);
TexturePtr ImageTexture(int32_t w, int32_t h, const uint8_t* rgb8);

MaterialPtr Lambertian(TexturePtr albedo);
MaterialPtr Metal(Vec3 albedo, double f);
MaterialPtr Dielectric(double ir, Vec3 tint);
MaterialPtr DiffuseLight(TexturePtr emit);
MaterialPtr Isotropic(TexturePtr albedo);

ObjectPtr Sphere(Vec3 center, double radius, MaterialPtr mat);
ObjectPtr SphereMoving(Vec3 c1, Vec3 c2, double radius, MaterialPtr mat);
ObjectPtr Quad(Vec3 q, Vec3 u, Vec3 v, MaterialPtr mat);
ObjectPtr HittableList();
void list_add(const ObjectPtr& list, ObjectPtr obj);
ObjectPtr create_bvh(const ObjectPtr& list, SceneRng& rng);  // returns a new list [BvhNode]
ObjectPtr make_box(Vec3 a, Vec3 b, MaterialPtr mat);
ObjectPtr Translate(ObjectPtr obj, Vec3 offset);
ObjectPtr RotateY(ObjectPtr obj, double angle_deg);
ObjectPtr ConstantMedium(ObjectPtr boundary, double density, TexturePtr albedo);

// ---- camera (render.rs:38-133) -------------------------------------------------------------
int nearest_square(int i);
rt_camera camera_new(double aspect_ratio, int image_width, int samples_per_pixel, int max_depth,
                     double vfov, Vec3 lookfrom, Vec3 lookat, Vec3 vup, double defocus_angle,
                     double focus_dist, Vec3 background);

// ---- serialisation into the rt_scene_blob slot format -------------------------------------
std::vector<uint64_t> serialize(const ObjectPtr& world, const ObjectPtr& lights /*nullable*/,
                                std::vector<uint8_t>* texels_out);

// ---- presets: main.rs scene functions -----------------------------------------------------
struct Preset {
  ObjectPtr world, lights;  // lights == nullptr  <=>  render_par (empty light list)
  rt_camera cam;
};
bool preset(const std::string& name, const std::string& variant, SceneRng& rng, int width,
            int spp, int depth, double aspect, Preset* out, std::string* err);

}  // namespace rt
