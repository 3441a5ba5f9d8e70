// scene.cpp — host scene construction, BVH build, camera, blob serialisation, main.rs presets.
// Each function restates the reference constructor cited beside it (f64, same operation order).
#include "scene.hpp"

#include <algorithm>
#include <cstring>
#include <map>

namespace rt {

static const double PI = 3.14159265358979323846;

// Rust f64::to_radians: self * (PI / 180.0)
static double to_radians(double deg) { return deg * (PI / 180.0); }

// f64::total_cmp as a strict-weak "less" (hittable.rs:189-200 uses total_cmp).
static bool total_less(double a, double b) {
  int64_t ia, ib;
  std::memcpy(&ia, &a, 8);
  std::memcpy(&ib, &b, 8);
  ia ^= (int64_t)(((uint64_t)(ia >> 63)) >> 1);
  ib ^= (int64_t)(((uint64_t)(ib >> 63)) >> 1);
  return ia < ib;
}

// ---------------------------------------------------------------- Perlin (perlin.rs:15-28, 97-117)
static void generate_perm(SceneRng& rng, int32_t* p) {
  for (int i = 0; i < RT_PERLIN_POINTS; ++i) p[i] = i;
  for (int i = RT_PERLIN_POINTS - 1; i >= 0; --i) {  // permute: (0..n).rev()
    int target = (int)rng.random_int(0, i);
    std::swap(p[i], p[target]);
  }
}

Perlin::Perlin(SceneRng& rng) {
  for (int i = 0; i < RT_PERLIN_POINTS; ++i) ranvec[i] = unit_vector(rng.random_vec3_range(-1., 1.));
  generate_perm(rng, perm_x);
  generate_perm(rng, perm_y);
  generate_perm(rng, perm_z);
}

// ---------------------------------------------------------------- textures (texture.rs)
TexturePtr SolidColor(Vec3 c) {
  auto t = std::make_shared<Texture>();
  t->kind = RT_TEX_SOLID;
  t->color = c;
  return t;
}
TexturePtr CheckerTexture(double scale, TexturePtr even, TexturePtr odd) {  // texture.rs:55-69
  auto t = std::make_shared<Texture>();
  t->kind = RT_TEX_CHECKER;
  t->inv_scale = 1. / scale;
  t->even = std::move(even);
  t->odd = std::move(odd);
  return t;
}
TexturePtr NoiseTexture(double scale, SceneRng& rng) {  // texture.rs:116-121
  auto t = std::make_shared<Texture>();
  t->kind = RT_TEX_NOISE;
  t->noise = std::make_shared<Perlin>(rng);
  t->scale = scale;
  return t;
}
TexturePtr ImageTexture(int32_t w, int32_t h, const uint8_t* rgb8) {  // texture.rs:89-93
  auto t = std::make_shared<Texture>();
  t->kind = RT_TEX_IMAGE;
  if (w > 0 && h > 0 && rgb8) {
    t->width = w;
    t->height = h;
    t->rgb8.assign(rgb8, rgb8 + (size_t)w * h * 3);
  }
  return t;
}

// ---------------------------------------------------------------- materials (material.rs)
static MaterialPtr mat(int kind) {
  auto m = std::make_shared<Material>();
  m->kind = kind;
  return m;
}
MaterialPtr Lambertian(TexturePtr albedo) {
  auto m = mat(RT_MAT_LAMBERTIAN);
  m->tex = std::move(albedo);
  return m;
}
MaterialPtr Metal(Vec3 albedo, double f) {  // material.rs:118-121: fuzz clamped to <= 1
  auto m = mat(RT_MAT_METAL);
  m->albedo = albedo;
  m->fuzz = f < 1. ? f : 1.;
  return m;
}
MaterialPtr Dielectric(double ir, Vec3 tint) {
  auto m = mat(RT_MAT_DIELECTRIC);
  m->ir = ir;
  m->tint = tint;
  return m;
}
MaterialPtr DiffuseLight(TexturePtr emit) {
  auto m = mat(RT_MAT_DIFFUSE_LIGHT);
  m->tex = std::move(emit);
  return m;
}
MaterialPtr Isotropic(TexturePtr albedo) {
  auto m = mat(RT_MAT_ISOTROPIC);
  m->tex = std::move(albedo);
  return m;
}

// ---------------------------------------------------------------- objects
ObjectPtr Sphere(Vec3 center, double radius, MaterialPtr m) {  // object.rs:83-92
  auto o = std::make_shared<Object>();
  o->tag = RT_OBJ_SPHERE;
  Vec3 rvec(radius, radius, radius);
  o->center = center;
  o->radius = radius;
  o->mat = std::move(m);
  o->moving = false;
  o->bbox = Aabb::from_points(center - rvec, center + rvec);
  return o;
}
ObjectPtr SphereMoving(Vec3 c1, Vec3 c2, double radius, MaterialPtr m) {  // object.rs:94-105
  auto o = std::make_shared<Object>();
  o->tag = RT_OBJ_SPHERE;
  Vec3 rvec(radius, radius, radius);
  Aabb b1 = Aabb::from_points(c1 - rvec, c1 + rvec);
  Aabb b2 = Aabb::from_points(c2 - rvec, c2 + rvec);
  o->center = c1;
  o->radius = radius;
  o->mat = std::move(m);
  o->moving = true;
  o->center_vec = c2 - c1;
  o->bbox = Aabb::from_boxes(b1, b2);
  return o;
}
ObjectPtr Quad(Vec3 q, Vec3 u, Vec3 v, MaterialPtr m) {  // object.rs:427-446
  auto o = std::make_shared<Object>();
  o->tag = RT_OBJ_QUAD;
  o->bbox = Aabb::from_points(q, q + u + v).pad();
  Vec3 n = cross(u, v);
  o->normal = unit_vector(n);
  o->w = n / dot(n, n);
  o->q = q;
  o->u = u;
  o->v = v;
  o->mat = std::move(m);
  o->d = dot(o->normal, q);
  o->area = n.length();
  return o;
}
ObjectPtr HittableList() {  // hittable.rs:61-66
  auto o = std::make_shared<Object>();
  o->tag = RT_OBJ_LIST;
  o->bbox = Aabb{};  // Aabb::empty()
  return o;
}
void list_add(const ObjectPtr& list, ObjectPtr obj) {  // hittable.rs:74-80
  list->bbox = Aabb::from_boxes(list->bbox, obj->bbox);
  list->objects.push_back(std::move(obj));
}

static bool box_less(const ObjectPtr& a, const ObjectPtr& b, int axis) {
  return total_less(a->bbox.axis(axis).min, b->bbox.axis(axis).min);
}

// BvhNode::new (hittable.rs:147-187): random axis per node (drawn before the span test),
// span 1 duplicates the object, span 2 orders the pair, else stable sort + median split.
static ObjectPtr bvh_node(std::vector<ObjectPtr>& objects, size_t start, size_t end,
                          SceneRng& rng) {
  int axis = (int)rng.random_int(0, 2);
  size_t span = end - start;
  ObjectPtr left, right;
  if (span == 1) {
    left = right = objects[start];
  } else if (span == 2) {
    if (box_less(objects[start], objects[start + 1], axis)) {
      left = objects[start];
      right = objects[start + 1];
    } else {
      left = objects[start + 1];
      right = objects[start];
    }
  } else {
    std::stable_sort(objects.begin() + start, objects.begin() + end,
                     [axis](const ObjectPtr& a, const ObjectPtr& b) { return box_less(a, b, axis); });
    size_t mid = start + span / 2;
    left = bvh_node(objects, start, mid, rng);
    right = bvh_node(objects, mid, end, rng);
  }
  auto o = std::make_shared<Object>();
  o->tag = RT_OBJ_BVH;
  o->bbox = Aabb::from_boxes(left->bbox, right->bbox);
  o->left = std::move(left);
  o->right = std::move(right);
  return o;
}

ObjectPtr create_bvh(const ObjectPtr& list, SceneRng& rng) {  // hittable.rs:82-84, 142-145
  ObjectPtr node = bvh_node(list->objects, 0, list->objects.size(), rng);
  ObjectPtr out = HittableList();
  list_add(out, node);
  return out;
}

ObjectPtr make_box(Vec3 a, Vec3 b, MaterialPtr m) {  // object.rs:509-560
  ObjectPtr sides = HittableList();
  Vec3 mn(std::fmin(a.x, b.x), std::fmin(a.y, b.y), std::fmin(a.z, b.z));
  Vec3 mx(std::fmax(a.x, b.x), std::fmax(a.y, b.y), std::fmax(a.z, b.z));
  Vec3 dx(mx.x - mn.x, 0., 0.), dy(0., mx.y - mn.y, 0.), dz(0., 0., mx.z - mn.z);
  list_add(sides, Quad(Vec3(mn.x, mn.y, mx.z), dx, dy, m));   // front
  list_add(sides, Quad(Vec3(mx.x, mn.y, mx.z), -dz, dy, m));  // right
  list_add(sides, Quad(Vec3(mx.x, mn.y, mn.z), -dx, dy, m));  // back
  list_add(sides, Quad(Vec3(mn.x, mn.y, mn.z), dz, dy, m));   // left
  list_add(sides, Quad(Vec3(mn.x, mx.y, mx.z), dx, -dz, m));  // top
  list_add(sides, Quad(Vec3(mn.x, mn.y, mn.z), dx, dz, m));   // bottom
  return sides;
}

ObjectPtr Translate(ObjectPtr obj, Vec3 offset) {  // transform.rs:43-54
  auto o = std::make_shared<Object>();
  o->tag = RT_OBJ_TRANSLATE;
  o->bbox = obj->bbox + offset;
  o->child = std::move(obj);
  o->offset = offset;
  return o;
}

ObjectPtr RotateY(ObjectPtr obj, double angle) {  // transform.rs:143-186
  auto o = std::make_shared<Object>();
  o->tag = RT_OBJ_ROTATE_Y;
  double radians = to_radians(angle);
  double s = std::sin(radians), c = std::cos(radians);
  const Aabb& bb = obj->bbox;
  Vec3 mn(INFINITY, INFINITY, INFINITY), mx(-INFINITY, -INFINITY, -INFINITY);
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j)
      for (int k = 0; k < 2; ++k) {
        double x = i * bb.x.max + (1. - i) * bb.x.min;
        double y = j * bb.y.max + (1. - j) * bb.y.min;
        double z = k * bb.z.max + (1. - k) * bb.z.min;
        double newx = c * x + s * z;
        double newz = -s * x + c * z;
        Vec3 tester(newx, y, newz);
        for (int a = 0; a < 3; ++a) {
          mn.set(a, std::fmin(mn.dim(a), tester.dim(a)));
          mx.set(a, std::fmax(mx.dim(a), tester.dim(a)));
        }
      }
  o->bbox = Aabb::from_points(mn, mx);
  o->child = std::move(obj);
  o->sin_theta = s;
  o->cos_theta = c;
  return o;
}

ObjectPtr ConstantMedium(ObjectPtr boundary, double density, TexturePtr albedo) {
  auto o = std::make_shared<Object>();  // constant_medium.rs:21-35
  o->tag = RT_OBJ_VOLUME;
  o->bbox = boundary->bbox;
  o->child = std::move(boundary);
  o->neg_inv_density = -1. / density;
  o->mat = Isotropic(std::move(albedo));
  return o;
}

// ---------------------------------------------------------------- camera (render.rs:38-133)
int nearest_square(int i) {
  double d = (double)i;
  int r = (int)std::sqrt(d);
  return r * r;
}

static void put3(double* dst, Vec3 v) {
  dst[0] = v.x;
  dst[1] = v.y;
  dst[2] = v.z;
}

rt_camera camera_new(double aspect_ratio, int image_width, int samples_per_pixel, int max_depth,
                     double vfov, Vec3 lookfrom, Vec3 lookat, Vec3 vup, double defocus_angle,
                     double focus_dist, Vec3 background) {
  int image_height = (int)((double)image_width / aspect_ratio);
  if (image_height < 1) image_height = 1;
  Vec3 center = lookfrom;
  double theta = to_radians(vfov);
  double h = std::tan(theta / 2.);
  if (focus_dist <= 0.) focus_dist = 1.;
  double viewport_height = 2. * h * focus_dist;
  double viewport_width = viewport_height * (double)image_width / (double)image_height;
  Vec3 w = unit_vector(lookfrom - lookat);
  Vec3 u = unit_vector(cross(vup, w));
  Vec3 v = cross(w, u);
  Vec3 viewport_u = viewport_width * u;
  Vec3 viewport_v = viewport_height * -v;
  Vec3 pixel_delta_u = viewport_u / (double)image_width;
  Vec3 pixel_delta_v = viewport_v / (double)image_height;
  Vec3 viewport_upper_left = center - (focus_dist * w) - viewport_u / 2. - viewport_v / 2.;
  Vec3 pixel00_loc = viewport_upper_left + 0.5 * (pixel_delta_u + pixel_delta_v);
  double defocus_radius = focus_dist * std::tan(to_radians(defocus_angle / 2.));
  int spp = nearest_square(samples_per_pixel);
  double sqrt_spp = std::sqrt((double)spp);

  rt_camera c;
  std::memset(&c, 0, sizeof(c));
  c.image_width = image_width;
  c.image_height = image_height;
  c.samples_per_pixel = spp;
  c.sqrt_spp = (int)sqrt_spp;
  c.max_depth = max_depth;
  c.recip_sqrt_spp = 1. / sqrt_spp;
  put3(c.center, center);
  put3(c.pixel00_loc, pixel00_loc);
  put3(c.pixel_delta_u, pixel_delta_u);
  put3(c.pixel_delta_v, pixel_delta_v);
  c.defocus_angle = defocus_angle;
  put3(c.defocus_disk_u, u * defocus_radius);
  put3(c.defocus_disk_v, v * defocus_radius);
  put3(c.background, background);
  return c;
}

// ---------------------------------------------------------------- serialisation
namespace {
struct Serializer {
  std::vector<uint64_t> out;
  std::vector<uint8_t>* texels;
  std::map<const Texture*, int64_t> tex_ids;
  std::map<const Material*, int64_t> mat_ids;
  std::map<const Perlin*, int64_t> perlin_ids;
  std::vector<const Texture*> texs;
  std::vector<const Material*> mats;
  std::vector<const Perlin*> perlins;

  void i(int64_t v) { out.push_back((uint64_t)v); }
  void f(double v) {
    uint64_t b;
    std::memcpy(&b, &v, 8);
    out.push_back(b);
  }
  void v3(Vec3 v) { f(v.x), f(v.y), f(v.z); }
  void bbox(const Aabb& b) {
    f(b.x.min), f(b.x.max), f(b.y.min), f(b.y.max), f(b.z.min), f(b.z.max);
  }

  int64_t tex_id(const TexturePtr& t) {
    auto it = tex_ids.find(t.get());
    if (it != tex_ids.end()) return it->second;
    if (t->kind == RT_TEX_CHECKER) {  // children first so ids are stable
      tex_id(t->even);
      tex_id(t->odd);
    }
    if (t->kind == RT_TEX_NOISE && !perlin_ids.count(t->noise.get())) {
      perlin_ids[t->noise.get()] = (int64_t)perlins.size();
      perlins.push_back(t->noise.get());
    }
    int64_t id = (int64_t)texs.size();
    tex_ids[t.get()] = id;
    texs.push_back(t.get());
    return id;
  }
  int64_t mat_id(const MaterialPtr& m) {
    auto it = mat_ids.find(m.get());
    if (it != mat_ids.end()) return it->second;
    if (m->tex) tex_id(m->tex);
    int64_t id = (int64_t)mats.size();
    mat_ids[m.get()] = id;
    mats.push_back(m.get());
    return id;
  }

  void obj(const ObjectPtr& o) {
    switch (o->tag) {
      case RT_OBJ_LIST:
        i(RT_OBJ_LIST), i((int64_t)o->objects.size()), bbox(o->bbox);
        for (auto& c : o->objects) obj(c);
        break;
      case RT_OBJ_BVH:
        i(RT_OBJ_BVH), bbox(o->bbox);
        obj(o->left);
        obj(o->right);
        break;
      case RT_OBJ_SPHERE:
        i(RT_OBJ_SPHERE), i(mat_id(o->mat)), i(o->moving ? 1 : 0), v3(o->center), f(o->radius),
            v3(o->center_vec), bbox(o->bbox);
        break;
      case RT_OBJ_QUAD:
        i(RT_OBJ_QUAD), i(mat_id(o->mat)), v3(o->q), v3(o->u), v3(o->v), v3(o->normal), v3(o->w),
            f(o->d), f(o->area), bbox(o->bbox);
        break;
      case RT_OBJ_TRANSLATE:
        i(RT_OBJ_TRANSLATE), v3(o->offset), bbox(o->bbox);
        obj(o->child);
        break;
      case RT_OBJ_ROTATE_Y:
        i(RT_OBJ_ROTATE_Y), f(o->sin_theta), f(o->cos_theta), bbox(o->bbox);
        obj(o->child);
        break;
      case RT_OBJ_VOLUME:
        i(RT_OBJ_VOLUME), i(mat_id(o->mat)), f(o->neg_inv_density), bbox(o->bbox);
        obj(o->child);
        break;
    }
  }
};
}  // namespace

std::vector<uint64_t> serialize(const ObjectPtr& world, const ObjectPtr& lights,
                                std::vector<uint8_t>* texels_out) {
  Serializer s;
  std::vector<uint8_t> texels;
  s.texels = &texels;
  s.out.assign(RT_BLOB_HEADER_SLOTS, 0);
  // Objects first (they register materials / textures), tables after.
  int64_t world_off = (int64_t)s.out.size();
  s.obj(world);
  int64_t lights_off = -1;
  if (lights) {
    lights_off = (int64_t)s.out.size();
    s.obj(lights);
  }
  int64_t tex_off = (int64_t)s.out.size();
  for (const Texture* t : s.texs) {
    size_t base = s.out.size();
    s.i(t->kind);
    switch (t->kind) {
      case RT_TEX_SOLID: s.v3(t->color); break;
      case RT_TEX_CHECKER:
        s.f(t->inv_scale), s.i(s.tex_ids.at(t->even.get())), s.i(s.tex_ids.at(t->odd.get()));
        break;
      case RT_TEX_IMAGE:
        s.i(t->width), s.i(t->height), s.i((int64_t)texels.size());
        texels.insert(texels.end(), t->rgb8.begin(), t->rgb8.end());
        break;
      case RT_TEX_NOISE: s.f(t->scale), s.i(s.perlin_ids.at(t->noise.get())); break;
    }
    while (s.out.size() < base + RT_TEX_SLOTS) s.i(0);
  }
  int64_t mat_off = (int64_t)s.out.size();
  for (const Material* m : s.mats) {
    size_t base = s.out.size();
    s.i(m->kind);
    switch (m->kind) {
      case RT_MAT_LAMBERTIAN:
      case RT_MAT_DIFFUSE_LIGHT:
      case RT_MAT_ISOTROPIC: s.i(s.tex_ids.at(m->tex.get())); break;
      case RT_MAT_METAL: s.v3(m->albedo), s.f(m->fuzz); break;
      case RT_MAT_DIELECTRIC: s.f(m->ir), s.v3(m->tint); break;
    }
    while (s.out.size() < base + RT_MAT_SLOTS) s.i(0);
  }
  int64_t perlin_off = (int64_t)s.out.size();
  for (const Perlin* p : s.perlins) {
    for (int k = 0; k < RT_PERLIN_POINTS; ++k) s.v3(p->ranvec[k]);
    for (int k = 0; k < RT_PERLIN_POINTS; ++k) s.i(p->perm_x[k]);
    for (int k = 0; k < RT_PERLIN_POINTS; ++k) s.i(p->perm_y[k]);
    for (int k = 0; k < RT_PERLIN_POINTS; ++k) s.i(p->perm_z[k]);
  }
  std::vector<uint64_t>& o = s.out;
  o[0] = RT_BLOB_MAGIC;
  o[1] = RT_BLOB_VERSION;
  o[2] = o.size();
  o[3] = s.texs.size();
  o[4] = (uint64_t)tex_off;
  o[5] = s.mats.size();
  o[6] = (uint64_t)mat_off;
  o[7] = s.perlins.size();
  o[8] = (uint64_t)perlin_off;
  o[9] = (uint64_t)world_off;
  o[10] = (uint64_t)lights_off;
  o[11] = texels.size();
  if (texels_out) *texels_out = std::move(texels);
  return std::move(s.out);
}

}  // namespace rt
