// presets.cpp — the reference's scene scripts (main.rs) restated on the C++ builder.
// Each preset keeps the reference geometry, materials and Camera::new literals; width / spp /
// depth / aspect can be overridden for the BASELINE configs. Scene randomness is
// drawn from the seeded SceneRng in the same order as the reference draws it.
#include "scene.hpp"

namespace rt {

namespace {

struct Overrides {
  int width, spp, depth;
  double aspect;
  int w(int ref) const { return width > 0 ? width : ref; }
  int s(int ref) const { return spp > 0 ? spp : ref; }
  int d(int ref) const { return depth > 0 ? depth : ref; }
  double a(double ref) const { return aspect > 0 ? aspect : ref; }
};

const Vec3 kUp(0., 1., 0.);

// cornell_box main.rs:417-512 (the scene behind final_images/book3.png). The "mixed_pdf" variant
// re-enables box2 (main.rs:473-480), drops the glass sphere and lights only the quad: the
// revision behind final_images/mixed_pdf.png.
void cornell_box(bool mixed_pdf, const Overrides& ov, Preset* out) {
  ObjectPtr world = HittableList();
  auto red = Lambertian(SolidColor({0.65, 0.05, 0.05}));
  auto white = Lambertian(SolidColor({0.73, 0.73, 0.73}));
  auto green = Lambertian(SolidColor({0.12, 0.45, 0.15}));
  auto light = DiffuseLight(SolidColor({15., 15., 15.}));
  list_add(world, Quad({555., 0., 0.}, {0., 555., 0.}, {0., 0., 555.}, green));
  list_add(world, Quad({0., 0., 0.}, {0., 555., 0.}, {0., 0., 555.}, red));
  list_add(world, Quad({343., 554., 332.}, {-130., 0., 0.}, {0., 0., -105.}, light));
  list_add(world, Quad({0., 0., 0.}, {555., 0., 0.}, {0., 0., 555.}, white));
  list_add(world, Quad({555., 555., 555.}, {-555., 0., 0.}, {0., 0., -555.}, white));
  list_add(world, Quad({0., 0., 555.}, {555., 0., 0.}, {0., 555., 0.}, white));
  ObjectPtr box1 = make_box({0., 0., 0.}, {165., 330., 165.}, white);
  box1 = RotateY(box1, 15.);
  box1 = Translate(box1, {265., 0., 295.});
  list_add(world, box1);
  ObjectPtr box2 = make_box({0., 0., 0.}, {165., 165., 165.}, white);
  box2 = RotateY(box2, -18.);
  box2 = Translate(box2, {130., 0., 65.});
  ObjectPtr lights = HittableList();
  list_add(lights, Quad({343., 554., 332.}, {-130., 0., 0.}, {0., 0., -105.}, light));
  if (mixed_pdf) {
    list_add(world, box2);
  } else {
    auto glass = Dielectric(1.5, {1., 1., 1.});
    list_add(world, Sphere({190., 90., 190.}, 90., glass));
    list_add(lights, Sphere({190., 90., 190.}, 90., light));
  }
  out->world = world;
  out->lights = lights;
  out->cam = camera_new(ov.a(1.), ov.w(600), ov.s(1000), ov.d(50), 40., {278., 278., -800.},
                        {278., 278., 0.}, kUp, 0., 0., {0., 0., 0.});
}

// cornell_smoke main.rs:514-601 (render_par: empty light list).
void cornell_smoke(const Overrides& ov, Preset* out) {
  ObjectPtr world = HittableList();
  auto red = Lambertian(SolidColor({0.65, 0.05, 0.05}));
  auto white = Lambertian(SolidColor({0.73, 0.73, 0.73}));
  auto green = Lambertian(SolidColor({0.12, 0.45, 0.15}));
  auto light = DiffuseLight(SolidColor({7., 7., 7.}));
  list_add(world, Quad({555., 0., 0.}, {0., 555., 0.}, {0., 0., 555.}, green));
  list_add(world, Quad({0., 0., 0.}, {0., 555., 0.}, {0., 0., 555.}, red));
  list_add(world, Quad({113., 554., 127.}, {330., 0., 0.}, {0., 0., 305.}, light));
  list_add(world, Quad({0., 0., 0.}, {555., 0., 0.}, {0., 0., 555.}, white));
  list_add(world, Quad({555., 555., 555.}, {-555., 0., 0.}, {0., 0., -555.}, white));
  list_add(world, Quad({0., 0., 555.}, {555., 0., 0.}, {0., 555., 0.}, white));
  ObjectPtr box1 = make_box({0., 0., 0.}, {165., 330., 165.}, white);
  box1 = Translate(RotateY(box1, 15.), {265., 0., 295.});
  ObjectPtr box2 = make_box({0., 0., 0.}, {165., 165., 165.}, white);
  box2 = Translate(RotateY(box2, -18.), {130., 0., 65.});
  list_add(world, ConstantMedium(box1, 0.01, SolidColor({0., 0., 0.})));
  list_add(world, ConstantMedium(box2, 0.01, SolidColor({1., 1., 1.})));
  out->world = world;
  out->lights = nullptr;
  out->cam = camera_new(ov.a(1.), ov.w(600), ov.s(100), ov.d(10), 40., {278., 278., -800.},
                        {278., 278., 0.}, kUp, 0., 0., {0., 0., 0.});
}

// final_scene main.rs:603-712 (book2). earthmap.jpg is absent from the reference repo, so the
// ImageTexture is the empty image and yields (0,1,1) (texture.rs:96-98).
void final_scene(SceneRng& rng, const Overrides& ov, Preset* out) {
  ObjectPtr boxes1 = HittableList();
  auto ground = Lambertian(SolidColor({0.48, 0.83, 0.53}));
  const int boxes_per_side = 20;
  for (int i = 0; i < boxes_per_side; ++i)
    for (int j = 0; j < boxes_per_side; ++j) {
      double w = 100.;
      double x0 = -1000. + i * w, z0 = -1000. + j * w, y0 = 0.;
      double x1 = x0 + w;
      double y1 = rng.random_range(1., 101.);
      double z1 = z0 + w;
      list_add(boxes1, make_box({x0, y0, z0}, {x1, y1, z1}, ground));
    }
  ObjectPtr world = HittableList();
  list_add(world, create_bvh(boxes1, rng));
  auto light = DiffuseLight(SolidColor({7., 7., 7.}));
  list_add(world, Quad({123., 554., 147.}, {300., 0., 0.}, {0., 0., 265.}, light));
  Vec3 center1(400., 400., 200.);
  Vec3 center2 = center1 + Vec3(30., 0., 0.);
  list_add(world, SphereMoving(center1, center2, 50., Lambertian(SolidColor({0.7, 0.3, 0.1}))));
  list_add(world, Sphere({260., 150., 45.}, 50., Dielectric(1.5, {1., 1., 1.})));
  list_add(world, Sphere({0., 150., 145.}, 50., Metal({0.8, 0.8, 0.9}, 1.0)));
  ObjectPtr boundary = Sphere({360., 150., 145.}, 70., Dielectric(1.5, {1., 1., 1.}));
  list_add(world, boundary);
  list_add(world, ConstantMedium(boundary, 0.2, SolidColor({0.2, 0.4, 0.9})));
  boundary = Sphere({0., 0., 0.}, 5000., Dielectric(1.5, {1., 1., 1.}));
  list_add(world, ConstantMedium(boundary, 0.0001, SolidColor({1., 1., 1.})));
  auto emat = Lambertian(ImageTexture(0, 0, nullptr));
  list_add(world, Sphere({400., 200., 400.}, 100., emat));
  auto pertext = NoiseTexture(0.1, rng);
  list_add(world, Sphere({220., 280., 300.}, 80., Lambertian(pertext)));
  ObjectPtr boxes2 = HittableList();
  auto white = Lambertian(SolidColor({0.73, 0.73, 0.73}));
  for (int k = 0; k < 1000; ++k) list_add(boxes2, Sphere(rng.random_vec3_range(0., 165.), 10., white));
  list_add(world, Translate(RotateY(create_bvh(boxes2, rng), 15.), {-100., 270., 395.}));
  out->world = world;
  out->lights = nullptr;
  out->cam = camera_new(ov.a(1.), ov.w(800), ov.s(10000), ov.d(40), 40., {478., 278., -600.},
                        {278., 278., 0.}, kUp, 0., 0., {0., 0., 0.});
}

// quads main.rs:315-372
void quads(const Overrides& ov, Preset* out) {
  ObjectPtr world = HittableList();
  list_add(world, Quad({-3., -2., 5.}, {0., 0., -4.}, {0., 4., 0.}, Lambertian(SolidColor({1., 0.2, 0.2}))));
  list_add(world, Quad({-2., -2., 0.}, {4., 0., 0.}, {0., 4., 0.}, Lambertian(SolidColor({0.2, 1.0, 0.2}))));
  list_add(world, Quad({3., -2., 1.}, {0., 0., 4.}, {0., 4., 0.}, Lambertian(SolidColor({0.2, 0.2, 1.0}))));
  list_add(world, Quad({-2., 3., 1.}, {4., 0., 0.}, {0., 0., 4.}, Lambertian(SolidColor({1.0, 0.5, 0.}))));
  list_add(world, Quad({-2., -3., 5.}, {4., 0., 0.}, {0., 0., -4.}, Lambertian(SolidColor({0.2, 0.8, 0.8}))));
  out->world = world;
  out->lights = nullptr;
  out->cam = camera_new(ov.a(1.), ov.w(400), ov.s(100), ov.d(50), 80., {0., 0., 9.}, {0., 0., 0.},
                        kUp, 0., 0., {0.6, 0.7, 1.});
}

// simple_light main.rs:374-415
void simple_light(SceneRng& rng, const Overrides& ov, Preset* out) {
  ObjectPtr world = HittableList();
  auto pertex = NoiseTexture(4., rng);
  list_add(world, Sphere({0., -1000., 0.}, 1000., Lambertian(pertex)));
  list_add(world, Sphere({0., 2., 0.}, 2., Lambertian(pertex)));
  auto difflight = DiffuseLight(SolidColor({4., 4., 4.}));
  list_add(world, Quad({3., 1., -2.}, {2., 0., 0.}, {0., 2., 0.}, difflight));
  list_add(world, Sphere({0., 7., 0.}, 2., difflight));
  out->world = world;
  out->lights = nullptr;
  out->cam = camera_new(ov.a(16. / 9.), ov.w(400), ov.s(400), ov.d(50), 20., {26., 3., 6.},
                        {0., 2., 0.}, kUp, 0., 0., {0., 0., 0.});
}

// two_spheres main.rs:212-250
void two_spheres(const Overrides& ov, Preset* out) {
  ObjectPtr world = HittableList();
  auto checker = CheckerTexture(0.3, SolidColor({0.2, 0.3, 0.1}), SolidColor({0.9, 0.9, 0.9}));
  list_add(world, Sphere({0., -10., 0.}, 10., Lambertian(checker)));
  list_add(world, Sphere({0., 10., 0.}, 10., Lambertian(checker)));
  out->world = world;
  out->lights = nullptr;
  out->cam = camera_new(ov.a(16. / 9.), ov.w(400), ov.s(100), ov.d(50), 20., {13., 2., 3.},
                        {0., 0., 0.}, kUp, 0., 0., {0.7, 0.8, 1.});
}

// two_perlin_spheres main.rs:279-313
void two_perlin_spheres(SceneRng& rng, const Overrides& ov, Preset* out) {
  ObjectPtr world = HittableList();
  auto pertext = NoiseTexture(4., rng);
  list_add(world, Sphere({0., -1000., 0.}, 1000., Lambertian(pertext)));
  list_add(world, Sphere({0., 2., 0.}, 2., Lambertian(pertext)));
  out->world = world;
  out->lights = nullptr;
  out->cam = camera_new(ov.a(16. / 9.), ov.w(400), ov.s(100), ov.d(50), 20., {13., 2., 3.},
                        {0., 0., 0.}, kUp, 0., 0., {0.6, 0.7, 1.});
}

// earth main.rs:252-277 (earthmap.jpg absent -> empty image, App. A S3)
void earth(const Overrides& ov, Preset* out) {
  ObjectPtr world = HittableList();
  list_add(world, Sphere({0., 0., 0.}, 2., Lambertian(ImageTexture(0, 0, nullptr))));
  out->world = world;
  out->lights = nullptr;
  out->cam = camera_new(ov.a(16. / 9.), ov.w(1000), ov.s(1000), ov.d(50), 20., {13., 3., 2.},
                        {0., 0., 0.}, kUp, 0., 0., {0.7, 0.8, 1.});
}

// scene_three_spheres main.rs:92-133 (defocus blur, hollow glass with negative radius, BVH)
void three_spheres(SceneRng& rng, const Overrides& ov, Preset* out) {
  ObjectPtr world = HittableList();
  auto ground = Lambertian(SolidColor({0.8, 0.8, 0.0}));
  auto center = Lambertian(SolidColor({0.1, 0.2, 0.5}));
  auto left = Dielectric(1.5, {1.0, 0.9, 0.8});
  auto right = Metal({0.8, 0.6, 0.2}, 0.);
  list_add(world, Sphere({0., 0., -1.}, 0.5, center));
  list_add(world, Sphere({-1., 0., -1.}, 0.5, left));
  list_add(world, Sphere({-1., 0., -1.}, -0.4, left));
  list_add(world, Sphere({0., -100.5, -1.}, 100., ground));
  list_add(world, Sphere({1., 0., -1.}, 0.5, right));
  rt_camera cam = camera_new(ov.a(16. / 9.), ov.w(800), ov.s(1000), ov.d(50), 90., {0., 0., 0.},
                             {0., 0., -1.}, kUp, 2., 1., {0.7, 0.8, 1.});
  out->world = create_bvh(world, rng);
  out->lights = nullptr;
  out->cam = cam;
}

// scene_random_balls main.rs:135-210 (book-1 cover: checker ground, moving spheres, BVH, defocus)
void random_balls(SceneRng& rng, const Overrides& ov, Preset* out) {
  ObjectPtr world = HittableList();
  auto checker = CheckerTexture(0.32, SolidColor({0.2, 0.3, 0.1}), SolidColor({0.9, 0.9, 0.9}));
  list_add(world, Sphere({0., -2000., 0.}, 2000., Lambertian(checker)));
  auto rv3 = [&]() {
    double x = rng.random_double(), y = rng.random_double(), z = rng.random_double();
    return Vec3(x, y, z);
  };
  for (int a = -11; a < 11; ++a)
    for (int b = -11; b < 11; ++b) {
      double choose_mat = rng.random_double();
      double cx = a + 0.9 * rng.random_double();
      double cz = b + 0.9 * rng.random_double();
      Vec3 c(cx, 0.2, cz);
      Vec3 c2 = c + Vec3(0., rng.random_range(0., 0.5), 0.);
      if ((c - Vec3(4., 0.2, 0.)).length_squared() > 0.9 * 0.9) {
        if (choose_mat < 0.8) {
          Vec3 a1 = rv3();
          Vec3 a2 = rv3();
          list_add(world, SphereMoving(c, c2, 0.2, Lambertian(SolidColor(a1 * a2))));
        } else if (choose_mat < 0.95) {
          Vec3 albedo = rng.random_vec3_range(0.5, 1.);
          double fuzz = rng.random_range(0., 0.5);
          list_add(world, Sphere(c, 0.2, Metal(albedo, fuzz)));
        } else {
          double ir = rng.random_range(1.2, 1.6);
          list_add(world, Sphere(c, 0.2, Dielectric(ir, {1., 1., 1.})));
        }
      }
    }
  list_add(world, Sphere({0., 1., 0.}, 1.0, Dielectric(1.5, {1., 1., 1.})));
  list_add(world, Sphere({-4., 1., 0.}, 1.0, Lambertian(SolidColor({0.4, 0.2, 0.1}))));
  list_add(world, Sphere({4., 1., 0.}, 1.0, Metal({0.7, 0.6, 0.5}, 0.0)));
  rt_camera cam = camera_new(ov.a(16. / 9.), ov.w(500), ov.s(400), ov.d(50), 20., {13., 2., 3.},
                             {0., 0., 0.}, kUp, 0.6, 10., {0.7, 0.8, 1.});
  out->world = create_bvh(world, rng);
  out->lights = nullptr;
  out->cam = cam;
}

}  // namespace

bool preset(const std::string& name, const std::string& variant, SceneRng& rng, int width,
            int spp, int depth, double aspect, Preset* out, std::string* err) {
  Overrides ov{width, spp, depth, aspect};
  if (name == "cornell_box") {
    if (!variant.empty() && variant != "mixed_pdf") {
      *err = "unknown cornell_box variant: " + variant;
      return false;
    }
    cornell_box(variant == "mixed_pdf", ov, out);
  } else if (name == "cornell_smoke") {
    cornell_smoke(ov, out);
  } else if (name == "final_scene") {
    final_scene(rng, ov, out);
  } else if (name == "quads") {
    quads(ov, out);
  } else if (name == "simple_light") {
    simple_light(rng, ov, out);
  } else if (name == "two_spheres") {
    two_spheres(ov, out);
  } else if (name == "two_perlin_spheres") {
    two_perlin_spheres(rng, ov, out);
  } else if (name == "earth") {
    earth(ov, out);
  } else if (name == "three_spheres") {
    three_spheres(rng, ov, out);
  } else if (name == "random_balls") {
    random_balls(rng, ov, out);
  } else {
    *err = "unknown preset: " + name;
    return false;
  }
  return true;
}

}  // namespace rt
