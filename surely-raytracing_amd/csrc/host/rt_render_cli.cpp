// rt_render_cli — the host program: the reference's main() (main.rs:713-729) on this stack.
//
//   scene selector (main.rs:714-728) -> preset scene (C++ builder, rt_host.h)
//   -> rt_render (gfx950, rt_mi355x.h)    [render_par_lights, render.rs:144-216]
//   -> auto_expose / write_color -> P3 PPM [render.rs:151, 199-215; color.rs:8-33]
//
// Usage: rt_render_cli [--scene N|name] [--variant mixed_pdf] [--width W] [--spp S]
//                      [--depth D] [--aspect A] [--seed K] [--build-seed K] [--device N]
//                      [--reference-semantics] [--auto-exposure] [--out file.ppm]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../../include/rt_host.h"
#include "../../../include/rt_mi355x.h"

static const char* scene_name(int n) {  // main.rs:715-728 selector values
  switch (n) {
    case -1: return "three_spheres";
    case 1: return "random_balls";
    case 2: return "two_spheres";
    case 3: return "earth";
    case 4: return "two_perlin_spheres";
    case 5: return "quads";
    case 6: return "simple_light";
    case 7: return "cornell_box";
    case 8: return "cornell_smoke";
    case 9: return "final_scene";
    default: return "final_scene";  // `_` arm: final_scene(400, 250, 4)
  }
}

int main(int argc, char** argv) {
  std::string scene = "cornell_box", variant, out = "image.ppm";
  int width = 0, spp = 0, depth = 0, device = 0;
  double aspect = 0;
  uint64_t seed = 1, build_seed = 1;
  bool refsem = false, autoexp = false;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() -> const char* {
      if (i + 1 >= argc) {
        std::fprintf(stderr, "missing value for %s\n", a.c_str());
        std::exit(2);
      }
      return argv[++i];
    };
    if (a == "--scene") {
      std::string v = next();
      char* end = nullptr;
      long n = std::strtol(v.c_str(), &end, 10);
      if (end && *end == 0) {
        scene = scene_name((int)n);
        if (n != 9 && std::string(scene) == "final_scene") {  // `_` arm parameters
          if (!width) width = 400;
          if (!spp) spp = 250;
          if (!depth) depth = 4;
        }
      } else {
        scene = v;
      }
    } else if (a == "--variant") variant = next();
    else if (a == "--width") width = std::atoi(next());
    else if (a == "--spp") spp = std::atoi(next());
    else if (a == "--depth") depth = std::atoi(next());
    else if (a == "--aspect") aspect = std::atof(next());
    else if (a == "--seed") seed = std::strtoull(next(), nullptr, 10);
    else if (a == "--build-seed") build_seed = std::strtoull(next(), nullptr, 10);
    else if (a == "--device") device = std::atoi(next());
    else if (a == "--reference-semantics") refsem = true;
    else if (a == "--auto-exposure") autoexp = true;
    else if (a == "--out") out = next();
    else {
      std::fprintf(stderr, "unknown argument %s\n", a.c_str());
      return 2;
    }
  }
  rth_scene* s = rth_scene_new(build_seed);
  int32_t world = -1, lights = -1;
  rt_camera cam;
  if (rth_preset(s, scene.c_str(), variant.c_str(), width, spp, depth, aspect, &world, &lights,
                 &cam) != 0) {
    std::fprintf(stderr, "preset: %s\n", rth_last_error());
    return 1;
  }
  rt_scene_blob blob;
  if (rth_serialize(s, world, lights, &blob) != 0) {
    std::fprintf(stderr, "serialize: %s\n", rth_last_error());
    return 1;
  }
  std::fprintf(stderr, "Rendering %s %dx%d, %d spp (requested %d), depth %d on HIP device %d\n",
               scene.c_str(), cam.image_width, cam.image_height, cam.samples_per_pixel,
               spp ? spp : cam.samples_per_pixel, cam.max_depth, device);
  rt_render_opts o;
  std::memset(&o, 0, sizeof(o));
  o.seed = seed;
  o.row_begin = 0;
  o.row_step = 1;
  o.n_rows = cam.image_height;
  o.flags = RT_FLAG_OVERWRITE | (refsem ? RT_FLAG_SEMANTICS_REFERENCE : 0u);
  o.device = device;
  std::vector<float> accum((size_t)cam.image_width * cam.image_height * 3, 0.f);
  rt_stats st;
  int rc = rt_render_blob(&blob, &cam, &o, accum.data(), &st);
  if (rc != RT_OK) {
    std::fprintf(stderr, "rt_render: %d %s\n", rc, rt_last_error());
    return 1;
  }
  double msps = (double)st.samples / (st.ms_kernel * 1e3);
  std::fprintf(stderr, "kernel %.2f ms, %.1f Msamples/s\n", st.ms_kernel, msps);
  int64_t n = (int64_t)cam.image_width * cam.image_height;
  double ev = autoexp ? rth_auto_expose(accum.data(), n, cam.samples_per_pixel) : 0.0;
  std::vector<uint8_t> rgb(accum.size());
  rth_write_color(accum.data(), n, (double)cam.samples_per_pixel, autoexp ? 1 : 0, ev, rgb.data());
  if (rth_write_ppm(out.c_str(), rgb.data(), cam.image_width, cam.image_height) != 0) {
    std::fprintf(stderr, "%s\n", rth_last_error());
    return 1;
  }
  std::fprintf(stderr, "Done! wrote %s\n", out.c_str());
  rth_scene_free(s);
  return 0;
}
