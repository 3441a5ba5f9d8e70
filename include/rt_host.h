/*
 * rt_host.h — C API of the host-side scene builder `librthost.so`.
 *
 * The reference keeps scene construction in Rust (main.rs + the constructors of hittable.rs,
 * object.rs, transform.rs, constant_medium.rs, material.rs, texture.rs, perlin.rs). The north
 * star keeps that API on the host and hands a flattened buffer across the C ABI
 * (rt_mi355x.h). Rust is not available in this image, so the host mirror is C++
 * (surely-raytracing_amd/csrc/host/scene.hpp, same constructor vocabulary); this header exposes
 * it to C / ctypes / cgo-style callers. Every constructor cites the reference function whose
 * construction-time arithmetic it restates.
 *
 * Object/material/texture handles are small non-negative int32 ids owned by an rth_scene.
 * Negative return = error (message in rth_last_error()).
 */
#ifndef RT_HOST_H
#define RT_HOST_H

#include <stdint.h>
#include "rt_mi355x.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rth_scene rth_scene;

const char* rth_last_error(void);

/* Scene-build randomness (main.rs:617,688; hittable.rs:150; perlin.rs:19,111) comes from one
 * seeded stream owned by the scene. */
rth_scene* rth_scene_new(uint64_t build_seed);
void rth_scene_free(rth_scene* s);
double rth_random_double(rth_scene* s);                       /* utils.rs:5-7   */
double rth_random_range(rth_scene* s, double min, double max); /* utils.rs:9-11  */
int64_t rth_random_int(rth_scene* s, int64_t min, int64_t max); /* utils.rs:13-15 */

/* textures (texture.rs) */
int32_t rth_solid_color(rth_scene* s, double r, double g, double b);              /* :36-39   */
int32_t rth_checker_texture(rth_scene* s, double scale, int32_t even, int32_t odd); /* :55-61 */
int32_t rth_noise_texture(rth_scene* s, double scale); /* :116-121, Perlin::new perlin.rs:15-28 */
int32_t rth_image_texture(rth_scene* s, int32_t width, int32_t height,
                          const uint8_t* rgb8); /* :89-93; width=height=0 -> absent image */

/* materials (material.rs) */
int32_t rth_lambertian(rth_scene* s, double r, double g, double b); /* :81-85  */
int32_t rth_lambertian_tex(rth_scene* s, int32_t tex);                /* :87-89  */
int32_t rth_metal(rth_scene* s, double r, double g, double b, double fuzz); /* :118-121 */
int32_t rth_dielectric(rth_scene* s, double ir, double r, double g, double b); /* :148-154 */
int32_t rth_diffuse_light(rth_scene* s, double r, double g, double b); /* :200-204 */
int32_t rth_diffuse_light_tex(rth_scene* s, int32_t tex);               /* :206-208 */
int32_t rth_isotropic(rth_scene* s, double r, double g, double b);     /* :230-234 */
int32_t rth_isotropic_tex(rth_scene* s, int32_t tex);                   /* :236-238 */

/* objects (object.rs, hittable.rs, transform.rs, constant_medium.rs) */
int32_t rth_sphere(rth_scene* s, const double center[3], double radius, int32_t mat); /* :83-92 */
int32_t rth_sphere_moving(rth_scene* s, const double c1[3], const double c2[3], double radius,
                          int32_t mat);                                            /* :94-105 */
int32_t rth_quad(rth_scene* s, const double q[3], const double u[3], const double v[3],
                 int32_t mat);                                                     /* :427-446 */
int32_t rth_make_box(rth_scene* s, const double a[3], const double b[3], int32_t mat); /* :509-560 */
int32_t rth_list_new(rth_scene* s);                                   /* hittable.rs:61-66  */
int32_t rth_list_add(rth_scene* s, int32_t list, int32_t obj);        /* hittable.rs:74-80  */
int32_t rth_list_create_bvh(rth_scene* s, int32_t list);              /* hittable.rs:82-84  */
int32_t rth_list_len(rth_scene* s, int32_t list);
int32_t rth_translate(rth_scene* s, int32_t obj, const double offset[3]); /* transform.rs:43-54 */
int32_t rth_rotate_y(rth_scene* s, int32_t obj, double angle_deg);     /* transform.rs:143-186 */
int32_t rth_constant_medium(rth_scene* s, int32_t boundary, double density, double r, double g,
                            double b);                            /* constant_medium.rs:21-27 */
int32_t rth_constant_medium_tex(rth_scene* s, int32_t boundary, double density, int32_t tex);
int rth_object_bbox(rth_scene* s, int32_t obj, double out6[6]);

/* Serialise world (a list) + lights (any object, or -1 = empty list as render_par) into the
 * rt_scene_blob format. The blob memory is owned by `s` and valid until the next call. */
int rth_serialize(rth_scene* s, int32_t world_list, int32_t lights, rt_scene_blob* out);

/* Camera::new (render.rs:62-133) in f64; spp is rounded by nearest_square (render.rs:38-41). */
int rth_camera_new(double aspect_ratio, int32_t image_width, int32_t samples_per_pixel,
                   int32_t max_depth, double vfov, const double lookfrom[3],
                   const double lookat[3], const double vup[3], double defocus_angle,
                   double focus_dist, const double background[3], rt_camera* out);

/* Scene presets restating main.rs (scene fns + their Camera::new literals). Overrides <= 0 keep
 * the reference value. variant: "" or "mixed_pdf" (cornell_box with box2 and lights = quad only,
 * the revision behind final_images/mixed_pdf.png). Names: cornell_box, cornell_smoke,
 * final_scene, quads, simple_light, two_spheres, two_perlin_spheres, random_balls,
 * three_spheres, earth. */
int rth_preset(rth_scene* s, const char* name, const char* variant, int32_t width,
               int32_t samples_per_pixel, int32_t max_depth, double aspect_ratio,
               int32_t* world_out, int32_t* lights_out, rt_camera* cam_out);

/* Output stage (color.rs:8-59, render.rs:325-339): raw sums -> sRGB8 exactly as write_color. */
double rth_auto_expose(const float* accum, int64_t n_pixels, int32_t samples_per_pixel);
int rth_write_color(const float* accum, int64_t n_pixels, double samples_per_pixel,
                    int use_exposure, double exposure, uint8_t* rgb8_out);
int rth_write_ppm(const char* path, const uint8_t* rgb8, int32_t width, int32_t height);

#ifdef __cplusplus
}
#endif
#endif /* RT_HOST_H */
