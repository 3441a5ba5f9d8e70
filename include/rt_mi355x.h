/*
 * rt_mi355x.h — C ABI of the MI355X (gfx950) path-tracing library `librtmi355x.so`.
 *
 * This is the drop-in boundary for the reference's per-pixel render loop:
 *
 *   reference (Rust, no FFI exists upstream)           this ABI
 *   -----------------------------------------------    ------------------------------------------
 *   render_par_lights(cam, world, pixels, suns, lights) rt_render / rt_render_device
 *       /root/reference/src/render.rs:144-216               (scene blob + camera + opts -> accum)
 *   render_par(cam, world, pixels, suns)                rt_render with blob.lights_off == -1
 *       /root/reference/src/render.rs:140-142               (empty light list, see RT_FLAG_SEMANTICS_REFERENCE)
 *   Camera::new derived fields                          rt_camera (filled host-side, render.rs:62-133)
 *       /root/reference/src/render.rs:15-36
 *   HittableList / Object tree (world, lights)          rt_scene_blob (prefix-serialised tree,
 *       /root/reference/src/hittable.rs:55-130,             f64 slots, see "Scene blob" below)
 *       object.rs:17-71, transform.rs, constant_medium.rs
 *   pixels: &mut Vec<Color> (raw sums, pre-zeroed)      float* accum_rgb (raw sums over spp,
 *       /root/reference/src/render.rs:136-138, 189          added into unless RT_FLAG_OVERWRITE)
 *   panics (expect / panic!)                            int status < 0 + rt_last_error()
 *
 * Output stays host-side: write_color / the PPM writer (color.rs:8-33) are NOT behind this ABI;
 * accum holds raw per-pixel sums exactly like the reference's `pixels` vector.
 *
 * Every entry point is plain C: pointers, sizes, PODs. No torch, no C++ types.
 */
#ifndef RT_MI355X_H
#define RT_MI355X_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 3

/* ---- status codes ------------------------------------------------------------------------ */
#define RT_OK 0
#define RT_ERR_INVALID_ARG (-1)
#define RT_ERR_BAD_BLOB (-2)      /* malformed scene blob                                   */
#define RT_ERR_UNSUPPORTED (-3)   /* valid reference scene the device path cannot express    */
#define RT_ERR_EMPTY_LIGHTS (-4)  /* reference semantics: empty light list panics            */
                                  /* (hittable.rs:115-129 via render.rs:140-142)            */
#define RT_ERR_HIP (-5)           /* HIP runtime failure (message in rt_last_error)         */
#define RT_ERR_NO_DEVICE (-6)

/* ---- scene blob ---------------------------------------------------------------------------
 * A flat array of 64-bit slots. A slot holds an int64 or the bit pattern of an IEEE f64.
 * The host computes every derived quantity in f64 exactly as the reference constructors do
 * (Quad::new object.rs:427-446, Sphere::new 83-105, RotateY::new transform.rs:143-186, ...);
 * consumers round to their working precision.
 *
 * Header (slot index: meaning)
 *   0 magic RT_BLOB_MAGIC      1 version RT_BLOB_VERSION    2 n_slots
 *   3 n_textures  4 textures_off   (RT_TEX_SLOTS slots each)
 *   5 n_materials 6 materials_off  (RT_MAT_SLOTS slots each)
 *   7 n_perlin    8 perlin_off     (RT_PERLIN_SLOTS each: ranvec 256x3 f64, perm_x/y/z 3x256 int)
 *   9 world_off                    (object tree: the world HittableList)
 *  10 lights_off                   (object tree, or -1 = empty light list, as render_par)
 *  11 n_texel_bytes                (size of blob.texels; images index into it)
 *
 * Object tree: prefix order, records by tag (slot counts include the tag):
 *   RT_OBJ_LIST      [tag, n, bbox6]                       then n children      (hittable.rs:55-130)
 *   RT_OBJ_BVH       [tag, bbox6]                          then left, right     (hittable.rs:135-241)
 *   RT_OBJ_SPHERE    [tag, mat, moving, c3, radius, cvec3, bbox6]               (object.rs:73-213)
 *   RT_OBJ_QUAD      [tag, mat, q3, u3, v3, normal3, w3, d, area, bbox6]        (object.rs:414-507)
 *   RT_OBJ_TRANSLATE [tag, offset3, bbox6]                 then child           (transform.rs:19-74)
 *   RT_OBJ_ROTATE_Y  [tag, sin, cos, bbox6]                then child           (transform.rs:76-186)
 *   RT_OBJ_VOLUME    [tag, mat, neg_inv_density, bbox6]    then boundary        (constant_medium.rs)
 *   bbox6 = xmin xmax ymin ymax zmin zmax.
 * Material record [kind, p0..p6]:
 *   LAMBERTIAN [1, tex]   METAL [2, r, g, b, fuzz]   DIELECTRIC [3, ir, r, g, b]
 *   DIFFUSE_LIGHT [4, tex]   ISOTROPIC [5, tex]                                 (material.rs:25-248)
 * Texture record [kind, p0..p6]:
 *   SOLID [1, r, g, b]   CHECKER [2, inv_scale, even_tex, odd_tex]
 *   IMAGE [3, width, height, texel_byte_offset]  (width or height 0 = image absent -> (0,1,1))
 *   NOISE [4, scale, perlin_index]                                              (texture.rs:10-131)
 * ------------------------------------------------------------------------------------------ */
#define RT_BLOB_MAGIC 0x52545343 /* 'RTSC' */
#define RT_BLOB_VERSION 1
#define RT_BLOB_HEADER_SLOTS 16
#define RT_TEX_SLOTS 8
#define RT_MAT_SLOTS 8
#define RT_PERLIN_POINTS 256
#define RT_PERLIN_SLOTS (RT_PERLIN_POINTS * 3 + RT_PERLIN_POINTS * 3)

enum rt_obj_tag {
  RT_OBJ_LIST = 1,
  RT_OBJ_BVH = 2,
  RT_OBJ_SPHERE = 3,
  RT_OBJ_QUAD = 4,
  RT_OBJ_TRANSLATE = 5,
  RT_OBJ_ROTATE_Y = 6,
  RT_OBJ_VOLUME = 7
};
enum rt_mat_kind {
  RT_MAT_LAMBERTIAN = 1,
  RT_MAT_METAL = 2,
  RT_MAT_DIELECTRIC = 3,
  RT_MAT_DIFFUSE_LIGHT = 4,
  RT_MAT_ISOTROPIC = 5
};
enum rt_tex_kind { RT_TEX_SOLID = 1, RT_TEX_CHECKER = 2, RT_TEX_IMAGE = 3, RT_TEX_NOISE = 4 };

typedef struct rt_scene_blob {
  const uint64_t* slots;
  uint64_t n_slots;
  const uint8_t* texels; /* RGB8 images, row-major, top row first (as image::to_rgb8) */
  uint64_t n_texels;
} rt_scene_blob;

/* ---- camera: Camera's derived fields (render.rs:15-36), computed on the host in f64 ---------- */
typedef struct rt_camera {
  int32_t image_width;
  int32_t image_height;
  int32_t samples_per_pixel; /* effective spp = nearest_square(spp) (render.rs:38-41, 108) */
  int32_t sqrt_spp;
  int32_t max_depth;
  int32_t _pad0;
  double recip_sqrt_spp;
  double center[3];
  double pixel00_loc[3];
  double pixel_delta_u[3];
  double pixel_delta_v[3];
  double defocus_angle;
  double defocus_disk_u[3];
  double defocus_disk_v[3];
  double background[3];
} rt_camera;

/* ---- render options ---------------------------------------------------------------------- */
#define RT_FLAG_OVERWRITE 0x1u             /* accum = sums instead of accum += sums          */
#define RT_FLAG_COUNT_OPS 0x2u             /* run the op-counting build, fill rt_stats.ops   */
#define RT_FLAG_SEMANTICS_REFERENCE 0x4u   /* exact reference semantics: empty lights -> error, */
                                           /* Isotropic scattering_pdf = 0 */
#define RT_FLAG_INTERPRETER 0x8u           /* product render with the interpreter walker, not the */
                                           /* scene-specialised kernel (same image, bit for bit)  */
#define RT_FLAG_REFERENCE_BVH 0x10u        /* product render walks BVH subtrees in the reference's */
                                           /* own tree and order, not their ordered BVHs (same    */
                                           /* image, bit for bit)                                 */

typedef struct rt_render_opts {
  uint64_t seed;      /* render RNG seed                                   */
  int32_t row_begin;  /* first image row of this call                                          */
  int32_t row_step;   /* 1 = contiguous band; G = cyclic tiling (rows row_begin + k*G)         */
  int32_t n_rows;     /* rows rendered; accum holds n_rows * image_width * 3 floats            */
  uint32_t flags;     /* RT_FLAG_*                                                             */
  int32_t sj_begin;   /* stratum rows [sj_begin, sj_begin+sj_count) of the sqrt_spp x sqrt_spp */
  int32_t sj_count;   /* grid (render.rs:185); 0 = all. A subset keeps the full-spp jitter.   */
  int32_t device;     /* HIP device ordinal (rt_render only)                                   */
  int32_t _pad0;
} rt_render_opts;

/* Deterministic op counters (RT_FLAG_COUNT_OPS). Identical paths => identical counts on the
 * CPU oracle and the GPU, so per-sample work is measured, not assumed. */
enum rt_op_counter {
  RT_OP_SAMPLES = 0,      /* camera paths started                                     */
  RT_OP_WORLD_QUERIES,    /* world.hit calls (render.rs:264)                          */
  RT_OP_QUAD_TESTS,       /* Quad::hit entered (object.rs:453)                        */
  RT_OP_QUAD_PLANE,       /* ... passed the |n.d| >= 1e-8 test                        */
  RT_OP_QUAD_INTERVAL,    /* ... t inside the interval: planar coords computed        */
  RT_OP_QUAD_HITS,        /* ... accepted                                             */
  RT_OP_SPHERE_TESTS,     /* Sphere::hit entered (object.rs:145)                      */
  RT_OP_SPHERE_ROOTS,     /* ... discriminant >= 0                                    */
  RT_OP_SPHERE_HITS,      /* ... accepted                                             */
  RT_OP_AABB_TESTS,       /* Aabb::hit (object.rs:340) from BvhNode::hit              */
  RT_OP_TRANSLATE,        /* Translate::hit entered                                   */
  RT_OP_ROTATE_Y,         /* RotateY::hit entered                                     */
  RT_OP_VOLUME_TESTS,     /* ConstantMedium::hit entered                              */
  RT_OP_VOLUME_DRAWS,     /* ... free-flight distance drawn                           */
  RT_OP_MISSES,           /* world miss -> background                                 */
  RT_OP_EMISSIVE_HITS,    /* DiffuseLight hit (path ends)                             */
  RT_OP_LAMBERTIAN,       /* Lambertian scatter + mixture PDF                         */
  RT_OP_METAL,
  RT_OP_DIELECTRIC,
  RT_OP_ISOTROPIC,
  RT_OP_LIGHT_PDF_QUAD,   /* Quad::pdf_value (object.rs:492)                          */
  RT_OP_LIGHT_PDF_SPHERE, /* Sphere::pdf_value (object.rs:190)                        */
  RT_OP_LIGHT_GEN,        /* light-PDF generate (pdf.rs:120-126, first branch)        */
  RT_OP_COSINE_GEN,       /* material-PDF generate                                    */
  RT_OP_NOISE_EVALS,      /* NoiseTexture::value (texture.rs:127-130)                 */
  RT_OP_DEPTH_CUTOFF,     /* path ended by max_depth                                  */
  RT_OP_COUNT
};

typedef struct rt_stats {
  double ms_kernel;  /* device time of the render kernels (HIP events)             */
  double ms_total;   /* host wall time of the call                                  */
  uint64_t samples;  /* pixel-samples rendered by this call                         */
  uint64_t ops[32];  /* rt_op_counter values (RT_FLAG_COUNT_OPS only)               */
  uint64_t out_bytes; /* f64 workspace bytes the path kernel stored (row totals, block   */
                      /* partials, tail samples) and rt_reduce read back: a design choice, */
                      /* not the path's algorithmic bytes (the W*H*12 B f32 framebuffer)   */
  uint32_t launches;  /* path-kernel launches (stratum-row chunks) of the render        */
  uint32_t _pad0;
} rt_stats;

typedef struct rt_scene rt_scene; /* opaque: device-resident flattened scene + workspace */

int rt_abi_version(void);
const char* rt_last_error(void);
int rt_device_count(int* count);

/* Validate a blob without touching a device (hittable/object invariants, tag and index ranges). */
int rt_scene_validate(const rt_scene_blob* blob);

/* Host-only diagnostics of the flattened layout (no device needed): out[0..8] = node words,
 * BVH-region words, BVH records, DUP records (span-1 leaves tested once), ConstantMedium
 * records, of which one-walk sphere / one-walk quad boundaries, light records, and BVH
 * subtrees walked through an ordered BVH by the product kernels, of those the ones with a compact
 * copy for the walk from LDS, and the bytes of that compact region. */
#define RT_LAYOUT_STATS 11
int rt_scene_layout_stats(const rt_scene_blob* blob, uint32_t* out, int n);

/* Host-only check of a product render's LDS plan and of the compact BVHs its walk reads from LDS
 * (no device needed): out[0..18] = workgroup size, static LDS bound, staged table
 * bytes, compact-tree LDS offset (0xffffffff: not in LDS), compact-tree bytes, stack LDS offset,
 * stack bytes per lane (header cbvh_stack), dynamic LDS, static + dynamic, the CU's LDS, compact
 * trees, deepest tree (internal nodes, root = 1), structural errors, largest stack slot the
 * walk stores to, largest number of pending entries, rays walked, box steps, one past the
 * largest compact-region byte read, the row totals' LDS offset (0xffffffff: the launch renders
 * no row items). The walks are a host restatement of the LDS walk over
 * n_rays random rays per tree without closest-hit culling (the worst case for the stack).
 * msg (may be NULL) receives the first structural error. `flags`: the render's RT_FLAG_*. */
#define RT_LDS_CHECK 19
int rt_scene_lds_check(const rt_scene_blob* blob, uint32_t flags, uint32_t n_rays, uint64_t seed,
                       uint64_t* out, int n, char* msg, uint32_t msg_len);

/* Validate, flatten (threaded node array, f64 payloads; rt_layout.h) and upload to `device`. */
int rt_scene_create(const rt_scene_blob* blob, int device, rt_scene** out);
void rt_scene_destroy(rt_scene* scene);
/* Bytes of the device-side flattened scene (nodes + materials + textures + tables). */
uint64_t rt_scene_device_bytes(const rt_scene* scene);
/* Scene-specialised product kernel (the world walker generated from the scene and compiled by
 * hiprtc on the first product render; a BVH subtree record calls the per-lane BVH walk from the
 * generated walker, so BVH scenes such as final_scene run it too).
 * *state: 1 compiled and in use, 0 not compiled yet, -1 not generated for this scene (or
 * RT_JIT=0), -2 compilation failed (the interpreter kernel runs). msg: the reason or the log. */
int rt_scene_jit_info(rt_scene* scene, int* state, char* msg, uint32_t msg_len);
/* Host-only check of the scene-specialised kernel (no device needed): generate the walker for
 * `blob` and compile it with hiprtc for `arch` (e.g. "gfx950"). RT_OK with *state = 1 (compiled;
 * msg receives the generated walker source) or -1 (not generated; msg says why); a negative
 * status when compilation fails (msg receives the log). */
int rt_jit_check(const rt_scene_blob* blob, const char* arch, int* state, char* msg,
                 uint32_t msg_len);

/* Re-entrancy (render_par_lights takes &HittableList and may run concurrently, render.rs:144-150):
 * renders of ONE scene may be issued from several host threads and on several streams at once,
 * each into its own output buffer. Every render call takes a private slot of per-render state
 * (pool-queue word, op counters, f64 workspace, events): a slot whose previous render has
 * finished or went to the same stream handle, else a new one (up to 8 per scene; beyond that a
 * call waits for a slot to finish); the call's stream always waits for the slot's previous
 * render (an event wait: equal handles such as hipStreamPerThread are different streams in
 * different threads), and a call that fails after enqueuing work still marks the slot busy
 * until that work ends. Renders on different streams therefore run concurrently and each
 * gives its serial image bit for bit. Two renders into the SAME output buffer are ordered only by
 * the caller (same stream, or events). rt_scene_destroy must not race with renders of the scene. */

/* Synchronous: render into a HOST buffer (n_rows * W * 3 floats). */
int rt_render(rt_scene* scene, const rt_camera* cam, const rt_render_opts* opts, float* accum_rgb,
              rt_stats* stats);

/* Asynchronous on `hip_stream` (hipStream_t, may be NULL): render into a DEVICE buffer.
 * If stats != NULL the call synchronises the stream to fill it. Limits: image_width <= 65535
 * and samples_per_pixel < 2^30 (sqrt_spp <= 32768; RT_ERR_UNSUPPORTED beyond); any number of
 * rows (row ranges taller than 32760 rows run as consecutive sub-renders, same image).
 * rt_scene_destroy waits for the scene's renders. */
int rt_render_device(rt_scene* scene, const rt_camera* cam, const rt_render_opts* opts,
                     float* accum_rgb_device, void* hip_stream, rt_stats* stats);

/* Device time (ms) of the path-tracing kernel alone (rt_trace, every chunk of one render summed;
 * HIP events recorded on the render stream around its launches) for the most recent renders
 * of `scene`, oldest first: up to max_n values, *n_out = count. Waits for those events. Used by
 * the benchmark's roofline so the figure excludes the per-pixel reduction. */
#define RT_TRACE_HISTORY 64
int rt_scene_trace_ms(rt_scene* scene, float* ms_out, int max_n, int* n_out);

/* Diagnostics: counters of a profiling build of the library (-DRT_PROF, tools_gpu/) from the
 * scene's latest render; zeros in the product build. */
int rt_scene_prof_counters(rt_scene* scene, uint64_t* out, int n);

/* Multi-GPU in ONE host process (no RCCL needed): the call's rows are dealt cyclically over
 * devices[0..n_devices) (row r of the call -> device r mod n), every device renders
 * its rows concurrently on its own stream, and the host buffer accum_rgb (opts->n_rows * W * 3)
 * receives the de-interleaved frame. Bit for bit the image of rt_render on one device (the RNG
 * is keyed by global pixel and sample). A device may be listed more than once. stats: samples,
 * ms_total (= ms_kernel: host wall time), launches = n_devices. render_par_lights over N GPUs
 * (render.rs:144-216). One process per GPU instead: rt_render_device on cyclic rows + an RCCL
 * gather. */
int rt_render_multi(const rt_scene_blob* blob, const rt_camera* cam, const rt_render_opts* opts,
                    const int* devices, int n_devices, float* accum_rgb, rt_stats* stats);

/* Persistent multi-GPU handle (one host process driving N GPUs, frame after frame; the same
 * role as render_par_lights rendering one frame per call over every core, render.rs:144-216).
 * rt_multi_create uploads the scene to each listed device ONCE (a device may be listed more than
 * once); every device keeps its scene, workspace, stream, row buffer and compiled kernel across
 * calls. rt_multi_render: the call's rows are dealt cyclically (row r of the call -> devices[r mod
 * n]), every device renders its rows on its own stream, the rows are copied peer to peer
 * (hipMemcpyPeerAsync, xGMI) into a staging buffer on devices[0], and a kernel there
 * de-interleaves them into accum_rgb_device0 (a devices[0] buffer of opts->n_rows * W * 3
 * floats; overwritten or added to as opts->flags says). Asynchronous on hip_stream (a devices[0]
 * stream, may be NULL); stats != NULL synchronises it. Bit for bit the image of rt_render_device
 * on one device. Consecutive frames of one handle are ordered on devices[0] (a frame waits for the
 * previous frame's gather, whatever stream each was issued on); calls from several host threads
 * are serialised. rt_multi_info: out[0..3] = frames rendered, scene uploads, staging-buffer
 * allocations, devices. */
typedef struct rt_multi rt_multi;
int rt_multi_create(const rt_scene_blob* blob, const int* devices, int n_devices, rt_multi** out);
int rt_multi_render(rt_multi* multi, const rt_camera* cam, const rt_render_opts* opts,
                    float* accum_rgb_device0, void* hip_stream, rt_stats* stats);
int rt_multi_info(rt_multi* multi, uint64_t* out, int n);
void rt_multi_destroy(rt_multi* multi);

/* One-shot drop-in for render_par_lights: create + render + destroy. */
int rt_render_blob(const rt_scene_blob* blob, const rt_camera* cam, const rt_render_opts* opts,
                   float* accum_rgb, rt_stats* stats);

#ifdef __cplusplus
}
#endif
#endif /* RT_MI355X_H */
