//! Mirrors of `include/rt_mi355x.h` (RT_ABI_VERSION 3): the C ABI of librtmi355x.so that
//! replaces the body of `render_par_lights` (reference src/render.rs:144-216). Field order and
//! widths match the header; tests/test_binding_mirror.py compares them with it.
#![allow(non_camel_case_types)]

use std::os::raw::{c_char, c_int, c_void};

pub const RT_ABI_VERSION: c_int = 3;

// status codes (rt_mi355x.h "status codes")
pub const RT_OK: c_int = 0;
pub const RT_ERR_INVALID_ARG: c_int = -1;
pub const RT_ERR_BAD_BLOB: c_int = -2;
pub const RT_ERR_UNSUPPORTED: c_int = -3;
pub const RT_ERR_EMPTY_LIGHTS: c_int = -4;
pub const RT_ERR_HIP: c_int = -5;
pub const RT_ERR_NO_DEVICE: c_int = -6;

// scene blob (rt_mi355x.h "scene blob")
pub const RT_BLOB_MAGIC: u64 = 0x52545343;
pub const RT_BLOB_VERSION: u64 = 1;
pub const RT_BLOB_HEADER_SLOTS: usize = 16;
pub const RT_TEX_SLOTS: usize = 8;
pub const RT_MAT_SLOTS: usize = 8;
pub const RT_PERLIN_POINTS: usize = 256;

// object tags, material and texture kinds
pub const RT_OBJ_LIST: i64 = 1;
pub const RT_OBJ_BVH: i64 = 2;
pub const RT_OBJ_SPHERE: i64 = 3;
pub const RT_OBJ_QUAD: i64 = 4;
pub const RT_OBJ_TRANSLATE: i64 = 5;
pub const RT_OBJ_ROTATE_Y: i64 = 6;
pub const RT_OBJ_VOLUME: i64 = 7;
pub const RT_MAT_LAMBERTIAN: u64 = 1;
pub const RT_MAT_METAL: u64 = 2;
pub const RT_MAT_DIELECTRIC: u64 = 3;
pub const RT_MAT_DIFFUSE_LIGHT: u64 = 4;
pub const RT_MAT_ISOTROPIC: u64 = 5;
pub const RT_TEX_SOLID: i64 = 1;
pub const RT_TEX_CHECKER: i64 = 2;
pub const RT_TEX_IMAGE: i64 = 3;
pub const RT_TEX_NOISE: i64 = 4;

// render flags
pub const RT_FLAG_OVERWRITE: u32 = 0x1;
pub const RT_FLAG_COUNT_OPS: u32 = 0x2;
pub const RT_FLAG_SEMANTICS_REFERENCE: u32 = 0x4;
pub const RT_FLAG_INTERPRETER: u32 = 0x8;
pub const RT_FLAG_REFERENCE_BVH: u32 = 0x10;

pub const RT_LAYOUT_STATS: c_int = 11;
pub const RT_LDS_CHECK: c_int = 19;
pub const RT_TRACE_HISTORY: c_int = 64;

#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct rt_scene_blob {
    pub slots: *const u64,
    pub n_slots: u64,
    pub texels: *const u8, // RGB8 images, row-major, top row first (image::to_rgb8)
    pub n_texels: u64,
}

/// Camera's derived fields (render.rs:15-36), computed on the host in f64.
#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct rt_camera {
    pub image_width: i32,
    pub image_height: i32,
    pub samples_per_pixel: i32, // nearest_square(spp), render.rs:38-41, 108
    pub sqrt_spp: i32,
    pub max_depth: i32, // < 2^24
    pub _pad0: i32,
    pub recip_sqrt_spp: f64,
    pub center: [f64; 3],
    pub pixel00_loc: [f64; 3],
    pub pixel_delta_u: [f64; 3],
    pub pixel_delta_v: [f64; 3],
    pub defocus_angle: f64,
    pub defocus_disk_u: [f64; 3],
    pub defocus_disk_v: [f64; 3],
    pub background: [f64; 3],
}

#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct rt_render_opts {
    pub seed: u64,      // render RNG seed
    pub row_begin: i32, // first image row of this call
    pub row_step: i32,  // 1 = contiguous band; G = cyclic tiling
    pub n_rows: i32,    // accum holds n_rows * image_width * 3 floats
    pub flags: u32,     // RT_FLAG_*
    pub sj_begin: i32,  // stratum rows [sj_begin, sj_begin + sj_count); 0 = all
    pub sj_count: i32,
    pub device: i32, // HIP device ordinal (rt_render only)
    pub _pad0: i32,
}

#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct rt_stats {
    pub ms_kernel: f64,
    pub ms_total: f64,
    pub samples: u64,
    pub ops: [u64; 32],  // rt_op_counter values (RT_FLAG_COUNT_OPS only)
    pub out_bytes: u64,  // f64 workspace bytes the path kernel stored
    pub launches: u32,   // path-kernel launches of the render
    pub _pad0: u32,
}

impl Default for rt_stats {
    fn default() -> Self {
        rt_stats { ms_kernel: 0.0, ms_total: 0.0, samples: 0, ops: [0; 32], out_bytes: 0,
                   launches: 0, _pad0: 0 }
    }
}

/// Opaque handles (rt_scene, rt_multi).
#[repr(C)]
pub struct rt_scene {
    _private: [u8; 0],
}
#[repr(C)]
pub struct rt_multi {
    _private: [u8; 0],
}

#[link(name = "rtmi355x")]
extern "C" {
    pub fn rt_abi_version() -> c_int;
    pub fn rt_last_error() -> *const c_char;
    pub fn rt_device_count(count: *mut c_int) -> c_int;
    pub fn rt_scene_validate(blob: *const rt_scene_blob) -> c_int;
    pub fn rt_scene_layout_stats(blob: *const rt_scene_blob, out: *mut u32, n: c_int) -> c_int;
    pub fn rt_scene_lds_check(blob: *const rt_scene_blob, flags: u32, n_rays: u32, seed: u64,
                              out: *mut u64, n: c_int, msg: *mut c_char, msg_len: u32) -> c_int;
    pub fn rt_scene_create(blob: *const rt_scene_blob, device: c_int, out: *mut *mut rt_scene)
        -> c_int;
    pub fn rt_scene_destroy(scene: *mut rt_scene);
    pub fn rt_scene_device_bytes(scene: *const rt_scene) -> u64;
    pub fn rt_scene_jit_info(scene: *mut rt_scene, state: *mut c_int, msg: *mut c_char,
                             msg_len: u32) -> c_int;
    pub fn rt_jit_check(blob: *const rt_scene_blob, arch: *const c_char, state: *mut c_int,
                        msg: *mut c_char, msg_len: u32) -> c_int;
    pub fn rt_render(scene: *mut rt_scene, cam: *const rt_camera, opts: *const rt_render_opts,
                     accum_rgb: *mut f32, stats: *mut rt_stats) -> c_int;
    pub fn rt_render_device(scene: *mut rt_scene, cam: *const rt_camera,
                            opts: *const rt_render_opts, accum_rgb_device: *mut f32,
                            hip_stream: *mut c_void, stats: *mut rt_stats) -> c_int;
    pub fn rt_scene_trace_ms(scene: *mut rt_scene, ms_out: *mut f32, max_n: c_int,
                             n_out: *mut c_int) -> c_int;
    pub fn rt_scene_prof_counters(scene: *mut rt_scene, out: *mut u64, n: c_int) -> c_int;
    pub fn rt_render_multi(blob: *const rt_scene_blob, cam: *const rt_camera,
                           opts: *const rt_render_opts, devices: *const c_int, n_devices: c_int,
                           accum_rgb: *mut f32, stats: *mut rt_stats) -> c_int;
    pub fn rt_multi_create(blob: *const rt_scene_blob, devices: *const c_int, n_devices: c_int,
                           out: *mut *mut rt_multi) -> c_int;
    pub fn rt_multi_render(multi: *mut rt_multi, cam: *const rt_camera,
                           opts: *const rt_render_opts, accum_rgb_device0: *mut f32,
                           hip_stream: *mut c_void, stats: *mut rt_stats) -> c_int;
    pub fn rt_multi_info(multi: *mut rt_multi, out: *mut u64, n: c_int) -> c_int;
    pub fn rt_multi_destroy(multi: *mut rt_multi);
    pub fn rt_render_blob(blob: *const rt_scene_blob, cam: *const rt_camera,
                          opts: *const rt_render_opts, accum_rgb: *mut f32,
                          stats: *mut rt_stats) -> c_int;
}
