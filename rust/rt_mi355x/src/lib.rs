//! rt_mi355x: the MI355X (gfx950) render loop of the reference's `render_par_lights`
//! (src/render.rs:144-216), behind the C ABI of librtmi355x.so (include/rt_mi355x.h).
//!
//! * [`ffi`]: `#[repr(C)]` mirrors of the header and the `extern "C"` entry points.
//! * [`blob`]: the scene-blob writer; the reference's types implement its traits in
//!   rust/reference_glue/ (child modules of their own modules).
//! * [`Scene`], [`render_blob`]: safe wrappers (status codes -> `Result`, `rt_last_error`).
//! * `gather` (feature "rccl-gather"): librtgather.so, the RCCL frame gather of one process per
//!   GPU (include/rt_gather.h).
//!
//! No dependencies; link with build.rs (RT_MI355X_LIB_DIR).

pub mod blob;
pub mod ffi;
#[cfg(feature = "rccl-gather")]
pub mod gather;

pub use blob::{Blob, BlobWriter, MaterialRecord, PerlinTables, TextureRecord, WriteBlob};

use std::ffi::CStr;
use std::os::raw::c_int;

/// A failed call: the library's status code and `rt_last_error()`.
#[derive(Debug, Clone)]
pub struct Error {
    pub code: c_int,
    pub message: String,
}

impl std::fmt::Display for Error {
    fn fmt(&self, f: &mut std::fmt::Formatter<'_>) -> std::fmt::Result {
        write!(f, "rt_mi355x error {}: {}", self.code, self.message)
    }
}
impl std::error::Error for Error {}

fn check(code: c_int) -> Result<(), Error> {
    if code == ffi::RT_OK {
        return Ok(());
    }
    let message = unsafe {
        let p = ffi::rt_last_error();
        if p.is_null() { String::new() } else { CStr::from_ptr(p).to_string_lossy().into_owned() }
    };
    Err(Error { code, message })
}

/// The library was built for this ABI.
pub fn abi_matches() -> bool {
    unsafe { ffi::rt_abi_version() == ffi::RT_ABI_VERSION }
}

pub fn device_count() -> Result<i32, Error> {
    let mut n: c_int = 0;
    check(unsafe { ffi::rt_device_count(&mut n) })?;
    Ok(n)
}

/// A flattened scene resident on one GPU (rt_scene_create). Renders of one scene may run from
/// several threads at once, each into its own buffer (rt_mi355x.h "Re-entrancy").
pub struct Scene {
    raw: *mut ffi::rt_scene,
}

unsafe impl Send for Scene {}
unsafe impl Sync for Scene {}

impl Scene {
    pub fn new(blob: &Blob, device: i32) -> Result<Scene, Error> {
        let view = blob.view();
        let mut raw: *mut ffi::rt_scene = std::ptr::null_mut();
        check(unsafe { ffi::rt_scene_create(&view, device, &mut raw) })?;
        Ok(Scene { raw })
    }

    /// Synchronous render into a host buffer of opts.n_rows * image_width * 3 floats: raw
    /// per-pixel sums over the samples, added into `accum` unless RT_FLAG_OVERWRITE.
    pub fn render(&self, cam: &ffi::rt_camera, opts: &ffi::rt_render_opts, accum: &mut [f32])
        -> Result<ffi::rt_stats, Error> {
        let need = opts.n_rows as usize * cam.image_width as usize * 3;
        if accum.len() < need {
            return Err(Error { code: ffi::RT_ERR_INVALID_ARG,
                               message: format!("accum holds {} floats, {} needed", accum.len(), need) });
        }
        let mut st = ffi::rt_stats::default();
        check(unsafe { ffi::rt_render(self.raw, cam, opts, accum.as_mut_ptr(), &mut st) })?;
        Ok(st)
    }

    /// Asynchronous render into a device buffer on a HIP stream (null = the default stream).
    ///
    /// # Safety
    /// `accum_device` must be a device allocation of opts.n_rows * image_width * 3 floats on
    /// this scene's device, and `hip_stream` a stream of that device (or null).
    pub unsafe fn render_device(&self, cam: &ffi::rt_camera, opts: &ffi::rt_render_opts,
                                accum_device: *mut f32, hip_stream: *mut std::os::raw::c_void)
        -> Result<(), Error> {
        check(ffi::rt_render_device(self.raw, cam, opts, accum_device, hip_stream,
                                    std::ptr::null_mut()))
    }

    pub fn device_bytes(&self) -> u64 {
        unsafe { ffi::rt_scene_device_bytes(self.raw) }
    }
}

impl Drop for Scene {
    fn drop(&mut self) {
        unsafe { ffi::rt_scene_destroy(self.raw) };
    }
}

/// One-shot drop-in for render_par_lights' loop: create, render, destroy (rt_render_blob).
pub fn render_blob(blob: &Blob, cam: &ffi::rt_camera, opts: &ffi::rt_render_opts,
                   accum: &mut [f32]) -> Result<ffi::rt_stats, Error> {
    let need = opts.n_rows as usize * cam.image_width as usize * 3;
    if accum.len() < need {
        return Err(Error { code: ffi::RT_ERR_INVALID_ARG,
                           message: format!("accum holds {} floats, {} needed", accum.len(), need) });
    }
    let view = blob.view();
    let mut st = ffi::rt_stats::default();
    check(unsafe { ffi::rt_render_blob(&view, cam, opts, accum.as_mut_ptr(), &mut st) })?;
    Ok(st)
}

/// Row-tiled rendering over several GPUs of one process (rt_render_multi): rows dealt
/// cyclically over `devices`, the frame de-interleaved into `accum`. Same image as one GPU.
pub fn render_multi(blob: &Blob, cam: &ffi::rt_camera, opts: &ffi::rt_render_opts,
                    devices: &[i32], accum: &mut [f32]) -> Result<ffi::rt_stats, Error> {
    let need = opts.n_rows as usize * cam.image_width as usize * 3;
    if accum.len() < need || devices.is_empty() {
        return Err(Error { code: ffi::RT_ERR_INVALID_ARG,
                           message: "accum too small or no devices".to_string() });
    }
    let view = blob.view();
    let mut st = ffi::rt_stats::default();
    check(unsafe {
        ffi::rt_render_multi(&view, cam, opts, devices.as_ptr(), devices.len() as c_int,
                             accum.as_mut_ptr(), &mut st)
    })?;
    Ok(st)
}
