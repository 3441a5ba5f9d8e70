//! render_par_lights (reference src/render.rs:144-216) with its loop body (171-197) on the GPU.
//! A child module of render.rs (it reads Camera's private fields and calls the output tail).
//! Add to render.rs:
//!     #[path = "rt_glue/render_mi355x.rs"]
//!     pub mod mi355x;
//! and call `render::mi355x::render_par_lights` where main.rs calls `render_par_lights`
//! (render_par = the same with an empty light list, render.rs:140-142).
use std::sync::Arc;

use super::{auto_expose, Camera};
use crate::color::{write_color, Color};
use crate::hittable::HittableList;
use crate::object::{Object, Sun};
use rt_mi355x::{ffi, BlobWriter, WriteBlob};

impl Camera {
    /// Camera::new's derived fields (render.rs:62-133), as computed there.
    pub(crate) fn to_rt_camera(&self) -> ffi::rt_camera {
        let v = |p: &crate::vec3::Vec3| [p.x(), p.y(), p.z()];
        ffi::rt_camera {
            image_width: self.image_width,
            image_height: self.image_height,
            samples_per_pixel: self.samples_per_pixel,
            sqrt_spp: self.sqrt_spp,
            max_depth: self.max_depth,
            _pad0: 0,
            recip_sqrt_spp: self.recip_sqrt_spp,
            center: v(&self.center),
            pixel00_loc: v(&self.pixel00_loc),
            pixel_delta_u: v(&self.pixel_delta_u),
            pixel_delta_v: v(&self.pixel_delta_v),
            defocus_angle: self.defocus_angle,
            defocus_disk_u: v(&self.defocus_disk_u),
            defocus_disk_v: v(&self.defocus_disk_v),
            background: v(&self.background),
        }
    }
}

/// The empty HittableList of render_par (render.rs:141) is the ABI's empty light list.
fn light_tree(lights: &Object) -> Option<&dyn WriteBlob> {
    match lights {
        Object::List(l) if l.objects.is_empty() => None,
        other => Some(other),
    }
}

pub fn render_par_lights(cam: &Camera, world: &HittableList, pixels: &mut Vec<Color>,
                         _suns: &Vec<Sun>, lights: Arc<Object>) {
    println!("P3\n{} {}\n255", cam.image_width, cam.image_height);
    let blob = BlobWriter::serialize(world, light_tree(&lights));
    let rc = cam.to_rt_camera();
    let opts = ffi::rt_render_opts { seed: 1, row_begin: 0, row_step: 1, n_rows: cam.image_height,
                                     flags: ffi::RT_FLAG_OVERWRITE, sj_begin: 0, sj_count: 0,
                                     device: 0, _pad0: 0 };
    let mut accum = vec![0f32; (cam.image_width * cam.image_height * 3) as usize];
    if let Err(e) = rt_mi355x::render_blob(&blob, &rc, &opts, &mut accum) {
        panic!("{}", e); // the reference panics where it cannot render (expect / panic!)
    }
    // raw per-pixel sums, added into the caller's pixels as render.rs:189 does
    for (px, c) in pixels.iter_mut().zip(accum.chunks_exact(3)) {
        *px = *px + Color::new(c[0] as f64, c[1] as f64, c[2] as f64);
    }
    // the output tail, unchanged (render.rs:199-215)
    let exposure = if cam.auto_exposure { Some(auto_expose(cam, pixels)) } else { None };
    for pixel in pixels.iter() {
        write_color(&mut std::io::stdout(), pixel, cam.samples_per_pixel as f64, exposure);
    }
}
