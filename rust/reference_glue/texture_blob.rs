//! Texture records of the reference's src/texture.rs (Texture 10-131): [kind, p0..p6].
//! Add to texture.rs:
//!     #[path = "rt_glue/texture_blob.rs"]
//!     mod rt_blob;
use super::Texture;
use rt_mi355x::{BlobWriter, TextureRecord};

impl TextureRecord for Texture {
    fn register_children<'a>(&'a self, w: &mut BlobWriter<'a>) {
        match self {
            Texture::Checker(c) => {
                w.texture(&c.even);
                w.texture(&c.odd);
            }
            Texture::Noise(n) => {
                w.perlin(&n.noise);
            }
            Texture::Solid(_) | Texture::Image(_) => {}
        }
    }

    fn write_record(&self, w: &mut BlobWriter<'_>) {
        match self {
            Texture::Solid(s) => {
                // blob: solid [1, r, g, b]
                w.i(1);
                w.v3(s.color_value.x(), s.color_value.y(), s.color_value.z());
            }
            Texture::Checker(c) => {
                // blob: checker [2, inv_scale, even, odd]
                let (e, o) = (w.texture_id(&c.even), w.texture_id(&c.odd));
                w.i(2);
                w.f(c.inv_scale);
                w.i(e);
                w.i(o);
            }
            Texture::Image(t) => {
                // blob: image [3, width, height, texel offset]
                let (iw, ih, bytes) = t.image.rgb8(); // rt_image_blob.rs
                let off = w.push_texels(bytes);
                w.i(3);
                w.i(iw as i64);
                w.i(ih as i64);
                w.i(off);
            }
            Texture::Noise(n) => {
                // blob: noise [4, scale, perlin]
                let id = w.perlin_id(&n.noise);
                w.i(4);
                w.f(n.scale);
                w.i(id);
            }
        }
    }
}
