//! RGB8 texels of the reference's src/rt_image.rs (RtImage 6-46): rows top first, as
//! image::to_rgb8 stores them. Add to rt_image.rs:
//!     #[path = "rt_glue/rt_image_blob.rs"]
//!     mod rt_blob;
use super::RtImage;

impl RtImage {
    pub(crate) fn rgb8(&self) -> (u32, u32, &[u8]) {
        (self.image_width, self.image_height, self.image.as_raw())
    }
}
