//! Scene-blob arm of the reference's src/constant_medium.rs (ConstantMedium 15-38).
//! Add to constant_medium.rs:
//!     #[path = "rt_glue/constant_medium_blob.rs"]
//!     mod rt_blob;
use super::ConstantMedium;
use crate::hittable::Hittable;
use crate::object::rt_blob::aabb6;
use rt_mi355x::{BlobWriter, WriteBlob};

impl WriteBlob for ConstantMedium {
    fn write_blob<'a>(&'a self, w: &mut BlobWriter<'a>) {
        // blob: volume [RT_OBJ_VOLUME, mat, neg_inv_density, bbox6], then the boundary
        let mat = w.material(&self.phase_function); // an Isotropic
        w.i(7);
        w.i(mat);
        w.f(self.neg_inv_density);
        w.bbox(aabb6(self.boundary.bounding_box().expect("boundary without a box")));
        self.boundary.write_blob(w);
    }
}
