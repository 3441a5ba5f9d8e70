//! Scene-blob arms of the reference's src/transform.rs (Translate 19-74, RotateY 76-186).
//! Add to transform.rs:
//!     #[path = "rt_glue/transform_blob.rs"]
//!     mod rt_blob;
use super::Transform;
use crate::object::rt_blob::aabb6;
use rt_mi355x::{BlobWriter, WriteBlob};

impl WriteBlob for Transform {
    fn write_blob<'a>(&'a self, w: &mut BlobWriter<'a>) {
        match self {
            Transform::Translate(t) => {
                // blob: translate [RT_OBJ_TRANSLATE, offset3, bbox6], then the child
                w.i(5);
                w.v3(t.offset.x(), t.offset.y(), t.offset.z());
                w.bbox(aabb6(&t.bbox));
                t.object.write_blob(w);
            }
            Transform::RotY(r) => {
                // blob: rot_y [RT_OBJ_ROTATE_Y, sin, cos, bbox6], then the child
                w.i(6);
                w.f(r.sin_theta);
                w.f(r.cos_theta);
                w.bbox(aabb6(&r.bbox));
                r.object.write_blob(w);
            }
        }
    }
}
