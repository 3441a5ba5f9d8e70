//! Scene-blob arms of the reference's src/hittable.rs (HittableList 55-130, BvhNode 135-241).
//! Add to hittable.rs:
//!     #[path = "rt_glue/hittable_blob.rs"]
//!     mod rt_blob;
use super::{BvhNode, HittableList};
use crate::object::rt_blob::aabb6;
use rt_mi355x::{BlobWriter, WriteBlob};

impl WriteBlob for HittableList {
    fn write_blob<'a>(&'a self, w: &mut BlobWriter<'a>) {
        // blob: list [RT_OBJ_LIST, n, bbox6], then the n children in order
        w.i(1);
        w.i(self.objects.len() as i64);
        w.bbox(aabb6(&self.bbox));
        for o in &self.objects {
            o.write_blob(w);
        }
    }
}

impl WriteBlob for BvhNode {
    fn write_blob<'a>(&'a self, w: &mut BlobWriter<'a>) {
        // blob: node [RT_OBJ_BVH, bbox6], then left, right (BvhNode::new's topology kept)
        w.i(2);
        w.bbox(aabb6(&self.bbox));
        self.left.write_blob(w);
        self.right.write_blob(w);
    }
}
