//! Scene-blob arms of the reference's src/object.rs (object.rs:17-71, Sphere 73-213, Quad 414-507).
//! A child module of object.rs, so it reads the private fields. Add to object.rs:
//!     #[path = "rt_glue/object_blob.rs"]
//!     pub(crate) mod rt_blob;
use super::{Aabb, Object, Quad, Sphere};
use crate::vec3::Vec3;
use rt_mi355x::{BlobWriter, WriteBlob};

/// bbox6 = xmin xmax ymin ymax zmin zmax (Aabb's Intervals, interval.rs:14-18)
pub(crate) fn aabb6(b: &Aabb) -> [f64; 6] {
    [b.x.min, b.x.max, b.y.min, b.y.max, b.z.min, b.z.max]
}

impl WriteBlob for Object {
    fn write_blob<'a>(&'a self, w: &mut BlobWriter<'a>) {
        match self {
            Object::List(l) => l.write_blob(w),      // hittable_blob.rs
            Object::Node(n) => n.write_blob(w),      // hittable_blob.rs
            Object::Sphere(s) => s.write_blob(w),
            Object::Quad(q) => q.write_blob(w),
            Object::Transform(t) => t.write_blob(w), // transform_blob.rs
            Object::Volume(v) => v.write_blob(w),    // constant_medium_blob.rs
            Object::_Plane(_) => panic!("Plane is not reachable from the reference's scenes"),
        }
    }
}

impl WriteBlob for Sphere {
    fn write_blob<'a>(&'a self, w: &mut BlobWriter<'a>) {
        // blob: sphere [RT_OBJ_SPHERE, mat, moving, center3, radius, center_vec3, bbox6]
        let mat = w.material(&self.mat);
        let cv = self.center_vec.unwrap_or(Vec3::new(0., 0., 0.));
        w.i(3);
        w.i(mat);
        w.i(self.center_vec.is_some() as i64);
        w.v3(self.center.x(), self.center.y(), self.center.z());
        w.f(self.radius);
        w.v3(cv.x(), cv.y(), cv.z());
        w.bbox(aabb6(&self.bbox));
    }
}

impl WriteBlob for Quad {
    fn write_blob<'a>(&'a self, w: &mut BlobWriter<'a>) {
        // blob: quad [RT_OBJ_QUAD, mat, q3, u3, v3, normal3, w3, d, area, bbox6]
        let mat = w.material(&self.mat);
        w.i(4);
        w.i(mat);
        w.v3(self.q.x(), self.q.y(), self.q.z());
        w.v3(self.u.x(), self.u.y(), self.u.z());
        w.v3(self.v.x(), self.v.y(), self.v.z());
        w.v3(self.normal.x(), self.normal.y(), self.normal.z());
        w.v3(self.w.x(), self.w.y(), self.w.z());
        w.f(self.d);
        w.f(self.area);
        w.bbox(aabb6(&self.bbox));
    }
}
