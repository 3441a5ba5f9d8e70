//! Perlin tables of the reference's src/perlin.rs (Perlin 7-28): ranvec (256 x 3 f64), then
//! perm_x, perm_y, perm_z (256 each). Add to perlin.rs:
//!     #[path = "rt_glue/perlin_blob.rs"]
//!     mod rt_blob;
use super::Perlin;
use rt_mi355x::{BlobWriter, PerlinTables};

impl PerlinTables for Perlin {
    fn write_tables(&self, w: &mut BlobWriter<'_>) {
        // blob: perlin [ranvec 256 x 3, perm_x 256, perm_y 256, perm_z 256]
        for v in &self.ranvec {
            w.v3(v.x(), v.y(), v.z());
        }
        for p in [&self.perm_x, &self.perm_y, &self.perm_z] {
            for &k in p.iter() {
                w.i(k as i64);
            }
        }
    }
}
