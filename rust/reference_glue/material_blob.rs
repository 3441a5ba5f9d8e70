//! Material records of the reference's src/material.rs (Material 25-248): [kind, p0..p6].
//! Add to material.rs:
//!     #[path = "rt_glue/material_blob.rs"]
//!     mod rt_blob;
use super::Material;
use rt_mi355x::{BlobWriter, MaterialRecord};

impl MaterialRecord for Material {
    fn record<'a>(&'a self, w: &mut BlobWriter<'a>) -> [u64; 8] {
        let mut r = [0u64; 8];
        match self {
            Material::Lambertian(m) => {
                // blob: lambertian [1, tex]
                r[0] = 1;
                r[1] = w.texture(&m.texture) as u64;
            }
            Material::Metal(m) => {
                // blob: metal [2, r, g, b, fuzz]
                r[0] = 2;
                r[1] = m.albedo.x().to_bits();
                r[2] = m.albedo.y().to_bits();
                r[3] = m.albedo.z().to_bits();
                r[4] = m.fuzz.to_bits();
            }
            Material::Dielectric(m) => {
                // blob: dielectric [3, ir, r, g, b]
                r[0] = 3;
                r[1] = m.ir.to_bits();
                r[2] = m.tint.x().to_bits();
                r[3] = m.tint.y().to_bits();
                r[4] = m.tint.z().to_bits();
            }
            Material::DiffuseLight(m) => {
                // blob: diffuse_light [4, tex]
                r[0] = 4;
                r[1] = w.texture(&m.emit) as u64;
            }
            Material::Isotropic(m) => {
                // blob: isotropic [5, tex]
                r[0] = 5;
                r[1] = w.texture(&m.albedo) as u64;
            }
        }
        r
    }
}
