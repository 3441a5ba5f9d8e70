//! The scene-blob writer: a reference `HittableList` / `Object` tree -> the 64-bit slot array of
//! rt_mi355x.h ("scene blob"). The reference's types implement the traits below in child modules
//! of their own modules (their fields are private there): rust/reference_glue/*.rs, one file per
//! reference module. tests/test_binding_mirror.py checks every arm against the C++ host builder's
//! blobs of all preset scenes.

use std::collections::HashMap;
use std::sync::Arc;

use crate::ffi;

/// An object of the tree (Object and its variants' payloads, HittableList, BvhNode, ...).
pub trait WriteBlob {
    fn write_blob<'a>(&'a self, w: &mut BlobWriter<'a>);
}
/// A texture: its children first (checker: even, odd; noise: its Perlin table), then its record.
pub trait TextureRecord {
    fn register_children<'a>(&'a self, w: &mut BlobWriter<'a>);
    fn write_record(&self, w: &mut BlobWriter<'_>);
}
/// A material value: its 8-slot record (registering the textures it reads).
pub trait MaterialRecord {
    fn record<'a>(&'a self, w: &mut BlobWriter<'a>) -> [u64; ffi::RT_MAT_SLOTS];
}
/// A Perlin generator: ranvec (256 x 3 f64), then perm_x, perm_y, perm_z.
pub trait PerlinTables {
    fn write_tables(&self, w: &mut BlobWriter<'_>);
}

pub struct BlobWriter<'a> {
    pub slots: Vec<u64>,
    pub texels: Vec<u8>,
    mats: Vec<[u64; ffi::RT_MAT_SLOTS]>, // material records, deduplicated by value
    texs: Vec<&'a dyn TextureRecord>,     // texture table, in id order
    tex_ids: HashMap<usize, i64>,         // Arc<Texture> identity -> id
    perlins: Vec<&'a dyn PerlinTables>,
    perlin_ids: HashMap<usize, i64>, // Perlin identity (its address) -> id
}

/// A finished blob: slots + texels, and the C view of them.
pub struct Blob {
    pub slots: Vec<u64>,
    pub texels: Vec<u8>,
}

impl Blob {
    pub fn view(&self) -> ffi::rt_scene_blob {
        ffi::rt_scene_blob {
            slots: self.slots.as_ptr(),
            n_slots: self.slots.len() as u64,
            texels: self.texels.as_ptr(),
            n_texels: self.texels.len() as u64,
        }
    }
}

impl<'a> BlobWriter<'a> {
    pub fn f(&mut self, x: f64) {
        self.slots.push(x.to_bits());
    }
    pub fn i(&mut self, x: i64) {
        self.slots.push(x as u64);
    }
    pub fn v3(&mut self, x: f64, y: f64, z: f64) {
        self.f(x);
        self.f(y);
        self.f(z);
    }
    /// bbox6 = xmin xmax ymin ymax zmin zmax
    pub fn bbox(&mut self, b: [f64; 6]) {
        for v in b {
            self.f(v);
        }
    }

    /// serialize(world, lights): objects first (they register materials and textures), then the
    /// texture, material and Perlin tables, then the header (rt_mi355x.h "Header"). `lights` =
    /// None for render_par's empty light list (lights_off = -1).
    pub fn serialize(world: &'a dyn WriteBlob, lights: Option<&'a dyn WriteBlob>) -> Blob {
        let mut w = BlobWriter {
            slots: vec![0; ffi::RT_BLOB_HEADER_SLOTS],
            texels: vec![],
            mats: vec![],
            texs: vec![],
            tex_ids: HashMap::new(),
            perlins: vec![],
            perlin_ids: HashMap::new(),
        };
        let world_off = w.slots.len() as i64;
        world.write_blob(&mut w);
        let lights_off = match lights {
            Some(l) => {
                let off = w.slots.len() as i64;
                l.write_blob(&mut w);
                off
            }
            None => -1,
        };
        let tex_off = w.slots.len() as i64;
        let texs = w.texs.clone();
        for t in &texs {
            let base = w.slots.len();
            t.write_record(&mut w);
            while w.slots.len() < base + ffi::RT_TEX_SLOTS {
                w.i(0);
            }
        }
        let mat_off = w.slots.len() as i64;
        let mats = std::mem::take(&mut w.mats);
        for m in &mats {
            w.slots.extend_from_slice(m);
        }
        let perlin_off = w.slots.len() as i64;
        let perlins = w.perlins.clone();
        for p in &perlins {
            p.write_tables(&mut w);
        }
        let n = w.slots.len() as u64;
        let head = [ffi::RT_BLOB_MAGIC, ffi::RT_BLOB_VERSION, n, texs.len() as u64, tex_off as u64,
                    mats.len() as u64, mat_off as u64, perlins.len() as u64, perlin_off as u64,
                    world_off as u64, lights_off as u64, w.texels.len() as u64];
        w.slots[..12].copy_from_slice(&head);
        Blob { slots: w.slots, texels: w.texels }
    }

    /// Texture id by Arc identity; children are registered first, so ids are stable and
    /// children precede parents.
    pub fn texture<T: TextureRecord>(&mut self, t: &'a Arc<T>) -> i64 {
        let key = Arc::as_ptr(t) as *const u8 as usize;
        if let Some(&id) = self.tex_ids.get(&key) {
            return id;
        }
        t.as_ref().register_children(self);
        let id = self.texs.len() as i64;
        self.tex_ids.insert(key, id);
        self.texs.push(t.as_ref());
        id
    }
    /// The id of an already registered texture (a checker's children).
    pub fn texture_id<T>(&self, t: &Arc<T>) -> i64 {
        self.tex_ids[&(Arc::as_ptr(t) as *const u8 as usize)]
    }
    pub fn perlin<P: PerlinTables>(&mut self, p: &'a P) -> i64 {
        let key = p as *const P as *const u8 as usize;
        if let Some(&id) = self.perlin_ids.get(&key) {
            return id;
        }
        let id = self.perlins.len() as i64;
        self.perlin_ids.insert(key, id);
        self.perlins.push(p);
        id
    }
    pub fn perlin_id<P>(&self, p: &P) -> i64 {
        self.perlin_ids[&(p as *const P as *const u8 as usize)]
    }
    /// Material id: materials are values in the reference (make_box clones `&ground` into six
    /// quads), so equal records share one id.
    pub fn material<M: MaterialRecord>(&mut self, m: &'a M) -> i64 {
        let rec = m.record(self);
        if let Some(k) = self.mats.iter().position(|r| *r == rec) {
            return k as i64;
        }
        self.mats.push(rec);
        (self.mats.len() - 1) as i64
    }
    /// RGB8 texels of an image texture; returns their byte offset in the blob's texel array.
    pub fn push_texels(&mut self, rgb8: &[u8]) -> i64 {
        let off = self.texels.len() as i64;
        self.texels.extend_from_slice(rgb8);
        off
    }
}
