//! Mirrors of `include/rt_gather.h`: librtgather.so, the framebuffer gather of a row-tiled render
//! over RCCL for a host that runs one process per GPU (feature "rccl-gather"; build.rs links it).
//! tests/test_binding_mirror.py compares the entry points with the header.
#![allow(non_camel_case_types)]

use std::os::raw::{c_char, c_int, c_void};

pub const RT_GATHER_ID_BYTES: usize = 128;

/// Opaque handle: an RCCL communicator and its device.
#[repr(C)]
pub struct rt_gather_comm {
    _private: [u8; 0],
}

#[link(name = "rtgather")]
extern "C" {
    pub fn rt_gather_last_error() -> *const c_char;
    pub fn rt_gather_unique_id(id_out: *mut u8) -> c_int;
    pub fn rt_gather_comm_create(id: *const u8, world: c_int, rank: c_int, device: c_int,
                                 out: *mut *mut rt_gather_comm) -> c_int;
    pub fn rt_gather_comm_destroy(comm: *mut rt_gather_comm);
    pub fn rt_gather_rows(height: c_int, world: c_int, rank: c_int) -> c_int;
    pub fn rt_gather_max_rows(height: c_int, world: c_int) -> c_int;
    pub fn rt_gather_frame(comm: *mut rt_gather_comm, local_rows: *const f32, width: c_int,
                           height: c_int, scratch: *mut f32, frame: *mut f32,
                           hip_stream: *mut c_void) -> c_int;
    pub fn rt_gather_deinterleave(gathered: *const f32, world: c_int, width: c_int,
                                  height: c_int, frame: *mut f32, hip_stream: *mut c_void)
        -> c_int;
}

/// A rank's member of the gather communicator.
pub struct FrameGather {
    raw: *mut rt_gather_comm,
    pub world: i32,
    pub rank: i32,
}

unsafe impl Send for FrameGather {}

fn gather_error(code: c_int) -> crate::Error {
    let message = unsafe {
        let p = rt_gather_last_error();
        if p.is_null() {
            String::new()
        } else {
            std::ffi::CStr::from_ptr(p).to_string_lossy().into_owned()
        }
    };
    crate::Error { code, message }
}

impl FrameGather {
    /// Rank 0: the communicator id, to be sent to every rank over any channel.
    pub fn unique_id() -> Result<[u8; RT_GATHER_ID_BYTES], crate::Error> {
        let mut id = [0u8; RT_GATHER_ID_BYTES];
        match unsafe { rt_gather_unique_id(id.as_mut_ptr()) } {
            0 => Ok(id),
            c => Err(gather_error(c)),
        }
    }

    /// Every rank (collective): join as `rank` of `world` on HIP device `device`.
    pub fn new(id: &[u8; RT_GATHER_ID_BYTES], world: i32, rank: i32, device: i32)
        -> Result<FrameGather, crate::Error> {
        let mut raw = std::ptr::null_mut();
        match unsafe { rt_gather_comm_create(id.as_ptr(), world, rank, device, &mut raw) } {
            0 => Ok(FrameGather { raw, world, rank }),
            c => Err(gather_error(c)),
        }
    }

    /// Rows this rank renders (row_begin = rank, row_step = world) and the padded row count of
    /// its device buffer.
    pub fn rows(&self, height: i32) -> (i32, i32) {
        unsafe { (rt_gather_rows(height, self.world, self.rank), rt_gather_max_rows(height, self.world)) }
    }

    /// Every rank (collective, asynchronous on `hip_stream`): gather the padded local rows to
    /// rank 0 and de-interleave them into `frame` there (scratch/frame null on other ranks).
    ///
    /// # Safety
    /// Device pointers of the sizes rt_gather.h states, on this communicator's device.
    pub unsafe fn gather(&self, local_rows: *const f32, width: i32, height: i32, scratch: *mut f32,
                         frame: *mut f32, hip_stream: *mut c_void) -> Result<(), crate::Error> {
        match rt_gather_frame(self.raw, local_rows, width, height, scratch, frame, hip_stream) {
            0 => Ok(()),
            c => Err(gather_error(c)),
        }
    }
}

impl Drop for FrameGather {
    fn drop(&mut self) {
        unsafe { rt_gather_comm_destroy(self.raw) };
    }
}
