"""Device buffers for GPU tests without torch: hipMalloc / hipMemcpy / hipFree through the HIP
runtime librtmi355x.so itself links (libamdhip64.so.7). A test process that initialises torch's
bundled HIP runtime next to it can find no device; the bench imports torch first and never
allocates through this helper. Test infrastructure only."""
import ctypes as C

import numpy as np

import surely_rt as rt

_hip = None


def hip() -> C.CDLL:
    global _hip
    if _hip is None:
        rt.device_lib()  # loads libamdhip64.so.7 as a dependency
        _hip = C.CDLL("libamdhip64.so.7")
        _hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
        _hip.hipFree.argtypes = [C.c_void_p]
        _hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        _hip.hipSetDevice.argtypes = [C.c_int]
        _hip.hipDeviceSynchronize.argtypes = []
        _hip.hipStreamCreateWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_uint]
        _hip.hipStreamSynchronize.argtypes = [C.c_void_p]
        _hip.hipStreamDestroy.argtypes = [C.c_void_p]
    return _hip


class Stream:
    """A non-blocking HIP stream on `device` (hipStreamCreateWithFlags)."""

    def __init__(self, device: int = 0):
        h = hip()
        assert h.hipSetDevice(device) == 0
        s = C.c_void_p()
        assert h.hipStreamCreateWithFlags(C.byref(s), 1) == 0  # hipStreamNonBlocking
        self.handle = s.value

    def sync(self):
        assert hip().hipStreamSynchronize(C.c_void_p(self.handle)) == 0

    def destroy(self):
        if self.handle:
            self.sync()
            hip().hipStreamDestroy(C.c_void_p(self.handle))
            self.handle = None


class DevBuf:
    """A float32 device buffer of `shape` on `device`."""

    H2D, D2H = 1, 2

    def __init__(self, shape, device: int = 0, init: np.ndarray | None = None):
        self.shape = tuple(shape)
        self.nbytes = int(np.prod(self.shape)) * 4
        self.device = device
        h = hip()
        assert h.hipSetDevice(device) == 0
        p = C.c_void_p()
        assert h.hipMalloc(C.byref(p), self.nbytes) == 0
        self.ptr = p.value
        self.upload(np.zeros(self.shape, np.float32) if init is None else init)

    def upload(self, a: np.ndarray):
        a = np.ascontiguousarray(a, np.float32)
        assert a.shape == self.shape
        assert hip().hipMemcpy(C.c_void_p(self.ptr), a.ctypes.data, self.nbytes, self.H2D) == 0

    def download(self) -> np.ndarray:
        hip().hipDeviceSynchronize()
        out = np.empty(self.shape, np.float32)
        assert hip().hipMemcpy(out.ctypes.data, C.c_void_p(self.ptr), self.nbytes, self.D2H) == 0
        return out

    def free(self):
        if self.ptr:
            hip().hipFree(C.c_void_p(self.ptr))
            self.ptr = None
