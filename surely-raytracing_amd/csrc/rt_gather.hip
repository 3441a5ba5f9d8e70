// rt_gather.hip — the framebuffer gather of a row-tiled multi-GPU render over RCCL
// (include/rt_gather.h). One ncclGather of every rank's padded cyclic rows to rank 0, then one
// de-interleave kernel there; the render library itself (librtmi355x.so) has no RCCL dependency.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <string>

#include "rt_gather.h"
#include "rt_mi355x.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& m) {
  g_err = m;
  return code;
}

// gathered: world blocks of max_rows rows; image row y lives in block y % world at row y / world
__global__ __launch_bounds__(256) void rt_gather_deinterleave_k(const float* __restrict__ gathered,
                                                                float* __restrict__ frame,
                                                                int row_floats, int height,
                                                                int world, int max_rows) {
  for (int y = blockIdx.y; y < height; y += gridDim.y) {  // grid y is capped at 65535 rows
    const float* src = gathered + ((size_t)(y % world) * max_rows + y / world) * row_floats;
    float* dst = frame + (size_t)y * row_floats;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < row_floats; i += gridDim.x * blockDim.x)
      dst[i] = src[i];
  }
}

}  // namespace

struct rt_gather_comm {
  ncclComm_t comm = nullptr;
  int world = 0, rank = 0, device = 0;
};

extern "C" {

const char* rt_gather_last_error(void) { return g_err.c_str(); }

int rt_gather_rows(int height, int world, int rank) {
  if (height < 0 || world <= 0 || rank < 0 || rank >= world) return 0;
  return rank < height ? (height - rank + world - 1) / world : 0;
}

int rt_gather_max_rows(int height, int world) {
  if (height <= 0 || world <= 0) return 0;
  return (height + world - 1) / world;
}

int rt_gather_unique_id(uint8_t id_out[RT_GATHER_ID_BYTES]) {
  if (!id_out) return fail(RT_ERR_INVALID_ARG, "null id");
  static_assert(sizeof(ncclUniqueId) == RT_GATHER_ID_BYTES, "RCCL unique id size");
  ncclUniqueId id;
  const ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) return fail(RT_ERR_HIP, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
  std::memcpy(id_out, &id, sizeof(id));
  return RT_OK;
}

int rt_gather_comm_create(const uint8_t id[RT_GATHER_ID_BYTES], int world, int rank, int device,
                          rt_gather_comm** out) {
  if (!id || !out || world <= 0 || rank < 0 || rank >= world)
    return fail(RT_ERR_INVALID_ARG, "bad id, world or rank");
  *out = nullptr;
  int prev = -1;
  (void)hipGetDevice(&prev);
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return fail(RT_ERR_HIP, std::string("hipSetDevice: ") + hipGetErrorString(e));
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  rt_gather_comm* c = new rt_gather_comm();
  c->world = world;
  c->rank = rank;
  c->device = device;
  const ncclResult_t r = ncclCommInitRank(&c->comm, world, uid, rank);
  if (prev >= 0) (void)hipSetDevice(prev);
  if (r != ncclSuccess) {
    delete c;
    return fail(RT_ERR_HIP, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
  }
  *out = c;
  return RT_OK;
}

void rt_gather_comm_destroy(rt_gather_comm* c) {
  if (!c) return;
  if (c->comm) (void)ncclCommDestroy(c->comm);
  delete c;
}

int rt_gather_deinterleave(const float* gathered, int world, int width, int height, float* frame,
                           void* hip_stream) {
  if (!gathered || !frame || world <= 0 || width <= 0 || height < 0)
    return fail(RT_ERR_INVALID_ARG, "bad gather arguments");
  if (height == 0) return RT_OK;
  const int row_floats = width * 3;
  const int gx = (row_floats + 255) / 256 < 64 ? (row_floats + 255) / 256 : 64;
  const int gy = height < 65535 ? height : 65535;
  hipLaunchKernelGGL(rt_gather_deinterleave_k, dim3((unsigned)gx, (unsigned)gy), dim3(256), 0,
                     (hipStream_t)hip_stream, gathered, frame, row_floats, height, world,
                     rt_gather_max_rows(height, world));
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(RT_ERR_HIP, std::string("deinterleave: ") + hipGetErrorString(e));
  return RT_OK;
}

int rt_gather_frame(rt_gather_comm* c, const float* local_rows, int width, int height,
                    float* scratch, float* frame, void* hip_stream) {
  if (!c || !local_rows || width <= 0 || height <= 0)
    return fail(RT_ERR_INVALID_ARG, "bad gather arguments");
  if (c->rank == 0 && (!scratch || !frame)) return fail(RT_ERR_INVALID_ARG, "rank 0 needs scratch and frame");
  int prev = -1;
  (void)hipGetDevice(&prev);
  hipError_t e = hipSetDevice(c->device);
  if (e != hipSuccess) return fail(RT_ERR_HIP, std::string("hipSetDevice: ") + hipGetErrorString(e));
  const size_t count = (size_t)rt_gather_max_rows(height, c->world) * width * 3;
  const ncclResult_t r = ncclGather(local_rows, c->rank == 0 ? scratch : nullptr, count, ncclFloat32, 0,
                                    c->comm, (hipStream_t)hip_stream);
  int rc = RT_OK;
  if (r != ncclSuccess) rc = fail(RT_ERR_HIP, std::string("ncclGather: ") + ncclGetErrorString(r));
  if (rc == RT_OK && c->rank == 0)
    rc = rt_gather_deinterleave(scratch, c->world, width, height, frame, hip_stream);
  if (prev >= 0) (void)hipSetDevice(prev);
  return rc;
}

}  // extern "C"
