/*
 * rt_gather.h — C ABI of `librtgather.so`: the framebuffer gather of a row-tiled render over
 * RCCL (xGMI), for a host that runs one process per GPU.
 *
 * The reference renders one frame per process over all cores (rayon, render.rs:153-197); across
 * the GPUs of a node the frame is dealt in cyclic rows (rank r renders rows r, r + N, ... with
 * rt_render_device) and this library brings the rows to rank 0 in ONE RCCL collective
 * (ncclGather, rccl.h:745) and de-interleaves them there. It is the C counterpart of bench.py's
 * torch.distributed gather (surely_rt/parallel.py), so a Rust (or C) host needs no RCCL binding of
 * its own. Separate from librtmi355x.so so that the render library does not depend on RCCL.
 *
 * Every entry point returns RT_OK (0) or a negative rt_mi355x.h status; rt_gather_last_error()
 * describes the last failure of the calling thread.
 */
#ifndef RT_GATHER_H
#define RT_GATHER_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_GATHER_ID_BYTES 128 /* NCCL_UNIQUE_ID_BYTES */

typedef struct rt_gather_comm rt_gather_comm; /* an RCCL communicator + its device */

const char* rt_gather_last_error(void);

/* Rank 0 creates the communicator's id (ncclGetUniqueId) and shares the bytes with every rank
 * over any channel (a file, MPI, torch.distributed, ...). */
int rt_gather_unique_id(uint8_t id_out[RT_GATHER_ID_BYTES]);

/* Every rank: join the communicator of `world` ranks as `rank`, on HIP device `device`
 * (ncclCommInitRank; collective, all ranks call it). */
int rt_gather_comm_create(const uint8_t id[RT_GATHER_ID_BYTES], int world, int rank, int device,
                          rt_gather_comm** out);
void rt_gather_comm_destroy(rt_gather_comm* comm);

/* Rows of `rank` under cyclic tiling of `height` rows over `world` ranks, and the padded count
 * every rank's buffer holds: ceil(height / world). */
int rt_gather_rows(int height, int world, int rank);
int rt_gather_max_rows(int height, int world);

/* Every rank (collective, asynchronous on hip_stream of its device): local_rows holds this
 * rank's rows (rt_render_device with row_begin = rank, row_step = world), padded to max_rows rows
 * of width * 3 floats. On rank 0, scratch (world * max_rows * width * 3 floats) receives every
 * rank's block and frame (height * width * 3 floats) the de-interleaved image; other ranks pass
 * NULL for both. Bit for bit the single-GPU frame (the RNG is keyed by global pixel and sample). */
int rt_gather_frame(rt_gather_comm* comm, const float* local_rows, int width, int height,
                    float* scratch, float* frame, void* hip_stream);

/* The de-interleave step alone (no RCCL; rank 0's half of rt_gather_frame, and a test of the row
 * layout with several shares on one GPU): gathered = world blocks of max_rows rows. */
int rt_gather_deinterleave(const float* gathered, int world, int width, int height, float* frame,
                           void* hip_stream);

#ifdef __cplusplus
}
#endif
#endif /* RT_GATHER_H */
