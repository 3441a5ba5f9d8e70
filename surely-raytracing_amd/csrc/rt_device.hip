// rt_device.hip — gfx950 path-tracing kernels + the C ABI of include/rt_mi355x.h.
//
// Replaces the reference's per-pixel render loop (render.rs:144-216) and everything it calls:
// get_ray (render.rs:218-249), ray_color (render.rs:251-311), HittableList/BvhNode::hit
// (hittable.rs:88-109, 216-236), Quad/Sphere/Aabb::hit (object.rs:145-184, 340-370, 453-490),
// Translate/RotateY::hit (transform.rs:57-135), ConstantMedium::hit (constant_medium.rs:41-95),
// Material scatter (material.rs:92-248), PDFs (pdf.rs:44-127), Onb (onb.rs:24-47), textures
// and Perlin noise (texture.rs:17-131, perlin.rs:30-96), vec3 math (vec3.rs).
//
// Work decomposition: persistent waves claim POOLS from a global queue; a pool
// is one 8x8 pixel tile x one stratum row s_j (x one block of kPoolSi stratum columns s_i for
// segment and tail pools). Each lane traces one path at a time (ray_color's recursion -> an
// iterative bounce loop with beta/L) and takes a row item (all of one pixel's samples of the
// row, summed per block and then per row in f64 in LDS), a segment item (one block) or, for the
// launch's last pools, one sample; when its item ends it writes the f64 value and claims the
// next item with a wave ballot + mbcnt, so lanes stay busy whatever the per-pixel path cost.
// rt_reduce forms each row's total from block partials where a lane did not, and adds the rows
// in the reference's sample order (s_i inside s_j, render.rs:185-189; the association differs
// from its single running sum only between blocks and between rows) into the caller's
// accumulator, so no atomics touch the framebuffer and results are bitwise reproducible and
// identical across 1..8 GPUs and any split of the work (the RNG is keyed by global pixel and
// sample).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "rt_mi355x.h"
#include "rt_flatten.hpp"
#include "rt_jit.hpp"
#include "rt_kernel.h"
#include "rt_layout.h"

using namespace rtk;

namespace {

// Ahead-of-time kernels: the interpreter traversal, one per feature combination.
template <bool COUNT, bool VOL, bool TEX, bool BVH, bool STAGED, bool VOLB = VOL,
          bool VOLI = true, int VN = 0>
__global__ __launch_bounds__(BlockOf<BVH>::value, (MinWaves<VOL, TEX, BVH>::value)) void rt_trace(
    TraceParams P) {
  trace_body<COUNT, VOL, TEX, BVH, STAGED, VOLB, VOLI, TravInterpN<VN>>(P);
}

// Per pixel, in the reference's sample order (s_j, then s_i: render.rs:185-189): for each
// stratum row s_j its total R = ((p_0 + p_1) + p_2) + ... over the block partials p_b (a row
// item's R as the lane formed it; a segment pair's from its block partials; a tail pair's from
// the sequential sums of its blocks' samples: the same running sums, bit for bit), added into
// one running total. The reference adds every sample into that total; here a block's samples are
// summed first and a row's blocks next, so the association differs from the reference's only
// between blocks and between rows, and it does not depend on how the launch split its pairs into
// row, segment and tail items. One wave per 8x8 tile, lane = pixel of the tile: each load
// instruction reads 64 * 8 contiguous bytes. Chunked calls carry the running total in `tot`.
// mode: bit0 first chunk, bit1 last chunk (write accum), bit2 overwrite.
constexpr int kRedU = 8;  // values loaded ahead per step of rt_reduce
__global__ __launch_bounds__(256) void rt_reduce(const double* __restrict__ part,
                                                 double* __restrict__ tot,
                                                 float* __restrict__ accum, int W, int n_rows,
                                                 int tiles_x, int n_tiles, int n_sj, int S,
                                                 int n_pairs_r, int n_pairs_a, int mode) {
  const int tile_id = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  const int pv = threadIdx.x & 63;
  if (tile_id >= n_tiles) return;
  const int tx = tile_id % tiles_x, ty = tile_id / tiles_x;
  const int tile_w = min(kWaveTile, W - tx * kWaveTile);
  const int tile_h = min(kWaveTile, n_rows - ty * kWaveTile);
  if (pv >= tile_w * tile_h) return;
  const int x = tx * kWaveTile + pv % tile_w, kr = ty * kWaveTile + pv / tile_w;
  const size_t i = (size_t)kr * W + x;
  const int n_blk = (S + kPoolSi - 1) / kPoolSi;
  double t0 = 0.0, t1 = 0.0, t2 = 0.0;
  if (!(mode & 1)) {
    t0 = tot[3 * i];
    t1 = tot[3 * i + 1];
    t2 = tot[3 * i + 2];
  }
  const int q0 = tile_id * n_sj;  // this tile's pairs q0 .. q0 + n_sj - 1 (s_j order)
  const int k_r = max(0, min(n_sj, n_pairs_r - q0)), k_a = max(0, min(n_sj, n_pairs_a - q0));
  int k = 0;
  // row pairs: one total each, 64 values apart; loads first, then the in-order adds (a share's
  // few waves are otherwise bound by one load's latency per value)
  {
    const double* r = part + ((size_t)q0 * 64 + pv) * 3;
    for (; k + kRedU <= k_r; k += kRedU) {
      double v[kRedU][3];
#pragma unroll
      for (int u = 0; u < kRedU; ++u) {
        const double* e = r + (size_t)(k + u) * 192;
        v[u][0] = e[0], v[u][1] = e[1], v[u][2] = e[2];
      }
#pragma unroll
      for (int u = 0; u < kRedU; ++u) t0 += v[u][0], t1 += v[u][1], t2 += v[u][2];
    }
    for (; k < k_r; ++k) {
      const double* e = r + (size_t)k * 192;
      t0 += e[0], t1 += e[1], t2 += e[2];
    }
  }
  // segment pairs: the row total of n_blk block partials
  for (; k < k_a; ++k) {
    const int q = q0 + k;
    const double* r =
        part + (((size_t)n_pairs_r + (size_t)(q - n_pairs_r) * n_blk) * 64 + pv) * 3;
    double r0 = r[0], r1 = r[1], r2 = r[2];
    int b = 1;
    for (; b + kRedU <= n_blk; b += kRedU) {
      double v[kRedU][3];
#pragma unroll
      for (int u = 0; u < kRedU; ++u) {
        const double* e = r + (size_t)(b + u) * 192;
        v[u][0] = e[0], v[u][1] = e[1], v[u][2] = e[2];
      }
#pragma unroll
      for (int u = 0; u < kRedU; ++u) r0 += v[u][0], r1 += v[u][1], r2 += v[u][2];
    }
    for (; b < n_blk; ++b) {
      const double* e = r + (size_t)b * 192;
      r0 += e[0], r1 += e[1], r2 += e[2];
    }
    t0 += r0, t1 += r1, t2 += r2;
  }
  // tail pairs: per-sample values, summed per block of kPoolSi samples, then the blocks
  const size_t tail0 = (size_t)n_pairs_r + (size_t)(n_pairs_a - n_pairs_r) * n_blk;
  for (; k < n_sj; ++k) {
    const int q = q0 + k;
    const double* rt = part + ((tail0 + (size_t)(q - n_pairs_a) * S) * 64 + pv) * 3;
    double R0 = 0.0, R1 = 0.0, R2 = 0.0;
    for (int s0 = 0; s0 < S; s0 += kPoolSi) {
      const int n = min(kPoolSi, S - s0);
      double v[kPoolSi][3];
#pragma unroll
      for (int u = 0; u < kPoolSi; ++u) {
        if (u < n) {
          const double* e = rt + (size_t)(s0 + u) * 192;
          v[u][0] = e[0], v[u][1] = e[1], v[u][2] = e[2];
        }
      }
      double r0 = 0.0, r1 = 0.0, r2 = 0.0;
#pragma unroll
      for (int u = 0; u < kPoolSi; ++u)
        if (u < n) r0 += v[u][0], r1 += v[u][1], r2 += v[u][2];
      if (s0 == 0) {
        R0 = r0, R1 = r1, R2 = r2;
      } else {
        R0 += r0, R1 += r1, R2 += r2;
      }
    }
    t0 += R0, t1 += R1, t2 += R2;
  }
  float* a = accum + 3 * i;
  if (mode & 2) {
    if (mode & 4) {
      a[0] = (float)t0, a[1] = (float)t1, a[2] = (float)t2;
    } else {
      a[0] = (float)((double)a[0] + t0), a[1] = (float)((double)a[1] + t1);
      a[2] = (float)((double)a[2] + t2);
    }
  } else {
    tot[3 * i] = t0, tot[3 * i + 1] = t1, tot[3 * i + 2] = t2;
  }
}

// rt_multi_render's gather on the first device: device k's compact rows (its cyclic share of
// the call's rows, k, k + G, ...) arrive in `stage` at row offset row0[k]; each row goes to row
// k + j * G of the frame, overwritten or added (the caller's accumulator, render.rs:189).
// to_frame = 0: the reverse (the caller's accumulator rows into the staging area, so that every
// device accumulates into its own rows exactly as rt_render_device does, render.rs:189).
__global__ __launch_bounds__(256) void rt_deinterleave(float* __restrict__ stage,
                                                       float* __restrict__ frame, int row_floats,
                                                       int n_rows, int G, int to_frame) {
  const int kr = blockIdx.y;  // row of the frame
  if (kr >= n_rows) return;
  const int k = kr % G, j = kr / G;
  // device k's rows start at sum_{k' < k} rows(k'), rows(k') = ceil((n_rows - k') / G)
  int row0 = 0;
  for (int q = 0; q < k; ++q) row0 += (n_rows - q + G - 1) / G;
  float* st = stage + (size_t)(row0 + j) * row_floats;
  float* fr = frame + (size_t)kr * row_floats;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < row_floats; i += gridDim.x * blockDim.x) {
    if (to_frame)
      fr[i] = st[i];
    else
      st[i] = fr[i];
  }
}

// ---------------------------------------------------------------- host side
thread_local std::string g_err;

int set_err(int code, const std::string& m) {
  g_err = m;
  return code;
}

#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                               \
      return set_err(RT_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));    \
  } while (0)

// The path kernel's LDS for one render (rt_trace's prologue stages these regions, in this order,
// from byte 0 of the dynamic LDS): the small tables or the Perlin tables (stage), then either the
// compact ordered BVHs and the LDS walk's per-lane stacks (cbvh_walk_t: lane l's slot k at
// stack_off + 4 (l + k block), header cbvh_stack = 4 x the deepest tree's depth bytes per lane),
// or as much of the reference BVH region as fits. One function for the render and for the host
// check of the plan (rt_scene_lds_check), so the two cannot drift apart.
struct LdsPlan {
  int block = 0;
  size_t static_lds = 0;  // the kernel's static LDS (per-lane f64 sums, ...), an upper bound
  uint32_t stage_scene = 0, stage_bytes = 0, n_perlin_lds = 0;
  uint32_t cbvh_lds_off = ~0u, stack_lds_off = 0, cbvh_bytes = 0;
  size_t cbvh_lds = 0;  // bytes of the trees and stacks
  uint32_t bvh_lds_words = 0, bvh_lds_off = 0;
  uint32_t row_lds_off = ~0u;  // BVH kernels: the row items' row totals (~0u: no row items)
  size_t lds_bytes = 0;  // dynamic LDS of the launch
};
LdsPlan plan_lds(const rtl_scene_header& hdr, uint32_t o_perl, uint32_t flags, bool want_jit,
                 size_t lds_module_max) {
  LdsPlan L;
  const bool count = (flags & RT_FLAG_COUNT_OPS) != 0;
  const bool bvh = hdr.has_bvh != 0;
  L.block = bvh ? kBlockBvh : kBlock;
  // static LDS of the path kernel: the per-lane f64 running sums (trace_body sh_acc; non-BVH
  // kernels also the row totals sh_row and the bounce's throughput factor and ending radiance,
  // sh_f / sh_le), the op counters, slack for the profiling build
  L.static_lds = (size_t)L.block * (bvh ? 24 : 96) + 512 + (count ? 128 : 0);
#ifdef RT_PROF
  L.static_lds += 4096;  // the profiling build's counters (tools_gpu/prof_*.py)
#endif
  // a scene whose tables up to the Perlin block fit kStageScene bytes is copied whole (per-lane
  // reads then never leave the CU); otherwise only its first Perlin tables
  const uint32_t used_perlins = hdr.has_textures ? hdr.n_perlins : 0u;
  const size_t scene_prefix = o_perl + (size_t)used_perlins * RTL_PERLIN_BYTES;
  L.stage_scene = scene_prefix <= kStageScene ? 1u : 0u;
  if (L.stage_scene) {
    L.n_perlin_lds = used_perlins;
    L.stage_bytes = (uint32_t)((scene_prefix + 15) & ~(size_t)15);
  } else {
    L.n_perlin_lds = std::min<uint32_t>(used_perlins, kPerlinLds);
    L.stage_bytes = L.n_perlin_lds * RTL_PERLIN_BYTES;
  }
  const size_t cap = (want_jit ? lds_module_max : kLdsTotal) - L.static_lds;
  L.cbvh_bytes = hdr.cbvh_words * 4u;
  const size_t need = (size_t)L.stage_bytes + L.cbvh_bytes + (size_t)hdr.cbvh_stack * L.block;
  if (bvh && !count && L.cbvh_bytes && !(flags & RT_FLAG_REFERENCE_BVH) &&
      !std::getenv("RT_NO_CBVH_LDS") && need <= cap) {
    L.cbvh_lds_off = L.stage_bytes;
    L.stack_lds_off = L.stage_bytes + L.cbvh_bytes;
    L.cbvh_lds = need - L.stage_bytes;
  }
  if (L.stage_scene) {
    L.bvh_lds_words = hdr.bvh_words;
  } else if (bvh && L.cbvh_lds_off == ~0u) {
    const size_t room = cap > L.stage_bytes ? cap - L.stage_bytes : 0;
    L.bvh_lds_words = (uint32_t)std::min<size_t>(hdr.bvh_words, room / 64 * 16);
    L.bvh_lds_off = L.stage_bytes;
  }
  L.lds_bytes = L.stage_bytes + (L.stage_scene ? 0u : (size_t)L.bvh_lds_words * 4u) + L.cbvh_lds;
  // BVH product kernels with the compact trees in LDS: the row items' per-lane row totals after
  // them when they fit (C4: 124 + 18 KB dynamic, 18 KB static), so that a whole frame keeps one
  // f64 value per (pixel, s_j) instead of one per block of kPoolSi samples
  const size_t row_bytes = (size_t)L.block * 3 * sizeof(double);
  if (bvh && L.cbvh_lds_off != ~0u && !std::getenv("RT_NO_BVH_ROWS") &&
      L.lds_bytes + row_bytes <= cap) {
    L.row_lds_off = (uint32_t)L.lds_bytes;
    L.lds_bytes += row_bytes;
  }
  return L;
}

// Byte offsets of the scene's tables in its one device allocation (rt_scene_create): nodes,
// materials, textures, lights, light offsets, Perlin tables, 16-byte aligned; texels last.
struct TableLayout {
  size_t o_nodes = 0, o_mats = 0, o_texs = 0, o_lig = 0, o_loff = 0, o_perl = 0, o_tx = 0, total = 0;
};
TableLayout table_layout(const rtf::FlatScene& F) {
  auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
  TableLayout T;
  // +256 B: the LANE walker fetches 64 bytes of every node it visits (END, 16 B, included) and
  // prefetches one quad record past a batch
  T.o_mats = al(T.o_nodes + F.nodes.size() * 4 + 256);
  T.o_texs = al(T.o_mats + F.mats.size() * 4);
  T.o_lig = al(T.o_texs + F.texs.size() * 4);
  T.o_loff = al(T.o_lig + F.lights.size() * 4);
  T.o_perl = al(T.o_loff + F.light_offs.size() * 4);
  T.o_tx = al(T.o_perl + F.perlin.size());
  T.total = al(T.o_tx + F.texels.size()) + 256;
  return T;
}

}  // namespace

// The per-render state of a scene: the f64 workspace, the pool-queue word and op counters, the
// stats events and a completion event. A render takes a slot that no render still uses (its done
// event has fired) or one whose last render went to the same stream (stream order then protects
// it); otherwise a new slot is made (up to kMaxSlots), so renders of one scene on different
// streams or host threads run concurrently on their own queue words and workspaces.
struct RenderSlot {
  uint8_t* work = nullptr;  // row totals / segment partials / tail samples + f64 running sums
  size_t work_bytes = 0;
  unsigned long long* ops = nullptr;  // 32 op counters, the pool-queue word (32), profiling (40..)
  unsigned int* queue = nullptr;
  hipEvent_t done = nullptr;  // recorded after the render's last kernel
  hipEvent_t ev0 = nullptr, ev1 = nullptr;  // rt_stats::ms_kernel
  hipStream_t last_stream = nullptr;
  bool recorded = false;  // `done` has been recorded at least once
  bool held = false;      // a render call is between acquire and release
};

struct rt_scene {
  int device = 0;
  rtl_scene_header hdr{};
  uint8_t* dev = nullptr;  // one allocation for all tables
  uint64_t dev_bytes = 0;
  const uint32_t *nodes = nullptr, *mats = nullptr, *texs = nullptr, *lights = nullptr,
                 *light_offs = nullptr;
  const uint8_t *perlin = nullptr, *texels = nullptr;
  uint32_t o_mats = 0, o_texs = 0, o_lights = 0, o_loffs = 0, o_perl = 0;  // byte offsets in dev
  int sphere_light0 = -1;  // first SPHERE light record (TraceParams::sphere_light0)
  static constexpr int kMaxSlots = 8;
  std::vector<std::unique_ptr<RenderSlot>> slots;  // grown on demand (RenderSlot)
  int last_slot = -1;                              // the slot of the latest render
  std::condition_variable slot_cv;                 // a held slot was released
  int n_cu = 0;                 // compute units of the device
  size_t mem_total = (size_t)8 << 30;  // device memory (hipMemGetInfo at creation)
  size_t lds_module_max = 64u << 10;  // LDS a module (hiprtc) launch may take (device limit)
  int resident_blocks[48] = {}; // per kernel variant: blocks resident per CU (0 = not queried)
  size_t resident_lds[48] = {};  // ... at this dynamic LDS size
  // scene-specialised product kernel (rt_jit.cpp): the generated world walker, compiled on the
  // first product render. jit_state: 0 = not compiled yet, 1 = compiled, -1 = scene not
  // generated (jit_msg says why), -2 = compile failed (jit_msg = log; the interpreter runs)
  std::string jit_walker, jit_msg;
  int jit_state = -1;
  rtj::Kernel jit_k[4];  // [tex][staged]
  // rt_trace launch timing: one event pair per launch, ring of kTraceRing, tagged by render id
  static constexpr int kTraceRing = 4 * RT_TRACE_HISTORY;
  hipEvent_t tev[kTraceRing][2] = {};
  uint64_t tev_render[kTraceRing] = {};
  uint64_t n_tev = 0, n_render = 0;
  std::mutex mu;
};

extern "C" {

int rt_abi_version(void) { return RT_ABI_VERSION; }
const char* rt_last_error(void) { return g_err.c_str(); }

int rt_device_count(int* count) {
  if (!count) return set_err(RT_ERR_INVALID_ARG, "null count");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) n = 0;
  *count = n;
  return RT_OK;
}

int rt_scene_validate(const rt_scene_blob* blob) {
  rtf::FlatScene F;
  std::string err;
  int rc = rtf::flatten(blob, &F, &err);
  if (rc != RT_OK) return set_err(rc, err);
  return RT_OK;
}

int rt_scene_layout_stats(const rt_scene_blob* blob, uint32_t* out, int n) {
  if (!out || n < 0) return set_err(RT_ERR_INVALID_ARG, "null out");
  rtf::FlatScene F;
  std::string err;
  int rc = rtf::flatten(blob, &F, &err);
  if (rc != RT_OK) return set_err(rc, err);
  uint32_t v[RT_LAYOUT_STATS] = {(uint32_t)F.nodes.size(), F.hdr.bvh_words, 0, 0, 0, 0, 0,
                                 F.hdr.n_lights, 0, 0, F.hdr.cbvh_words * 4u};
  for (size_t p = 0; p < F.hdr.n_rec_words; p += rtf::record_words(F.nodes[p])) {
    const uint32_t h = F.nodes[p], ty = h & 0xffu;
    if (ty == RTL_BVH) ++v[2];
    if (ty == RTL_BVH && F.nodes[p + 3] != 0u) {
      ++v[8];
      if (F.nodes[F.nodes[p + 3] + 1] != 0xffffffffu) ++v[9];
    }
    if (ty == RTL_DUP) ++v[3];
    if (ty == RTL_VOLUME) {
      ++v[4];
      if (h & RTL_VOLF_SPHERE) ++v[5];
      if (h & RTL_VOLF_QUADS) ++v[6];
    }
  }
  for (int k = 0; k < n && k < RT_LAYOUT_STATS; ++k) out[k] = v[k];
  return RT_OK;
}

int rt_scene_lds_check(const rt_scene_blob* blob, uint32_t flags, uint32_t n_rays, uint64_t seed,
                       uint64_t* out, int n, char* msg, uint32_t msg_len) {
  if (!out || n < 0) return set_err(RT_ERR_INVALID_ARG, "null out");
  rtf::FlatScene F;
  std::string err;
  const int rc = rtf::flatten(blob, &F, &err);
  if (rc != RT_OK) return set_err(rc, err);
  const TableLayout TL = table_layout(F);
  // the product kernel's plan on a device whose workgroups may take the CU's whole LDS
  const LdsPlan L = plan_lds(F.hdr, (uint32_t)TL.o_perl, flags, true, kLdsTotal);
  const rtf::WalkCheck W = rtf::check_compact_trees(F.nodes, F.hdr, n_rays, seed);
  const uint64_t v[RT_LDS_CHECK] = {
      (uint64_t)L.block, L.static_lds, L.stage_bytes, L.cbvh_lds_off, L.cbvh_bytes, L.stack_lds_off,
      F.hdr.cbvh_stack, L.lds_bytes, L.static_lds + L.lds_bytes, kLdsTotal, W.trees, W.max_depth,
      W.errors, W.max_store_slot, W.max_live, W.rays, W.steps, W.max_read, L.row_lds_off};
  for (int k = 0; k < n && k < RT_LDS_CHECK; ++k) out[k] = v[k];
  if (msg && msg_len) {
    std::strncpy(msg, W.first_error.c_str(), msg_len - 1);
    msg[msg_len - 1] = '\0';
  }
  return RT_OK;
}

int rt_scene_create(const rt_scene_blob* blob, int device, rt_scene** out) {
  if (!out) return set_err(RT_ERR_INVALID_ARG, "null out");
  *out = nullptr;
  rtf::FlatScene F;
  std::string err;
  int rc = rtf::flatten(blob, &F, &err);
  if (rc != RT_OK) return set_err(rc, err);
  {
    // The LDS walk (rt_kernel.h cbvh_walk_t) trusts the compact trees: its only global loads are
    // the leaf records it reaches through their references, and its stack stores are bounded by
    // the header's cbvh_stack. Every tree is checked before upload (structure, references, leaf
    // records, depth; no ray walks): a malformed tree is refused here, not met on the device.
    const rtf::WalkCheck W = rtf::check_compact_trees(F.nodes, F.hdr, 0, 0);
    if (W.errors) return set_err(RT_ERR_BAD_BLOB, "compact BVH check: " + W.first_error);
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return set_err(RT_ERR_NO_DEVICE, "no HIP device available");
  if (device < 0 || device >= ndev) return set_err(RT_ERR_INVALID_ARG, "bad device ordinal");
  HIP_TRY(hipSetDevice(device));
  // Pack the tables into one allocation, in the order the kernel stages them into LDS (a
  // prefix of it: nodes, materials, textures, lights, light offsets, Perlin tables), 16-byte
  // aligned; texels last (never staged).
  const TableLayout TL = table_layout(F);
  const size_t o_nodes = TL.o_nodes, s_nodes = F.nodes.size() * 4;
  const size_t o_mats = TL.o_mats, s_mats = F.mats.size() * 4;
  const size_t o_texs = TL.o_texs, s_texs = F.texs.size() * 4;
  const size_t o_lig = TL.o_lig, s_lig = F.lights.size() * 4;
  const size_t o_loff = TL.o_loff, s_loff = F.light_offs.size() * 4;
  const size_t o_perl = TL.o_perl, s_perl = F.perlin.size();
  const size_t o_tx = TL.o_tx, s_tx = F.texels.size();
  const size_t total = TL.total;
  std::vector<uint8_t> host(total, 0);
  auto cp = [&](size_t off, const void* src, size_t n) {
    if (n) std::memcpy(host.data() + off, src, n);
  };
  cp(o_nodes, F.nodes.data(), s_nodes);
  cp(o_mats, F.mats.data(), s_mats);
  cp(o_texs, F.texs.data(), s_texs);
  cp(o_perl, F.perlin.data(), s_perl);
  cp(o_lig, F.lights.data(), s_lig);
  cp(o_loff, F.light_offs.data(), s_loff);
  cp(o_tx, F.texels.data(), s_tx);
  rt_scene* sc = new rt_scene();
  sc->device = device;
  sc->hdr = F.hdr;
  hipError_t e = hipMalloc(&sc->dev, total);
  if (e == hipSuccess) e = hipMemcpy(sc->dev, host.data(), total, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&sc->n_cu, hipDeviceAttributeMultiprocessorCount,
                                                 device);
  int lds_block = 0;
  if (e == hipSuccess)
    e = hipDeviceGetAttribute(&lds_block, hipDeviceAttributeMaxSharedMemoryPerBlock, device);
  if (e == hipSuccess && lds_block > 0)
    sc->lds_module_max = std::min<size_t>((size_t)lds_block, kLdsTotal);
  if (e == hipSuccess) {
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess && tot > 0) sc->mem_total = tot;
  }
  for (int k = 0; k < rt_scene::kTraceRing && e == hipSuccess; ++k) {
    e = hipEventCreate(&sc->tev[k][0]);
    if (e == hipSuccess) e = hipEventCreate(&sc->tev[k][1]);
  }
  if (e != hipSuccess) {
    rt_scene_destroy(sc);
    return set_err(RT_ERR_HIP, std::string("scene upload: ") + hipGetErrorString(e));
  }
  sc->dev_bytes = total;
  sc->nodes = (const uint32_t*)(sc->dev + o_nodes);
  sc->mats = (const uint32_t*)(sc->dev + o_mats);
  sc->texs = (const uint32_t*)(sc->dev + o_texs);
  sc->perlin = sc->dev + o_perl;
  sc->lights = (const uint32_t*)(sc->dev + o_lig);
  sc->light_offs = (const uint32_t*)(sc->dev + o_loff);
  sc->texels = sc->dev + o_tx;
  sc->o_mats = (uint32_t)o_mats;
  sc->o_texs = (uint32_t)o_texs;
  sc->o_lights = (uint32_t)o_lig;
  sc->o_loffs = (uint32_t)o_loff;
  sc->o_perl = (uint32_t)o_perl;
  const char* jit_env = std::getenv("RT_JIT");
  if (jit_env && std::strcmp(jit_env, "0") == 0) {
    sc->jit_msg = "disabled by RT_JIT=0";
  } else {
    sc->jit_walker = rtj::generate(F, &sc->jit_msg);
    sc->jit_state = sc->jit_walker.empty() ? -1 : 0;
  }
  sc->sphere_light0 = -1;
  for (size_t i = 0; i < F.light_offs.size(); ++i)
    if ((F.lights[F.light_offs[i]] & 0xffu) == RTL_SPHERE) {
      sc->sphere_light0 = (int)i;
      break;
    }
  *out = sc;
  return RT_OK;
}

void rt_scene_destroy(rt_scene* sc) {
  if (!sc) return;
  int prev = -1;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(sc->device);
  // renders are asynchronous on the caller's streams (rt_render_device): wait for them before
  // the module cache may unload this scene's kernel code object (release_kernel evicts idle
  // modules) and before the tables and workspace are freed
  (void)hipDeviceSynchronize();
  for (const rtj::Kernel& k : sc->jit_k) rtj::release_kernel(k);  // the module cache's holds
  if (sc->dev) (void)hipFree(sc->dev);
  for (const auto& sl : sc->slots) {
    if (sl->work) (void)hipFree(sl->work);
    if (sl->ops) (void)hipFree(sl->ops);
    if (sl->done) (void)hipEventDestroy(sl->done);
    if (sl->ev0) (void)hipEventDestroy(sl->ev0);
    if (sl->ev1) (void)hipEventDestroy(sl->ev1);
  }
  for (int k = 0; k < rt_scene::kTraceRing; ++k)
    for (int j = 0; j < 2; ++j)
      if (sc->tev[k][j]) (void)hipEventDestroy(sc->tev[k][j]);
  delete sc;
  if (prev >= 0) (void)hipSetDevice(prev);
}

uint64_t rt_scene_device_bytes(const rt_scene* sc) { return sc ? sc->dev_bytes : 0; }

int rt_jit_check(const rt_scene_blob* blob, const char* arch, int* state, char* msg,
                 uint32_t msg_len) {
  if (!blob || !arch || !state) return set_err(RT_ERR_INVALID_ARG, "null argument");
  rtf::FlatScene F;
  std::string err;
  int rc = rtf::flatten(blob, &F, &err);
  if (rc != RT_OK) return set_err(rc, err);
  std::string why, out;
  const std::string walker = rtj::generate(F, &why);
  *state = walker.empty() ? -1 : 1;
  out = walker.empty() ? why : walker;
  if (!walker.empty()) {
    std::vector<char> code;
    std::string log;
    rc = rtj::compile(rtj::kernel_source(walker, rtj::product_flags(F, true)), arch, &code, &log);
    if (rc != 0) {
      *state = -2;
      out = log;
    }
  }
  if (msg && msg_len) {
    std::strncpy(msg, out.c_str(), msg_len - 1);
    msg[msg_len - 1] = '\0';
  }
  return *state == -2 ? set_err(RT_ERR_HIP, out) : RT_OK;
}

int rt_scene_jit_info(rt_scene* sc, int* state, char* msg, uint32_t msg_len) {
  if (!sc || !state) return set_err(RT_ERR_INVALID_ARG, "null argument");
  std::lock_guard<std::mutex> lock(sc->mu);
  *state = sc->jit_state;
  if (msg && msg_len) {
    std::strncpy(msg, sc->jit_msg.c_str(), msg_len - 1);
    msg[msg_len - 1] = '\0';
  }
  return RT_OK;
}

// A slot for a render on `stream` (RenderSlot), with sc->mu held through `lock`: a free one (its
// last render has finished, or went to the same stream handle), else a new one, else wait for a
// release. A reused slot's `done` event is always waited for on `stream` (hipStreamWaitEvent):
// equal handles are not the same stream everywhere (hipStreamPerThread, the per-thread default
// stream), so stream order alone cannot be trusted; on the same stream the wait costs nothing.
static int acquire_slot(rt_scene* sc, std::unique_lock<std::mutex>& lock, hipStream_t stream,
                        RenderSlot** out) {
  for (;;) {
    RenderSlot* pick = nullptr;
    for (const auto& sl : sc->slots) {
      if (sl->held) continue;
      if (sl->recorded && sl->last_stream == stream) {  // stream order: no wait needed
        pick = sl.get();
        break;
      }
      if (!pick) {
        const hipError_t q = sl->recorded ? hipEventQuery(sl->done) : hipSuccess;
        if (q == hipSuccess) pick = sl.get();
        else if (q != hipErrorNotReady) return set_err(RT_ERR_HIP, std::string("slot event: ") + hipGetErrorString(q));
      }
    }
    if (!pick && (int)sc->slots.size() < rt_scene::kMaxSlots) {
      std::unique_ptr<RenderSlot> sl(new RenderSlot());
      hipError_t e = hipMalloc(&sl->ops, sizeof(unsigned long long) * 64 + 256);
      if (e == hipSuccess) e = hipEventCreateWithFlags(&sl->done, hipEventDisableTiming);
      if (e == hipSuccess) e = hipEventCreate(&sl->ev0);
      if (e == hipSuccess) e = hipEventCreate(&sl->ev1);
      if (e != hipSuccess) {
        if (sl->ops) (void)hipFree(sl->ops);
        if (sl->done) (void)hipEventDestroy(sl->done);
        if (sl->ev0) (void)hipEventDestroy(sl->ev0);
        if (sl->ev1) (void)hipEventDestroy(sl->ev1);
        return set_err(RT_ERR_HIP, std::string("render slot: ") + hipGetErrorString(e));
      }
      sl->queue = (unsigned int*)(sl->ops + 32);
      sc->slots.push_back(std::move(sl));
      pick = sc->slots.back().get();
    }
    if (!pick) {  // every slot busy: wait for the oldest unheld one, or for a release
      for (const auto& sl : sc->slots)
        if (!sl->held) {
          pick = sl.get();
          break;
        }
      if (pick) {
        HIP_TRY(hipEventSynchronize(pick->done));
      } else {
        sc->slot_cv.wait(lock);
        continue;
      }
    }
    if (pick->recorded) HIP_TRY(hipStreamWaitEvent(stream, pick->done, 0));
    pick->held = true;
    sc->last_slot = (int)(std::find_if(sc->slots.begin(), sc->slots.end(),
                                       [&](const std::unique_ptr<RenderSlot>& u) {
                                         return u.get() == pick;
                                       }) - sc->slots.begin());
    *out = pick;
    return RT_OK;
  }
}

// Releases a held slot on every exit path of a render call. Once the call has enqueued work on
// `stream` (enqueued), a call that fails half way still records the slot's `done` event after
// that work: the next render to take the slot then waits for the kernels that may still use its
// workspace and queue word, instead of for the previous render's event.
struct SlotHold {
  rt_scene* sc;
  std::unique_lock<std::mutex>& lock;
  RenderSlot* sl = nullptr;
  hipStream_t stream = nullptr;
  bool enqueued = false;   // work of this call is on `stream`
  bool finished = false;   // `done` was recorded after all of it
  ~SlotHold() {
    if (!sl) return;
    if (!lock.owns_lock()) lock.lock();
    if (enqueued && !finished) {
      if (hipEventRecord(sl->done, stream) == hipSuccess) {
        sl->recorded = true;
        sl->last_stream = stream;
      } else {
        (void)hipStreamSynchronize(stream);  // no event: drain the stream before the slot is reused
      }
    }
    sl->held = false;
    sc->slot_cv.notify_all();
  }
};

static int render_device_rows(rt_scene* sc, const rt_camera* cam, const rt_render_opts* opts,
                              float* accum, void* stream_v, rt_stats* stats) {
  auto t0 = std::chrono::steady_clock::now();
  if (!sc || !cam || !opts || !accum) return set_err(RT_ERR_INVALID_ARG, "null argument");
  const int W = cam->image_width, S = cam->sqrt_spp;
  if (W <= 0 || cam->image_height <= 0 || S <= 0 || cam->max_depth < 0 ||
      cam->max_depth > 0xffffff || opts->n_rows < 0 ||
      opts->row_step <= 0 || opts->row_begin < 0)
    return set_err(RT_ERR_INVALID_ARG, "bad camera or row range");
  if (opts->n_rows > 0 &&
      (int64_t)opts->row_begin + (int64_t)(opts->n_rows - 1) * opts->row_step >= cam->image_height)
    return set_err(RT_ERR_INVALID_ARG, "row range outside the image");
  if ((int64_t)W * cam->image_height >= (1ll << 32) || (int64_t)S * S >= (1ll << 32))
    return set_err(RT_ERR_UNSUPPORTED, "image or spp too large for 32-bit pixel/sample keys");
  // lane item keys pack x (16 bits), the call's row index (15 bits), s_j (15 bits, beside the
  // row-item bit) and s_i (16 bits)
  if (W > 65535 || opts->n_rows > 32767)
    return set_err(RT_ERR_UNSUPPORTED, "image_width > 65535 or n_rows > 32767 in one call");
  if (S > 32768) return set_err(RT_ERR_UNSUPPORTED, "spp > 2^30 (sqrt_spp > 32768)");
  const int sj0 = opts->sj_count > 0 ? opts->sj_begin : 0;
  const int n_sj = opts->sj_count > 0 ? opts->sj_count : S;
  if (sj0 < 0 || sj0 + n_sj > S) return set_err(RT_ERR_INVALID_ARG, "bad stratum range");
  if (sc->hdr.n_lights == 0 && (opts->flags & RT_FLAG_SEMANTICS_REFERENCE) && sc->hdr.pdf_materials)
    return set_err(RT_ERR_EMPTY_LIGHTS,
                   "empty light list with a diffuse/volume material: the reference panics "
                   "(hittable.rs:115-129)");
  std::unique_lock<std::mutex> lock(sc->mu);
  hipStream_t stream = (hipStream_t)stream_v;
  HIP_TRY(hipSetDevice(sc->device));
  if (stats) std::memset(stats, 0, sizeof(*stats));
  const size_t n_px = (size_t)opts->n_rows * W;
  if (n_px == 0) return RT_OK;
  SlotHold hold{sc, lock};
  {
    const int rc = acquire_slot(sc, lock, stream, &hold.sl);
    if (rc != RT_OK) return rc;
  }
  RenderSlot* const sl = hold.sl;
  TraceParams P;
  std::memset(&P, 0, sizeof(P));
  P.nodes = sc->nodes;
  P.mats = sc->mats;
  P.texs = sc->texs;
  P.perlin = sc->perlin;
  P.lights = sc->lights;
  P.light_offs = sc->light_offs;
  P.texels = sc->texels;
  P.ops = sl->ops;
  P.queue = sl->queue;
  P.root = sc->hdr.root;
  P.n_lights = sc->hdr.n_lights;
  P.lights_is_list = sc->hdr.lights_is_list;
  P.lights_nested = sc->hdr.lights_nested;
  P.inv_n_lights = sc->hdr.n_lights ? 1.0 / (double)sc->hdr.n_lights : 0.0;
  P.sphere_light0 = sc->sphere_light0;
  P.flags = opts->flags;
  const bool count = (opts->flags & RT_FLAG_COUNT_OPS) != 0;
#ifdef RT_PROF  // profiling build: the product kernels also fill the ops buffer (section cycles)
  const bool ops_buf = true;
#else
  const bool ops_buf = count;
#endif
  // VOL kernels: ConstantMedium nodes or an Isotropic material (also usable outside one)
  const bool vol = (sc->hdr.has_volume | sc->hdr.has_isotropic) != 0;
  const bool tex = sc->hdr.has_textures != 0;
  const bool bvh = sc->hdr.has_bvh != 0;
  // product renders of a generated scene run its scene-specialised kernel (same template
  // arguments and launch bounds as the ahead-of-time kernel, top-level walk unrolled; rt_jit.cpp)
  const bool want_jit = !count && !(opts->flags & RT_FLAG_INTERPRETER) && sc->jit_state >= 0;
  // LDS: staged tables, then the compact ordered BVHs (rt_layout.h CBVH) with the walk's
  // per-lane stacks, or as much of the reference BVH region as fits (plan_lds); with the compact
  // trees in LDS the reference BVH region stays in global memory (only lanes flagged for the
  // reference-order re-walk read it)
  const LdsPlan LP = plan_lds(sc->hdr, sc->o_perl, opts->flags, want_jit, sc->lds_module_max);
  const int block = LP.block;
  const size_t static_lds = LP.static_lds;
  P.stage_scene = LP.stage_scene;
  P.n_perlin_lds = LP.n_perlin_lds;
  P.stage_src = LP.stage_scene ? sc->dev : sc->perlin;
  P.stage_bytes = LP.stage_bytes;
  P.bvh_words = sc->hdr.bvh_words;
  P.cbvh_src = (const uint8_t*)(sc->nodes + sc->hdr.cbvh_word0);
  P.cbvh_bytes = LP.cbvh_bytes;
  P.cbvh_lds_off = LP.cbvh_lds_off;
  P.stack_lds_off = LP.stack_lds_off;
  P.bvh_lds_words = LP.bvh_lds_words;
  P.bvh_lds_off = LP.bvh_lds_off;
  P.row_lds_off = LP.row_lds_off;
  P.o_mats = sc->o_mats;
  P.o_texs = sc->o_texs;
  P.o_lights = sc->o_lights;
  P.o_loffs = sc->o_loffs;
  P.o_perl = sc->o_perl;
  const size_t lds_bytes = LP.lds_bytes;
  for (int k = 0; k < 3; ++k) {
    P.center[k] = cam->center[k];
    P.p00[k] = cam->pixel00_loc[k];
    P.du[k] = cam->pixel_delta_u[k];
    P.dv[k] = cam->pixel_delta_v[k];
    P.ddu[k] = cam->defocus_disk_u[k];
    P.ddv[k] = cam->defocus_disk_v[k];
    P.bg[k] = cam->background[k];
  }
  P.rs = cam->recip_sqrt_spp;
  P.defocus = cam->defocus_angle > 0.0;
  P.W = W;
  P.n_rows = opts->n_rows;
  P.row_begin = opts->row_begin;
  P.row_step = opts->row_step;
  P.sqrt_spp = S;
  P.max_depth = cam->max_depth;
  P.seed_lo = (uint32_t)opts->seed;
  P.seed_hi = (uint32_t)(opts->seed >> 32);
  P.tiles_x = (W + kWaveTile - 1) / kWaveTile;
  const int tiles_y = (opts->n_rows + kWaveTile - 1) / kWaveTile;
  const int n_tiles = P.tiles_x * tiles_y;
  P.n_blk = (S + kPoolSi - 1) / kPoolSi;
  typedef void (*kern_t)(TraceParams);
  // [count][vol][tex][bvh]; a scene without a BVH whose tables are staged in LDS runs the
  // STAGED variant (LDS-typed table reads), BVH kernels read the tables from global memory
  static const kern_t table[16] = {
      rt_trace<false, false, false, false, false>, rt_trace<false, false, false, true, false>,
      rt_trace<false, false, true, false, false>,  rt_trace<false, false, true, true, false>,
      rt_trace<false, true, false, false, false>,  rt_trace<false, true, false, true, false>,
      rt_trace<false, true, true, false, false>,   rt_trace<false, true, true, true, false>,
      rt_trace<true, false, false, false, false>,  rt_trace<true, false, false, true, false>,
      rt_trace<true, false, true, false, false>,   rt_trace<true, false, true, true, false>,
      rt_trace<true, true, false, false, false>,   rt_trace<true, true, false, true, false>,
      rt_trace<true, true, true, false, false>,    rt_trace<true, true, true, true, false>};
  // [count][vol][tex], no BVH, staged
  static const kern_t table_staged[8] = {
      rt_trace<false, false, false, false, true>, rt_trace<false, false, true, false, true>,
      rt_trace<false, true, false, false, true>,  rt_trace<false, true, true, false, true>,
      rt_trace<true, false, false, false, true>,  rt_trace<true, false, true, false, true>,
      rt_trace<true, true, false, false, true>,   rt_trace<true, true, true, false, true>};
  const bool staged = !bvh && P.stage_scene && !sc->hdr.nested_volumes;
  const int kidx = ((opts->flags & RT_FLAG_COUNT_OPS) ? 8 : 0) + (vol ? 4 : 0) + (tex ? 2 : 0) +
                   (bvh ? 1 : 0) + (staged ? 16 : 0);
  // BVH scenes whose volumes all sit outside BVH subtrees (final_scene) run the variant whose
  // per-lane walker has no volume branch; when those volumes are all one-walk spheres, the
  // top-level walker carries no two-walk interpreter either
  static const kern_t table_bvh_novolb[8] = {
      rt_trace<false, true, false, true, false, false>, rt_trace<false, true, true, true, false, false>,
      rt_trace<true, true, false, true, false, false>,  rt_trace<true, true, true, true, false, false>,
      rt_trace<false, true, false, true, false, false, false>,
      rt_trace<false, true, true, true, false, false, false>,
      rt_trace<true, true, false, true, false, false, false>,
      rt_trace<true, true, true, true, false, false, false>};
  const bool novolb = bvh && vol && !sc->hdr.volume_in_bvh;
  // the op-counting build always walks twice, so only product kernels drop the interpreter
  const bool novoli = novolb && sc->hdr.volumes_one_walk_spheres && !(opts->flags & RT_FLAG_COUNT_OPS);
  const int vb = (novoli ? 4 : 0) + (kidx >= 8 ? 2 : 0) + (tex ? 1 : 0);
  kern_t kern = staged ? table_staged[kidx / 2 - 8] : (novolb ? table_bvh_novolb[vb] : table[kidx]);
  int kslot = novolb ? 32 + vb : kidx;
  // ConstantMedium nested in volume boundaries (rt_flatten.cpp: at most RTL_VOLUME_NEST deep):
  // the generic texture/volume kernels that walk them (no scene-specialised kernel)
  static const kern_t table_nested[4] = {
      rt_trace<false, true, true, false, false, true, true, RTL_VOLUME_NEST>,
      rt_trace<false, true, true, true, false, true, true, RTL_VOLUME_NEST>,
      rt_trace<true, true, true, false, false, true, true, RTL_VOLUME_NEST>,
      rt_trace<true, true, true, true, false, true, true, RTL_VOLUME_NEST>};
  if (sc->hdr.nested_volumes) {
    const int ni = ((opts->flags & RT_FLAG_COUNT_OPS) ? 2 : 0) + (bvh ? 1 : 0);
    kern = table_nested[ni];
    kslot = 44 + ni;
  }
  hipFunction_t jfn = nullptr;
  if (want_jit && lds_bytes + static_lds <= sc->lds_module_max) {
    rtj::Kernel& jk = sc->jit_k[(tex ? 1 : 0) + (staged ? 2 : 0)];
    if (!jk.fn) {
      std::string log;
      rtj::Flags jf;
      jf.vol = vol;
      jf.tex = tex;
      jf.bvh = bvh;
      jf.staged = staged;
      jf.volb = novolb ? false : vol;
      jf.voli = !novoli;
      if (rtj::get_kernel(sc->jit_walker, sc->device, jf, &jk, &log) != 0) {
        sc->jit_state = -2;
        sc->jit_msg = log;
      } else {
        // a dispatch the hardware cannot place aborts the whole queue (the CP's register or
        // LDS check), so the code object's resources are checked against this launch first:
        // workgroup size, VGPRs x waves per SIMD within the 512-entry file, LDS within the CU
        const int waves_per_simd = (block / 64 + 3) / 4;
        const int regs = (jk.regs + 7) & ~7;
        char why[256];
        std::snprintf(why, sizeof(why),
                      "scene-specialised kernel%s: %d regs, max %d threads, %d B static LDS, "
                      "%d B scratch/lane; launch %d threads, %zu B dynamic LDS",
                      jk.cached ? " (code-object cache)" : "", jk.regs, jk.max_threads,
                      jk.static_lds, jk.scratch, block, lds_bytes);
        if (jk.max_threads < block || regs * waves_per_simd > 512 ||
            (size_t)jk.static_lds + lds_bytes > sc->lds_module_max ||
            (size_t)jk.static_lds > static_lds) {
          sc->jit_state = -2;
          sc->jit_msg = std::string("not launched: ") + why;
          rtj::release_kernel(jk);
          jk = rtj::Kernel{};
        } else {
          sc->jit_msg = why;
        }
      }
    }
    if (jk.fn) {
      sc->jit_state = 1;
      jfn = jk.fn;
      kslot = 40 + (tex ? 1 : 0) + (staged ? 2 : 0);
    }
  }
  // (module kernels take their dynamic LDS size at launch)
  if (!jfn && lds_bytes > (64u << 10))
    HIP_TRY(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds_bytes));
  if (sc->resident_blocks[kslot] == 0 || sc->resident_lds[kslot] != lds_bytes) {
    int nb = 0;
    const hipError_t oe =
        jfn ? hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&nb, jfn, block, lds_bytes)
            : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)kern, block, lds_bytes);
    if (oe != hipSuccess || nb <= 0)
      return set_err(RT_ERR_HIP, std::string("occupancy query: the path kernel does not fit a CU (") +
                                     (oe != hipSuccess ? hipGetErrorString(oe) : "0 blocks") + ")");
    sc->resident_blocks[kslot] = nb;
    sc->resident_lds[kslot] = lds_bytes;
  }
  const int64_t max_blocks = (int64_t)sc->resident_blocks[kslot] * std::max(1, sc->n_cu);
  // Outputs (TraceParams::part): one f64 RGB value per (pixel, s_j) of the row pairs, one per
  // (pixel, s_j, block) of the segment pairs and one per sample of the tail pairs.
  //  * A launch of many pairs per resident wave (a whole frame on one GPU: C2 has 60) renders
  //    row items, then a band of segment items about four pairs per resident wave long, then a
  //    tail of single samples an eighth of a pair per wave long. When the row pools run out, the
  //    lanes still finishing a row have up to sqrt_spp paths left (rows through glass take
  //    several times the mean), and the band keeps the other lanes busy meanwhile; the tail
  //    does the same for the segments' last ~kPoolSi / 2 samples. The workspace is then about
  //    one value per (pixel, s_j): C2 0.59 GB instead of 2.1.
  //  * Smaller launches (an N-way share, chunks) balance better without rows (C2 over 8 GPUs:
  //    0.940 of ideal with segments, 0.894 with half the pairs as rows, profiles/
  //    r03_scaling_probe_*.log): segment items, then a tail of one pair per resident wave.
  //  * BVH kernels render rows when their plan fits the row totals beside the compact trees.
  // RT_SEG_PAIRS (rows with that band) and RT_TAIL_PAIRS override the sizes (tests: the image
  // does not depend on the split).
  const int64_t res_waves = max_blocks * (block / 64);
  const bool rows_ok = !bvh || LP.row_lds_off != ~0u;
  const char* seg_env = std::getenv("RT_SEG_PAIRS");
  const char* tail_env = std::getenv("RT_TAIL_PAIRS");
  struct Split {
    int64_t pairs, r, a, values;  // row pairs [0, r), segment pairs [r, a), tail [a, pairs)
  };
  auto split = [&](int cn) {
    Split sp;
    sp.pairs = (int64_t)n_tiles * cn;
    const bool rows = rows_ok && (seg_env ? true : sp.pairs >= 24 * res_waves);
    int64_t tail = rows ? std::max<int64_t>(1, res_waves / 8) : res_waves;
    if (tail_env) tail = std::strtoll(tail_env, nullptr, 10);
    const int64_t band = seg_env ? std::strtoll(seg_env, nullptr, 10) : 4 * res_waves;
    const int64_t tb = std::min<int64_t>(sp.pairs, std::max<int64_t>(0, tail));
    sp.a = sp.pairs - tb;
    sp.r = rows ? std::max<int64_t>(0, sp.a - std::max<int64_t>(0, band)) : 0;
    sp.values = sp.r + (sp.a - sp.r) * P.n_blk + tb * S;  // 64-value slots
    return sp;
  };
  const size_t tot_bytes = (n_px * 3 * sizeof(double) + 255) & ~(size_t)255;
  const size_t val_bytes = (size_t)64 * 3 * sizeof(double);  // one f64 RGB value per pixel
  auto part_bytes = [&](int cn) { return (size_t)split(cn).values * val_bytes; };
  // a launch's f64 RGB outputs are indexed in 32 bits (end_sample) and its pools in 31
  auto indexable = [&](int cn) {
    const Split sp = split(cn);
    return sp.values * 64 < (1ll << 32) && sp.r + (sp.pairs - sp.r) * P.n_blk <= 0x7fffffff;
  };
  // Chunks of stratum rows keep the workspace under RT_WORKSPACE_MB (default 40 GiB, at most a
  // quarter of the device's memory): the whole C5 frame (3840 x 2160, 10000 spp, ~19 GB of row
  // totals) renders in one launch; 800x800 x 961 spp takes one (~0.59 GB).
  size_t cap = std::min<size_t>((size_t)40960 << 20, sc->mem_total / 4);
  if (const char* e = std::getenv("RT_WORKSPACE_MB")) cap = (size_t)std::strtoull(e, nullptr, 10) << 20;
  int chunk = n_sj;
  while (chunk > 1 && (tot_bytes + part_bytes(chunk) > cap || !indexable(chunk)))
    chunk = (chunk + 1) / 2;
  const size_t need = tot_bytes + part_bytes(chunk);
  if (!indexable(chunk)) return set_err(RT_ERR_UNSUPPORTED, "grid too large");
  if (need > sl->work_bytes) {
    // the slot's previous render (another stream's, or this one's) may still read the old
    // workspace: let it finish first
    if (sl->recorded) HIP_TRY(hipEventSynchronize(sl->done));
    if (sl->work) HIP_TRY(hipFree(sl->work));
    sl->work = nullptr;
    sl->work_bytes = 0;
    HIP_TRY(hipMalloc(&sl->work, need));
    sl->work_bytes = need;
  }
  double* tot = (double*)sl->work;
  P.part = (double*)(sl->work + tot_bytes);
  hold.stream = stream;
  hold.enqueued = true;  // from here on a failure still records `done` (SlotHold)
  if (ops_buf) HIP_TRY(hipMemsetAsync(sl->ops, 0, sizeof(unsigned long long) * 32, stream));
#ifdef RT_PROF
  HIP_TRY(hipMemsetAsync(sl->ops + 40, 0, sizeof(unsigned long long) * 21, stream));
#endif
  if (stats) HIP_TRY(hipEventRecord(sl->ev0, stream));
  uint64_t out_bytes = 0;
  uint32_t launches = 0;
  for (int c0 = sj0; c0 < sj0 + n_sj; c0 += chunk) {
    const int cn = std::min(chunk, sj0 + n_sj - c0);
    out_bytes += part_bytes(cn);
    ++launches;
    const Split sp = split(cn);
    P.sj0 = c0;
    P.n_sj = cn;
    P.n_pairs_r = (int)sp.r;
    P.n_pairs_a = (int)sp.a;
    P.n_pools = (int)(sp.r + (sp.pairs - sp.r) * P.n_blk);
    // persistent grid: as many waves as the device holds at once (never more than pools)
    const int64_t blocks = std::min(max_blocks, ((int64_t)P.n_pools + (block / 64) - 1) / (block / 64));
    HIP_TRY(hipMemsetAsync(sl->queue, 0, sizeof(unsigned int), stream));
    const int ring = (int)(sc->n_tev % rt_scene::kTraceRing);
    HIP_TRY(hipEventRecord(sc->tev[ring][0], stream));
    if (jfn) {
      void* args[] = {&P};
      HIP_TRY(hipModuleLaunchKernel(jfn, (unsigned)blocks, 1, 1, (unsigned)block, 1, 1,
                                    (unsigned)lds_bytes, stream, args, nullptr));
    } else {
      hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(block), lds_bytes, stream, P);
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(sc->tev[ring][1], stream));
    sc->tev_render[ring] = sc->n_render;
    ++sc->n_tev;
    const int mode = (c0 == sj0 ? 1 : 0) | (c0 + cn == sj0 + n_sj ? 2 : 0) |
                     ((opts->flags & RT_FLAG_OVERWRITE) ? 4 : 0);
    hipLaunchKernelGGL(rt_reduce, dim3((unsigned)((n_tiles + 3) / 4)), dim3(256), 0, stream, P.part,
                       tot, accum, W, opts->n_rows, P.tiles_x, n_tiles, cn, S, P.n_pairs_r,
                       P.n_pairs_a, mode);
    HIP_TRY(hipGetLastError());
  }
  ++sc->n_render;
  if (stats) HIP_TRY(hipEventRecord(sl->ev1, stream));
  HIP_TRY(hipEventRecord(sl->done, stream));
  sl->recorded = true;
  sl->last_stream = stream;
  hold.finished = true;
  if (stats) {
    lock.unlock();  // the slot stays held: other renders of the scene go on meanwhile
    HIP_TRY(hipStreamSynchronize(stream));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, sl->ev0, sl->ev1));
    stats->ms_kernel = ms;
    stats->samples = (uint64_t)n_px * (uint64_t)n_sj * (uint64_t)S;
    stats->out_bytes = out_bytes;
    stats->launches = launches;
    if (ops_buf) {
      unsigned long long h[32];
      HIP_TRY(hipMemcpy(h, sl->ops, sizeof(h), hipMemcpyDeviceToHost));
      for (int k = 0; k < 32; ++k) stats->ops[k] = h[k];
    }
    stats->ms_total =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
  return RT_OK;
}

// Lane item keys hold the call's row index in 15 bits (render_device_rows): taller row ranges
// are rendered as consecutive sub-calls of kRowsPerCall rows into the matching rows of accum.
// The RNG is keyed by the global pixel and sample, so the image does not depend on the split.
constexpr int kRowsPerCall = 32760;

int rt_render_device(rt_scene* sc, const rt_camera* cam, const rt_render_opts* opts,
                     float* accum, void* stream_v, rt_stats* stats) {
  if (!sc || !cam || !opts || !accum) return set_err(RT_ERR_INVALID_ARG, "null argument");
  if (opts->n_rows <= kRowsPerCall || cam->image_width <= 0)
    return render_device_rows(sc, cam, opts, accum, stream_v, stats);
  auto t0 = std::chrono::steady_clock::now();
  rt_stats part{}, sum{};
  for (int k0 = 0; k0 < opts->n_rows; k0 += kRowsPerCall) {
    rt_render_opts o = *opts;
    o.row_begin = opts->row_begin + k0 * opts->row_step;
    o.n_rows = std::min(kRowsPerCall, opts->n_rows - k0);
    const int rc = render_device_rows(sc, cam, &o, accum + (size_t)k0 * cam->image_width * 3,
                                      stream_v, stats ? &part : nullptr);
    if (rc != RT_OK) return rc;
    if (stats) {
      sum.ms_kernel += part.ms_kernel;
      sum.samples += part.samples;
      sum.out_bytes += part.out_bytes;
      sum.launches += part.launches;
      for (int k = 0; k < 32; ++k) sum.ops[k] += part.ops[k];
    }
  }
  if (stats) {
    sum.ms_total =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    *stats = sum;
  }
  return RT_OK;
}

// Profiling builds (-DRT_PROF, not shipped): the ordered-BVH walk counters of the last render
// (rt_kernel.h obvh_walk). Other builds return zeros.
int rt_scene_prof_counters(rt_scene* sc, uint64_t* out, int n) {
  if (!sc || !out || n < 0) return set_err(RT_ERR_INVALID_ARG, "null argument");
  std::lock_guard<std::mutex> lock(sc->mu);
  HIP_TRY(hipSetDevice(sc->device));
  unsigned long long h[24] = {};
#ifdef RT_PROF
  if (sc->last_slot >= 0) {
    RenderSlot* sl = sc->slots[sc->last_slot].get();
    HIP_TRY(hipEventSynchronize(sl->done));
    HIP_TRY(hipMemcpy(h, sl->ops + 40, sizeof(h), hipMemcpyDeviceToHost));
  }
#endif
  for (int k = 0; k < n && k < 24; ++k) out[k] = h[k];
  return RT_OK;
}

int rt_scene_trace_ms(rt_scene* sc, float* ms_out, int max_n, int* n_out) {
  if (!sc || !ms_out || !n_out || max_n < 0) return set_err(RT_ERR_INVALID_ARG, "null argument");
  std::lock_guard<std::mutex> lock(sc->mu);
  HIP_TRY(hipSetDevice(sc->device));
  const uint64_t R = rt_scene::kTraceRing;
  const uint64_t first = sc->n_tev > R ? sc->n_tev - R : 0;
  // a render whose first launches fell out of the ring is incomplete: skip it
  const uint64_t skip_render = sc->n_tev > R ? sc->tev_render[first % R] : UINT64_MAX;
  std::vector<std::pair<uint64_t, double>> per;  // (render id, ms), oldest first
  for (uint64_t i = first; i < sc->n_tev; ++i) {
    const int k = (int)(i % R);
    const uint64_t id = sc->tev_render[k];
    if (id == skip_render) continue;
    HIP_TRY(hipEventSynchronize(sc->tev[k][1]));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, sc->tev[k][0], sc->tev[k][1]));
    if (per.empty() || per.back().first != id) per.push_back({id, 0.0});
    per.back().second += ms;
  }
  const int n = (int)std::min<size_t>((size_t)max_n, per.size());
  for (int i = 0; i < n; ++i) ms_out[i] = (float)per[per.size() - n + i].second;
  *n_out = n;
  return RT_OK;
}

int rt_render(rt_scene* sc, const rt_camera* cam, const rt_render_opts* opts, float* accum,
              rt_stats* stats) {
  auto t0 = std::chrono::steady_clock::now();
  if (!sc || !cam || !opts || !accum) return set_err(RT_ERR_INVALID_ARG, "null argument");
  if (opts->n_rows < 0 || cam->image_width <= 0) return set_err(RT_ERR_INVALID_ARG, "bad size");
  HIP_TRY(hipSetDevice(sc->device));
  size_t bytes = (size_t)opts->n_rows * cam->image_width * 3 * sizeof(float);
  if (bytes == 0) return RT_OK;
  float* d = nullptr;
  HIP_TRY(hipMalloc(&d, bytes));
  hipError_t e = (opts->flags & RT_FLAG_OVERWRITE) ? hipSuccess
                                                   : hipMemcpy(d, accum, bytes, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    (void)hipFree(d);
    return set_err(RT_ERR_HIP, std::string("upload accum: ") + hipGetErrorString(e));
  }
  rt_stats local;
  int rc = rt_render_device(sc, cam, opts, d, nullptr, stats ? stats : &local);
  if (rc == RT_OK) {
    e = hipMemcpy(accum, d, bytes, hipMemcpyDeviceToHost);
    if (e != hipSuccess) rc = set_err(RT_ERR_HIP, std::string("download accum: ") + hipGetErrorString(e));
  }
  (void)hipFree(d);
  if (rc == RT_OK && stats)
    stats->ms_total =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return rc;
}

int rt_render_multi(const rt_scene_blob* blob, const rt_camera* cam, const rt_render_opts* opts,
                    const int* devices, int n_devices, float* accum, rt_stats* stats) {
  auto t0 = std::chrono::steady_clock::now();
  if (!blob || !cam || !opts || !devices || !accum || n_devices <= 0)
    return set_err(RT_ERR_INVALID_ARG, "null argument or no devices");
  if (opts->n_rows < 0 || opts->row_step <= 0 || cam->image_width <= 0)
    return set_err(RT_ERR_INVALID_ARG, "bad row range");
  const int W = cam->image_width, G = n_devices;
  const size_t row_floats = (size_t)W * 3;
  int prev_device = -1;  // the caller's current device, restored on return
  (void)hipGetDevice(&prev_device);
  struct Part {
    rt_scene* sc = nullptr;
    hipStream_t stream = nullptr;
    float* dbuf = nullptr;
    std::vector<float> host;
    rt_render_opts o{};
  };
  std::vector<Part> parts(G);
  int rc = RT_OK;
  auto cleanup = [&]() {
    for (Part& p : parts) {
      if (p.sc) (void)hipSetDevice(p.sc->device);
      if (p.stream) (void)hipStreamSynchronize(p.stream);
      if (p.dbuf) (void)hipFree(p.dbuf);
      if (p.stream) (void)hipStreamDestroy(p.stream);
      rt_scene_destroy(p.sc);
    }
  };
  // device k renders rows k, k + G, ... of the call's rows (cyclic), each on its
  // own stream; all devices run concurrently, the host only waits at the end
  for (int k = 0; k < G && rc == RT_OK; ++k) {
    Part& p = parts[k];
    p.o = *opts;
    p.o.row_begin = opts->row_begin + k * opts->row_step;
    p.o.row_step = opts->row_step * G;
    p.o.n_rows = k < opts->n_rows ? (opts->n_rows - k + G - 1) / G : 0;
    p.o.device = devices[k];
    if (p.o.n_rows == 0) continue;
    rc = rt_scene_create(blob, devices[k], &p.sc);
    if (rc != RT_OK) break;
    hipError_t e = hipStreamCreateWithFlags(&p.stream, hipStreamNonBlocking);
    const size_t n = (size_t)p.o.n_rows * row_floats;
    if (e == hipSuccess) e = hipMalloc(&p.dbuf, n * sizeof(float));
    if (e == hipSuccess && !(opts->flags & RT_FLAG_OVERWRITE)) {
      p.host.resize(n);  // this device's rows of the caller's accumulator, accumulated on device
      for (int j = 0; j < p.o.n_rows; ++j)
        std::memcpy(&p.host[(size_t)j * row_floats],
                    accum + (size_t)(k + (size_t)j * G) * row_floats, row_floats * sizeof(float));
      e = hipMemcpyAsync(p.dbuf, p.host.data(), n * sizeof(float), hipMemcpyHostToDevice, p.stream);
    }
    if (e != hipSuccess) {
      rc = set_err(RT_ERR_HIP, std::string("rt_render_multi setup: ") + hipGetErrorString(e));
      break;
    }
    rc = rt_render_device(p.sc, cam, &p.o, p.dbuf, p.stream, nullptr);
  }
  for (int k = 0; k < G && rc == RT_OK; ++k) {
    Part& p = parts[k];
    if (!p.sc) continue;
    const size_t n = (size_t)p.o.n_rows * row_floats;
    p.host.resize(n);
    hipError_t e = hipSetDevice(p.sc->device);
    if (e == hipSuccess)
      e = hipMemcpyAsync(p.host.data(), p.dbuf, n * sizeof(float), hipMemcpyDeviceToHost, p.stream);
    if (e == hipSuccess) e = hipStreamSynchronize(p.stream);
    if (e != hipSuccess) {
      rc = set_err(RT_ERR_HIP, std::string("rt_render_multi gather: ") + hipGetErrorString(e));
      break;
    }
    for (int j = 0; j < p.o.n_rows; ++j)  // de-interleave into the caller's rows
      std::memcpy(accum + (size_t)(k + (size_t)j * G) * row_floats, &p.host[(size_t)j * row_floats],
                  row_floats * sizeof(float));
  }
  if (rc == RT_OK && stats) {
    std::memset(stats, 0, sizeof(*stats));
    const int S = cam->sqrt_spp, n_sj = opts->sj_count > 0 ? opts->sj_count : S;
    stats->samples = (uint64_t)opts->n_rows * W * (uint64_t)n_sj * S;
    stats->ms_total =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    stats->ms_kernel = stats->ms_total;
    stats->launches = (uint32_t)G;
  }
  const std::string err = rc == RT_OK ? std::string() : g_err;
  cleanup();
  if (rc != RT_OK) g_err = err;
  if (prev_device >= 0) (void)hipSetDevice(prev_device);
  return rc;
}

// ---------------------------------------------------------------- persistent multi-GPU handle
// rt_multi_create uploads the scene to every listed device once; each device keeps its scene,
// its workspace, its stream, its compact row buffer and (after the first frame) its compiled
// scene-specialised kernel across rt_multi_render calls. A frame: every device renders its
// cyclic rows into its own buffer on its own stream, the buffers are copied peer-to-peer
// (hipMemcpyPeerAsync: xGMI between MI355X devices) into a staging area on the first device,
// and one kernel there de-interleaves the rows into the caller's frame.
struct rt_multi {
  struct Dev {
    rt_scene* sc = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    float* rows = nullptr;  // compact rows of this device's share
    size_t rows_bytes = 0;
  };
  std::vector<int> devices;
  std::vector<Dev> dev;
  float* stage = nullptr;  // on devices[0]: every device's rows, device after device
  size_t stage_bytes = 0;
  hipEvent_t start = nullptr;  // on devices[0]: the frame's start on the caller's stream
  // on devices[0]: the previous frame's end (its gather out of `stage`); a frame rendered on
  // another caller stream waits for it before reusing the staging area and the device rows
  hipEvent_t frame_done = nullptr;
  bool frame_recorded = false;
  uint64_t frames = 0, uploads = 0, stage_allocs = 0;
  std::mutex mu;
};

int rt_multi_create(const rt_scene_blob* blob, const int* devices, int n_devices,
                    rt_multi** out) {
  if (!blob || !devices || n_devices <= 0 || !out)
    return set_err(RT_ERR_INVALID_ARG, "null argument or no devices");
  *out = nullptr;
  int prev = -1;
  (void)hipGetDevice(&prev);
  rt_multi* m = new rt_multi();
  m->devices.assign(devices, devices + n_devices);
  m->dev.resize(n_devices);
  int rc = RT_OK;
  for (int k = 0; k < n_devices && rc == RT_OK; ++k) {
    rc = rt_scene_create(blob, devices[k], &m->dev[k].sc);
    if (rc != RT_OK) break;
    ++m->uploads;
    hipError_t e = hipStreamCreateWithFlags(&m->dev[k].stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&m->dev[k].done, hipEventDisableTiming);
    // direct peer copies into the first device (already enabled / same device: not an error)
    if (e == hipSuccess && devices[k] != devices[0]) {
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, devices[k], devices[0]) == hipSuccess && can) {
        const hipError_t pe = hipDeviceEnablePeerAccess(devices[0], 0);
        if (pe != hipSuccess && pe != hipErrorPeerAccessAlreadyEnabled) e = pe;
        (void)hipGetLastError();
      }
    }
    if (e != hipSuccess) rc = set_err(RT_ERR_HIP, std::string("rt_multi_create: ") + hipGetErrorString(e));
  }
  if (rc == RT_OK) {
    hipError_t e = hipSetDevice(devices[0]);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&m->start, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&m->frame_done, hipEventDisableTiming);
    if (e != hipSuccess) rc = set_err(RT_ERR_HIP, std::string("rt_multi_create: ") + hipGetErrorString(e));
  }
  if (prev >= 0) (void)hipSetDevice(prev);
  if (rc != RT_OK) {
    const std::string err = g_err;
    rt_multi_destroy(m);
    g_err = err;
    return rc;
  }
  *out = m;
  return RT_OK;
}

void rt_multi_destroy(rt_multi* m) {
  if (!m) return;
  int prev = -1;
  (void)hipGetDevice(&prev);
  for (size_t k = 0; k < m->dev.size(); ++k) {
    rt_multi::Dev& d = m->dev[k];
    (void)hipSetDevice(m->devices[k]);
    if (d.stream) (void)hipStreamSynchronize(d.stream);
    if (d.rows) (void)hipFree(d.rows);
    if (d.done) (void)hipEventDestroy(d.done);
    if (d.stream) (void)hipStreamDestroy(d.stream);
    rt_scene_destroy(d.sc);
  }
  (void)hipSetDevice(m->devices[0]);
  if (m->stage) (void)hipFree(m->stage);
  if (m->start) (void)hipEventDestroy(m->start);
  if (m->frame_done) (void)hipEventDestroy(m->frame_done);
  delete m;
  if (prev >= 0) (void)hipSetDevice(prev);
}

int rt_multi_render(rt_multi* m, const rt_camera* cam, const rt_render_opts* opts,
                    float* accum_rgb_device0, void* hip_stream, rt_stats* stats) {
  auto t0 = std::chrono::steady_clock::now();
  if (!m || !cam || !opts || !accum_rgb_device0)
    return set_err(RT_ERR_INVALID_ARG, "null argument");
  if (opts->n_rows < 0 || opts->row_step <= 0 || cam->image_width <= 0)
    return set_err(RT_ERR_INVALID_ARG, "bad row range");
  if (opts->n_rows > 0 &&
      (int64_t)opts->row_begin + (int64_t)(opts->n_rows - 1) * opts->row_step >= cam->image_height)
    return set_err(RT_ERR_INVALID_ARG, "row range outside the image");
  std::lock_guard<std::mutex> lock(m->mu);
  int prev = -1;
  (void)hipGetDevice(&prev);
  const int G = (int)m->devices.size(), d0 = m->devices[0];
  const size_t row_floats = (size_t)cam->image_width * 3;
  const size_t frame_bytes = (size_t)opts->n_rows * row_floats * sizeof(float);
  hipStream_t out_stream = (hipStream_t)hip_stream;
  auto fail = [&](hipError_t e, const char* what) {
    if (prev >= 0) (void)hipSetDevice(prev);
    return set_err(RT_ERR_HIP, std::string("rt_multi_render ") + what + ": " + hipGetErrorString(e));
  };
  if (opts->n_rows == 0) return RT_OK;
  hipError_t e = hipSetDevice(d0);
  if (e == hipSuccess && m->frame_recorded) e = hipStreamWaitEvent(out_stream, m->frame_done, 0);
  if (e == hipSuccess && m->stage_bytes < frame_bytes) {
    // the previous frame's gather reads the staging buffer: it must have finished (a failed
    // wait leaves the buffer in use, so it is reported, not freed)
    if (m->frame_recorded) e = hipEventSynchronize(m->frame_done);
    if (e != hipSuccess) return fail(e, "staging buffer (waiting for the previous frame)");
    if (m->stage) (void)hipFree(m->stage);
    m->stage = nullptr;
    m->stage_bytes = 0;
    e = hipMalloc(&m->stage, frame_bytes);
    if (e == hipSuccess) m->stage_bytes = frame_bytes, ++m->stage_allocs;
  }
  if (e != hipSuccess) return fail(e, "staging buffer");
  const bool accumulate = !(opts->flags & RT_FLAG_OVERWRITE);
  const int gx = (int)std::min<size_t>(64, (row_floats + 255) / 256);
  if (accumulate) {  // the caller's rows to the staging area: each device accumulates its own
    hipLaunchKernelGGL(rt_deinterleave, dim3((unsigned)gx, (unsigned)opts->n_rows), dim3(256), 0,
                       out_stream, m->stage, accum_rgb_device0, (int)row_floats, opts->n_rows, G, 0);
    e = hipGetLastError();
    if (e != hipSuccess) return fail(e, "scatter");
  }
  // the caller's stream on the first device orders the frame: every device starts after it
  e = hipEventRecord(m->start, out_stream);
  if (e != hipSuccess) return fail(e, "start event");
  std::vector<char> used(G, 0);
  uint64_t samples = 0;
  size_t row0 = 0;
  int rc = RT_OK;
  for (int k = 0; k < G && rc == RT_OK; ++k) {
    rt_multi::Dev& d = m->dev[k];
    rt_render_opts o = *opts;
    o.row_begin = opts->row_begin + k * opts->row_step;
    o.row_step = opts->row_step * G;
    o.n_rows = k < opts->n_rows ? (opts->n_rows - k + G - 1) / G : 0;
    o.device = m->devices[k];
    // compact rows: overwritten, or the caller's rows (scattered above) accumulated into
    if (o.n_rows == 0) continue;
    const size_t bytes = (size_t)o.n_rows * row_floats * sizeof(float);
    e = hipSetDevice(m->devices[k]);
    if (e == hipSuccess && d.rows_bytes < bytes) {
      if (d.rows) (void)hipFree(d.rows);
      d.rows = nullptr;
      d.rows_bytes = 0;
      e = hipMalloc(&d.rows, bytes);
      if (e == hipSuccess) d.rows_bytes = bytes;
    }
    if (e == hipSuccess) e = hipStreamWaitEvent(d.stream, m->start, 0);
    if (e == hipSuccess && accumulate)
      e = hipMemcpyPeerAsync(d.rows, m->devices[k], m->stage + row0 * row_floats, d0, bytes, d.stream);
    if (e != hipSuccess) {
      rc = fail(e, "device setup");
      break;
    }
    rc = rt_render_device(d.sc, cam, &o, d.rows, d.stream, nullptr);
    if (rc != RT_OK) break;
    // the rows travel to the first device's staging area (xGMI peer copy, or a local copy)
    e = hipMemcpyPeerAsync(m->stage + row0 * row_floats, d0, d.rows, m->devices[k], bytes, d.stream);
    if (e == hipSuccess) e = hipEventRecord(d.done, d.stream);
    if (e != hipSuccess) {
      rc = fail(e, "peer copy");
      break;
    }
    used[k] = 1;
    samples += (uint64_t)o.n_rows * cam->image_width *
               (uint64_t)(opts->sj_count > 0 ? opts->sj_count : cam->sqrt_spp) * cam->sqrt_spp;
    row0 += (size_t)o.n_rows;
  }
  if (rc == RT_OK) {
    e = hipSetDevice(d0);
    for (int k = 0; k < G && e == hipSuccess; ++k)
      if (used[k]) e = hipStreamWaitEvent(out_stream, m->dev[k].done, 0);
    if (e == hipSuccess) {
      hipLaunchKernelGGL(rt_deinterleave, dim3((unsigned)gx, (unsigned)opts->n_rows), dim3(256), 0,
                         out_stream, m->stage, accum_rgb_device0, (int)row_floats, opts->n_rows, G, 1);
      e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipEventRecord(m->frame_done, out_stream);
    if (e == hipSuccess) m->frame_recorded = true;
    if (e == hipSuccess && stats) e = hipStreamSynchronize(out_stream);
    if (e != hipSuccess) rc = fail(e, "gather");
  }
  if (rc == RT_OK) {
    ++m->frames;
    if (stats) {
      std::memset(stats, 0, sizeof(*stats));
      stats->samples = samples;
      stats->launches = (uint32_t)G;
      stats->ms_total =
          std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      stats->ms_kernel = stats->ms_total;
    }
  }
  if (prev >= 0) (void)hipSetDevice(prev);
  return rc;
}

int rt_multi_info(rt_multi* m, uint64_t* out, int n) {
  if (!m || !out || n < 0) return set_err(RT_ERR_INVALID_ARG, "null argument");
  std::lock_guard<std::mutex> lock(m->mu);
  const uint64_t v[4] = {m->frames, m->uploads, m->stage_allocs, (uint64_t)m->devices.size()};
  for (int k = 0; k < n && k < 4; ++k) out[k] = v[k];
  return RT_OK;
}

int rt_render_blob(const rt_scene_blob* blob, const rt_camera* cam, const rt_render_opts* opts,
                   float* accum, rt_stats* stats) {
  if (!opts) return set_err(RT_ERR_INVALID_ARG, "null opts");
  rt_scene* sc = nullptr;
  int rc = rt_scene_create(blob, opts->device, &sc);
  if (rc != RT_OK) return rc;
  rc = rt_render(sc, cam, opts, accum, stats);
  rt_scene_destroy(sc);
  return rc;
}

}  // extern "C"
