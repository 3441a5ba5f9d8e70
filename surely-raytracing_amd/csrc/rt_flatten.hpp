// rt_flatten.hpp — rt_scene_blob (include/rt_mi355x.h) -> threaded device layout (rt_layout.h).
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/rt_mi355x.h"
#include "rt_layout.h"

namespace rtf {

struct FlatScene {
  rtl_scene_header hdr{};
  std::vector<uint32_t> nodes;        // threaded pre-order node words
  std::vector<uint32_t> mats;         // RTL_MAT_WORDS each
  std::vector<uint32_t> texs;         // RTL_TEX_WORDS each
  std::vector<uint8_t> perlin;        // RTL_PERLIN_BYTES each
  std::vector<uint32_t> lights;       // node-format light records
  std::vector<uint32_t> light_offs;   // word offset of each light record
  std::vector<uint8_t> texels;
};

// Conservative bounds of a leaf record (QUAD, QUADS batch, SPHERE), by record word position.
// ref_complete: the reference's own Aabb of the primitive (object.rs:427-431: q and q + u + v,
// padded) contains the whole primitive, so its BVH culls no true candidate.
struct PrimBox {
  double lo[3] = {0, 0, 0}, hi[3] = {0, 0, 0};
  bool valid = false, ref_complete = false;
};

// rt_obvh.cpp: append an ordered BVH (rt_layout.h OBVH) for every eligible BVH subtree root in
// `roots` (word positions of BVH records) and link it from the root's word 3.
// Also appends the compact copies of those trees (rt_layout.h CBVH) as one region and returns
// its first word and size in words (0, 0 when there is none).
void build_ordered_bvhs(std::vector<uint32_t>& nodes, uint32_t rec_words,
                        const std::vector<PrimBox>& boxes, const std::vector<uint32_t>& roots,
                        uint32_t* cbvh_word0, uint32_t* cbvh_words, uint32_t* cbvh_stack);

// Words of the node record starting with header word h (rt_layout.h).
uint32_t record_words(uint32_t h);

// rt_obvh.cpp: host checks of the compact trees the LDS walk reads (rt_kernel.h cbvh_walk_t):
// their structure (references in range, every internal node and leaf reached once from the root,
// leaf records that are QUAD / QUADS / SPHERE records inside the record region, blocks inside the
// CBVH region, 16-byte aligned), their internal-node depth against the header's cbvh_stack, and
// a host restatement of the walk's LDS addressing over random rays with no closest-hit culling
// (every box the slab test keeps is visited: the worst case for the stack): the largest stack
// slot the walk stores to (the far child is stored every step, rt_kernel.h) and the largest
// byte offset it reads in the region.
struct WalkCheck {
  uint32_t trees = 0;           // compact trees
  uint32_t max_depth = 0;       // largest internal-node depth (root = 1)
  uint32_t errors = 0;          // structural errors (0 = every tree well formed)
  uint32_t max_store_slot = 0;  // largest stack slot stored to (0-based entries)
  uint32_t max_live = 0;        // largest number of pending entries
  uint64_t rays = 0, steps = 0;  // walks emulated, box steps taken
  uint64_t max_read = 0;        // one past the largest CBVH-region byte read
  std::string first_error;
};
WalkCheck check_compact_trees(const std::vector<uint32_t>& nodes, const rtl_scene_header& hdr,
                              uint32_t n_rays, uint64_t seed);

// Returns RT_OK or a negative rt status; *err explains failures.
int flatten(const rt_scene_blob* blob, FlatScene* out, std::string* err);

}  // namespace rtf
