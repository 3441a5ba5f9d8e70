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

// Words of the node record starting with header word h (rt_layout.h).
uint32_t record_words(uint32_t h);

// Returns RT_OK or a negative rt status; *err explains failures.
int flatten(const rt_scene_blob* blob, FlatScene* out, std::string* err);

}  // namespace rtf
