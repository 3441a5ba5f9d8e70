// rt_jit.hpp — scene-specialised path kernels: the world walker generated from the flattened
// scene and compiled at run time by hiprtc (rt_jit.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "rt_flatten.hpp"

namespace rtj {

// Source of `struct TravGen` (the world query of ray_color, render.rs:264-267) for this scene:
// the wave-uniform node sequence that the interpreter (rt_kernel.h traverse<UNI>) walks at run
// time, unrolled, with every record's constants as literals; a BVH subtree record becomes a call
// of the interpreter's per-lane walker. Empty when the scene has records the generator does not
// emit or is too large; *why says which.
std::string generate(const rtf::FlatScene& F, std::string* why);

// Template arguments of the path kernel (rt_kernel.h trace_body) the generated walker runs in;
// the same as the ahead-of-time interpreter kernel the scene would otherwise launch.
struct Flags {
  bool vol = false, tex = false, staged = false, bvh = false, volb = false, voli = true;
};
// Flags of the product kernel for scene header `hdr` (rt_device.hip's kernel choice).
Flags product_flags(const rtf::FlatScene& F, bool staged);

// Kernel for (generated walker, feature flags) on `device`, compiled on first use and cached for
// the process. Returns 0 or a negative rt status with *log filled.
struct Kernel {
  hipModule_t mod = nullptr;
  hipFunction_t fn = nullptr;
  // code-object resources as the runtime reports them (hipFuncGetAttribute), checked against
  // the launch before every first use (rt_device.hip)
  int regs = 0, max_threads = 0, static_lds = 0, scratch = 0;
  bool cached = false;  // loaded from the code-object cache (rt_jit.cpp cache_path), not compiled
};
int get_kernel(const std::string& walker, int device, const Flags& f, Kernel* out,
               std::string* log);
// A scene's hold on a kernel from get_kernel ends (rt_scene_destroy). The process-wide cache keeps
// every kernel some scene holds, plus up to kIdleModules unheld ones for scenes created again
// with the same geometry; older unheld modules are unloaded (hipModuleUnload).
constexpr int kIdleModules = 8;
void release_kernel(const Kernel& k);

// The hiprtc translation unit (embedded headers + walker + rt_trace_jit wrapper) and its
// compilation for `arch` (e.g. "gfx950") into a code object; host-only, no device needed.
// use_cache = false bypasses the code-object cache (a cached entry that failed to load).
std::string kernel_source(const std::string& walker, const Flags& f);
int compile(const std::string& src, const std::string& arch, std::vector<char>* code,
            std::string* log, bool use_cache = true);

}  // namespace rtj
