// rt_jit.cpp — scene-specialised path kernels (rt_jit.hpp).
//
// The interpreter (rt_kernel.h traverse<UNI=true>) walks the flattened scene at run time: a
// scalar load of each record header, a scalar branch on its type, the record's constants in
// SGPRs, and register copies wherever the node types' states join. Outside BVH subtrees that
// node sequence does not depend on the ray (render.rs:264 -> hittable.rs:88-109 visits every
// list child in order), so it is known when the scene is created. generate() writes it out as
// straight-line code: the same arithmetic functions in the same order (aquad_test, quad_test,
// sphere_test_v, translate_in, rotate_y_in), each record's constants as exact hex-float
// literals, the rcp of the ray direction formed once per frame and axis, and the winner kept
// as one packed (record, frame) code. Per-lane results are therefore bit-identical to the
// interpreter's (tests/test_gpu_parity.py), which remains the op-counting build's path. A
// ConstantMedium record calls the interpreter's volume_hit (its boundary walks stay
// interpreted), and a BVH subtree record calls the interpreter's per-lane walker (traverse<UNI =
// false>, hittable.rs:216-236) with the generated walk's closest hit, exactly as the UNI
// interpreter hands the subtree over.
//
// hiprtc compiles rt_kernel.h (embedded at build time, build/rt_jit_sources.inc) plus the
// generated walker and an rt_trace wrapper with the same template arguments and launch bounds
// as the ahead-of-time kernel (about a second per scene on the host); modules are cached per
// (source, device) for the process.
#include "rt_jit.hpp"

#include <dlfcn.h>
#include <hip/hiprtc.h>
#include <unistd.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <fstream>
#include <iterator>
#include <sstream>
#include <utility>
#include <vector>

#include "rt_jit_sources.inc"  // kJitSrcNames[], kJitSrcText[], kJitSrcCount (Makefile)

namespace rtj {
namespace {
// FNV-1a, 64 bits, over a sequence of strings (each terminated by its length)
uint64_t fnv1a(uint64_t h, const char* p, size_t n) {
  for (size_t i = 0; i < n; ++i) h = (h ^ (uint8_t)p[i]) * 0x100000001b3ull;
  for (int k = 0; k < 8; ++k) h = (h ^ (uint8_t)(n >> (8 * k))) * 0x100000001b3ull;
  return h;
}

// Where the code object of this translation unit lives in the code-object cache, or "" when the
// cache is off. The directory is RT_JIT_CACHE_DIR, by default jit_cache/ next to this library
// (build/jit_cache, filled at build time by tools/jit_cache_fill.py for the benchmark scenes); the
// file name is a 128-bit hash of the source, every header text and every compile option (which
// include the target), so an edited header or option never loads a stale object. RT_JIT_CACHE=0
// turns the cache off. Why: the hiprtc a process binds to is whichever libhiprtc.so.7 it loaded
// first (PyTorch's bundled ROCm 7.0 compiler once torch is imported, the system's 7.2 one
// otherwise or under rocprofv3, which preloads the system runtime), and the two allocate
// registers differently (final_scene: 163 VGPRs and no spills against 168 + 71 spilled); with the
// cache the benchmark, the tests and the profiler all run the one binary built at build time.
std::string cache_path(const std::string& src, const std::vector<const char*>& headers,
                       const std::vector<const char*>& opts) {
  const char* off = std::getenv("RT_JIT_CACHE");
  if (off && std::strcmp(off, "0") == 0) return "";
  std::string dir;
  if (const char* d = std::getenv("RT_JIT_CACHE_DIR")) {
    dir = d;
  } else {
    Dl_info info;
    if (!dladdr((const void*)&fnv1a, &info) || !info.dli_fname) return "";
    dir = info.dli_fname;
    const size_t slash = dir.rfind('/');
    dir = (slash == std::string::npos ? std::string(".") : dir.substr(0, slash)) + "/jit_cache";
  }
  uint64_t a = 0xcbf29ce484222325ull, b = 0x84222325cbf29ce4ull;
  auto add = [&](const char* p) {
    const size_t n = std::strlen(p);
    a = fnv1a(a, p, n);
    b = fnv1a(b ^ 0x9e3779b97f4a7c15ull, p, n);
  };
  add(src.c_str());
  for (const char* h : headers) add(h);
  for (const char* o : opts) add(o);
  char name[64];
  std::snprintf(name, sizeof name, "/%016llx%016llx.co", (unsigned long long)a,
                (unsigned long long)b);
  return dir + name;
}


// Largest scene the generator unrolls (primitive tests per world query) and the packed winner
// code's range: (record + 1) | frame_id << 24, frame_id = the frame's ordinal in the walk (0 = the
// world frame); kBvhCode marks "the last hit came from a BVH subtree" (record/frame in bhn/bhf).
constexpr size_t kMaxPrims = 512;
constexpr size_t kMaxWords = 0xfffffe;
constexpr size_t kMaxFrames = 254;
constexpr uint32_t kBvhCode = 0xffffffffu;

double word_double(const std::vector<uint32_t>& N, size_t w) {
  const uint64_t bits = (uint64_t)N[w] | ((uint64_t)N[w + 1] << 32);
  double d;
  std::memcpy(&d, &bits, sizeof d);
  return d;
}
// payload double k of the record at `rec` (rt_layout.h: doubles start at word 4)
double pd(const std::vector<uint32_t>& N, size_t rec, int k) { return word_double(N, rec + 4 + 2 * k); }

std::string lit(double v) {  // exact: hex-float literal of the same bits
  // (%a prints non-finite values as inf / nan, which are not C++ literals: a degenerate quad's
  // normal, unit(0) = NaN, is valid reference input)
  if (std::isnan(v)) return "(__builtin_nan(\"\"))";
  if (std::isinf(v)) return v > 0 ? "(__builtin_inf())" : "(-__builtin_inf())";
  char b[64];
  std::snprintf(b, sizeof b, "(%a)", v);
  return b;
}
std::string lit3(double x, double y, double z) {
  return "mk(" + lit(x) + ", " + lit(y) + ", " + lit(z) + ")";
}

struct Gen {
  const std::vector<uint32_t>& N;
  std::ostringstream o;
  bool rcp[3] = {false, false, false};  // rcp of d per axis formed in the current frame
  size_t prims = 0;
  std::vector<int> frames{-1};  // frame_id -> frame record (-1 = world)
  bool bvh = false;             // a BVH subtree call was emitted

  explicit Gen(const std::vector<uint32_t>& n) : N(n) {}

  void frame_changed() { rcp[0] = rcp[1] = rcp[2] = false; }
  void need_rcp(int k) {
    static const char* ax = "xyz";
    if (!rcp[k]) {
      o << "    r" << ax[k] << " = rcp_nr1(d." << ax[k] << ");\n";
      rcp[k] = true;
    }
  }
  // xform_in of the record at x (transform.rs:59, 86-107). A translation leaves d, a rotation
  // about y leaves d.y as they are (rt_kernel.h translate_in / rotate_y_in), so the reciprocals
  // of those components stay valid.
  void xform(size_t x) {
    if ((N[x] & 0xffu) == RTL_TRANSLATE) {
      o << "    C.inc(RT_OP_TRANSLATE);\n    translate_in(" << lit3(pd(N, x, 2), pd(N, x, 3), pd(N, x, 4))
        << ", o);\n";
    } else {
      o << "    C.inc(RT_OP_ROTATE_Y);\n    rotate_y_in(" << lit(pd(N, x, 2)) << ", " << lit(pd(N, x, 3))
        << ", o, d);\n";
      rcp[0] = rcp[2] = false;
    }
  }
  uint32_t code(size_t rec, int frame) {
    size_t id = 0;
    while (id < frames.size() && frames[id] != frame) ++id;
    if (id == frames.size()) frames.push_back(frame);
    return (uint32_t)(rec + 1) | ((uint32_t)id << 24);
  }
  // world_quad_test of the QUAD record at q (object.rs:453-490)
  void quad(size_t q, int frame) {
    const uint32_t axis = RTL_QUAD_AXIS(N[q]);
    o << "    t = closest;\n";
    if (axis) {
      const int k = (int)axis - 1;
      need_rcp(k);
      o << "    h = aquad_test<COUNT, " << k << ">(AQuad{" << N[q] << "u, " << lit(pd(N, q, 0)) << ", "
        << lit(pd(N, q, 1)) << ", " << lit(pd(N, q, 2)) << ", " << lit(pd(N, q, 3)) << ", "
        << lit(pd(N, q, 4)) << "}, o, d, mk(rx, ry, rz), tmin, closest, t, C);\n";
    } else {
      o << "    h = quad_test<COUNT>(N + " << (q + RTL_QUAD_GEN) << "u, o, d, tmin, closest, t, C);\n";
    }
    o << "    closest = t;\n    code = h ? " << code(q, frame) << "u : code;\n";
    ++prims;
  }
  // sphere_test of the SPHERE record at s (object.rs:107-112, 145-184)
  void sphere(size_t s, int frame) {
    o << "    t = closest;\n    {\n      d3 c = " << lit3(pd(N, s, 0), pd(N, s, 1), pd(N, s, 2)) << ";\n";
    if (N[s] & RTL_SPHERE_MOVING)
      o << "      c = vfma(tm, " << lit3(pd(N, s, 4), pd(N, s, 5), pd(N, s, 6)) << ", c);\n";
    o << "      h = sphere_test_v<COUNT>(c, " << lit(pd(N, s, 3)) << ", o, d, tmin, closest, t, C);\n"
      << "    }\n    closest = t;\n    code = h ? " << code(s, frame) << "u : code;\n";
    ++prims;
  }
};

// The one-walk boundary query of the ConstantMedium record at `node` (rt_kernel.h
// volume_two_hits: constant_medium.rs:46-55's rec1/rec2 as the two smallest candidates), its
// instance chain and primitives unrolled with their constants as literals. Appends `struct
// VolTwo_<node>` to `o`; false when the boundary is not a one-walk form.
bool gen_volume_two_hits(const std::vector<uint32_t>& N, size_t node, std::ostringstream& o) {
  const uint32_t kind = N[node] & (RTL_VOLF_SPHERE | RTL_VOLF_QUADS);
  if (!kind) return false;
  std::ostringstream b;
  size_t x = N[node + 3];
  for (int guard = 0;; ++guard) {  // the instance chain in front of the primitive(s)
    if (x + 4 > N.size() || guard > 4096) return false;
    const uint32_t ty = N[x] & 0xffu;
    if (ty == RTL_TRANSLATE) {
      b << "    translate_in(" << lit3(pd(N, x, 2), pd(N, x, 3), pd(N, x, 4)) << ", o);\n";
    } else if (ty == RTL_ROTATE_Y) {
      b << "    rotate_y_in(" << lit(pd(N, x, 2)) << ", " << lit(pd(N, x, 3)) << ", o, d);\n";
    } else {
      break;
    }
    x = N[x + 3];
  }
  const uint32_t ty = N[x] & 0xffu;
  if (kind == RTL_VOLF_SPHERE) {
    if (ty != RTL_SPHERE) return false;
    b << "    d3 center = " << lit3(pd(N, x, 0), pd(N, x, 1), pd(N, x, 2)) << ";\n";
    if (N[x] & RTL_SPHERE_MOVING)
      b << "    center = vfma(tm, " << lit3(pd(N, x, 4), pd(N, x, 5), pd(N, x, 6)) << ", center);\n";
    b << "    const double r = " << lit(pd(N, x, 3)) << ";\n"
         "    const d3 oc = o - center;\n"
         "    const double a = dot(d, d);\n"
         "    const double half_b = dot(oc, d);\n"
         "    const double c = dot(oc, oc) - r * r;\n"
         "    const double disc = fma(half_b, half_b, -(a * c));\n"
         "    const bool real = !(disc < 0.0);\n"
         "    const double sqrtd = sqrt_nr(disc);\n"
         "    const double ra = rcp_nr(a);\n"
         "    const double near = (-half_b - sqrtd) * ra;\n"
         "    const double far = (sqrtd - half_b) * ra;\n"
         "    const bool n1 = (-kInf < near) & (near < kInf), f1 = (-kInf < far) & (far < kInf);\n"
         "    t1 = n1 ? near : far;\n"
         "    const double tmin2 = t1 + 0.0001;\n"
         "    const bool n2 = (tmin2 < near) & (near < kInf), f2 = (tmin2 < far) & (far < kInf);\n"
         "    t2 = n2 ? near : far;\n"
         "    return real & (n1 | f1) & (n2 | f2);\n";
  } else {
    if (ty != RTL_QUAD && ty != RTL_QUADS) return false;
    const bool batch = ty == RTL_QUADS;
    const uint32_t cnt = batch ? (N[x] >> 8) : 1u;
    const size_t q0 = batch ? x + 4 : x;
    b << "    const d3 r = mk(rcp_nr1(d.x), rcp_nr1(d.y), rcp_nr1(d.z));\n"
         "    double m1 = kInf, m2 = kInf;  // the two smallest candidates, +inf = none\n";
    static const char* ax = "xyz";
    for (uint32_t k = 0; k < cnt; ++k) {
      const size_t q = q0 + (size_t)k * RTL_QUAD_WORDS;
      if (q + RTL_QUAD_WORDS > N.size()) return false;
      const uint32_t axis = RTL_QUAD_AXIS(N[q]);
      const int K = axis == 1u ? 0 : (axis == 2u ? 1 : 2);  // volume_two_hits' switch
      b << "    {\n      const AQuad q = {" << N[q] << "u, " << lit(pd(N, q, 0)) << ", "
        << lit(pd(N, q, 1)) << ", " << lit(pd(N, q, 2)) << ", " << lit(pd(N, q, 3)) << ", "
        << lit(pd(N, q, 4)) << "};\n"
        << "      double t;\n      bool inr;\n      aquad_core<" << K << ">(q, o, d, r, t, inr);\n"
        << "      const double dk = d." << ax[K] << ";\n"
           "      const bool v = !(fabs(dk) < 1e-8) & (-kInf <= t) & inr;\n"
           "      const double te = v ? t : kInf;\n"
           "      m2 = __builtin_fmin(m2, __builtin_fmax(m1, te));\n"
           "      m1 = __builtin_fmin(m1, te);\n    }\n";
    }
    b << "    const bool have1 = m1 < kInf, have2 = m2 < kInf;\n"
         "    t1 = m1;\n"
         "    const double tmin2 = m1 + 0.0001;\n"
         "    bool hit2;\n"
         "    if (m1 >= tmin2) {\n      t2 = m1;\n      hit2 = true;\n"
         "    } else if (have2 && m2 >= tmin2) {\n      t2 = m2;\n      hit2 = true;\n"
         "    } else {\n      t2 = 0.0;\n      hit2 = false;\n      fallback = have2;\n    }\n"
         "    return have1 & (hit2 | fallback);\n";
  }
  o << "struct VolTwo_" << node << " {\n"
       "  static __device__ __forceinline__ bool two_hits(const TraceParams& P, uint32_t node,\n"
       "      uint32_t kind, d3 o, d3 d, double tm, double& t1, double& t2, bool& fallback) {\n"
       "    (void)P; (void)node; (void)kind; (void)tm;\n"
       "    fallback = false;\n"
    << b.str() << "  }\n};\n";
  return true;
}

// The light-list PDF value of the mixture (rt_kernel.h light_pdf: HittableList::pdf_value
// hittable.rs:115-124 over Quad/Sphere::pdf_value object.rs:492-501, 190-202), the list unrolled
// with each light's constants as literals: the same expressions in the same order.
// Straight-line code for light entry i (rt_kernel.h light_entry_pdf): sets `pv`.
bool gen_light_entry(const rtf::FlatScene& F, size_t i, int nest, int sphere0, int& uid,
                     std::ostringstream& o, std::string* why) {
  const std::vector<uint32_t>& L = F.lights;
  if (i >= F.light_offs.size() || F.light_offs[i] + 4 > L.size()) {
    *why = "malformed light table";
    return false;
  }
  const size_t off = F.light_offs[i];
  const uint32_t type = L[off] & 0xffu;
  o << "    // light " << i << "\n    pv = 0.0;\n";
  if (type == RTL_LLIST) {  // a nested HittableList: left fold of its children, times 1/len
    if (nest <= 0) {
      *why = "light lists nested too deep";
      return false;
    }
    const uint32_t n = L[off] >> 8, first = L[off + 1];
    const std::string acc = "lsum" + std::to_string(uid++);
    o << "    {\n    wt " << acc << " = 0;\n";
    for (uint32_t k = 0; k < n; ++k) {
      if (!gen_light_entry(F, first + k, nest - 1, sphere0, uid, o, why)) return false;
      o << "    " << acc << (k == 0 ? " = pv;\n" : " = " + acc + " + pv;\n");
    }
    o << "    pv = " << acc << " * (wt)" << lit(pd(L, off, 0)) << ";\n    }\n";
  } else if (type == RTL_QUAD) {
    o << "    {\n      C.inc(RT_OP_LIGHT_PDF_QUAD);\n      double t = 0.0;\n      bool hq;\n";
    const uint32_t axis = RTL_QUAD_AXIS(L[off]);
    if (axis) {
      const int k = (int)axis - 1;
      const char* r[3] = {"0.", "0.", "0."};
      const char* rc[3] = {"rcp_nr1(dir.x)", "rcp_nr1(dir.y)", "rcp_nr1(dir.z)"};
      r[k] = rc[k];
      o << "      hq = aquad_test<COUNT, " << k << ">(AQuad{" << L[off] << "u";
      for (int j = 0; j < 5; ++j) o << ", " << lit(pd(L, off, RTL_LQUAD_AXIS_D + j));
      o << "}, origin, dir, mk(" << r[0] << ", " << r[1] << ", " << r[2]
        << "), 0.001, kInf, t, C);\n";
    } else {
      o << "      hq = quad_test<COUNT>((kptr)P.lights + " << off
        << "u, origin, dir, 0.001, kInf, t, C);\n";
    }
    o << "      const wt q = quad_light_w(dir, t, "
      << lit3(pd(L, off, 0), pd(L, off, 1), pd(L, off, 2)) << ", " << lit(pd(L, off, 7))
      << ");\n      pv = hq ? q : (wt)0;\n    }\n";
  } else if (type == RTL_SPHERE) {
    const std::string c = lit3(pd(L, off, 0), pd(L, off, 1), pd(L, off, 2));
    const std::string r = lit(pd(L, off, 3));
    o << "    {\n      C.inc(RT_OP_LIGHT_PDF_SPHERE);\n      bool hs;\n"
         "      if (COUNT) {\n        double t = 0.0;\n"
         "        hs = sphere_test<COUNT>((kptr)P.lights + " << off
      << "u, origin, dir, 0.0, 0.001, kInf, t, C);\n      } else {\n"
         "        const d3 oc = origin - " << c << ";\n"
         "        const double a = dot(dir, dir);\n"
         "        const double half_b = dot(oc, dir);\n"
         "        const double r = " << r << ";\n"
         "        const double c = dot(oc, oc) - r * r;\n"
         "        const double disc = fma(half_b, half_b, -(a * c));\n"
         "        const double c1 = fma(0.001, a, half_b);\n"
         "        hs = !(disc < 0.0) & ((c1 < 0.0) | (disc > c1 * c1));\n      }\n"
         "      double cos_max = 0.0;\n";
    if ((int)i == sphere0) {
      o << "      cos_max = cos_sl0;\n";
    } else {
      o << "      if (hs) {\n        d3 cmo = " << c << " - origin;\n        double r = " << r
        << ";\n        cos_max = sqrt_nr(1.0 - r * r / dot(cmo, cmo));\n      }\n";
    }
    o << "      const wt q = sphere_light_w(cos_max);\n      pv = hs ? q : (wt)0;\n    }\n";
  }
  return true;
}

bool gen_lights_pdf(const rtf::FlatScene& F, std::ostringstream& o, std::string* why) {
  const std::vector<uint32_t>& L = F.lights;
  o << "  template <bool COUNT>\n"
       "  static __device__ __forceinline__ wt lights_pdf(const TraceParams& P, d3 origin, d3 dir,\n"
       "      double cos_sl0, Ctr<COUNT>& C) {\n"
       "    (void)P; (void)origin; (void)dir; (void)cos_sl0;\n"
       "    wt sum = 0, pv = 0;\n";
  int sphere0 = -1;  // rt_device.hip sphere_light0: the first sphere light
  for (size_t i = 0; i < F.light_offs.size(); ++i)
    if ((L[F.light_offs[i]] & 0xffu) == RTL_SPHERE) {
      sphere0 = (int)i;
      break;
    }
  const size_t n = F.hdr.n_lights;  // the interpreter's P.n_lights (top-level entries)
  if (n > F.light_offs.size()) {
    *why = "malformed light table";
    return false;
  }
  int uid = 0;
  for (size_t i = 0; i < n; ++i) {
    if (!gen_light_entry(F, i, RTL_LIGHT_NEST, sphere0, uid, o, why)) return false;
    o << (i == 0 ? "    sum = pv;\n" : "    sum = sum + pv;\n");
  }
  if (F.hdr.lights_is_list && n) {
    o << "    return sum * (wt)" << lit(1.0 / (double)n) << ";\n  }\n";
  } else {
    o << "    return sum;\n  }\n";
  }
  return true;
}

}  // namespace

std::string generate(const rtf::FlatScene& F, std::string* why) {
  const std::vector<uint32_t>& N = F.nodes;
  if (F.hdr.nested_volumes) {
    *why = "ConstantMedium nested in a volume boundary: the interpreter kernel walks it";
    return "";
  }
  if (N.size() > kMaxWords) {
    *why = "node array too large for the packed winner code";
    return "";
  }
  Gen G(N);
  std::ostringstream& o = G.o;
  std::ostringstream pre;  // policies the walker refers to (generated volume boundary queries)
  o << "struct TravGen {\n"
       "  template <bool COUNT, bool VOL, bool BVH, bool VOLB, bool VOLI>\n"
       "  static __device__ __forceinline__ bool world(const TraceParams& P, d3& ro, d3& rd, double tm,\n"
       "      double& t_out, uint32_t& hn, int& hf, Rng& g, Ctr<COUNT>& C) {\n"
       "    const kptr N = (kptr)P.nodes;\n"
       "    (void)N; (void)tm; (void)g;\n"
       "    const double tmin = 0.0001;  // render.rs:267\n"
       "    double closest = kInf, t = 0.0;\n"
       "    double rx = 0.0, ry = 0.0, rz = 0.0;\n"
       "    bool h = false;\n"
       "    uint32_t code = 0u;  // (record + 1) | frame_id << 24 of the closest hit\n"
       "    uint32_t bhn = 0u;   // BVH subtree winner (code == kBvhCode)\n"
       "    int bhf = -1;\n"
       "    d3 o = ro, d = rd;\n";
  size_t node = F.hdr.root;
  int frame = -1;
  bool wlen = false;  // |rd| emitted for the world frame's volumes
  for (size_t guard = 0;; ++guard) {
    if (node + 4 > N.size() || guard > N.size()) {
      *why = "malformed node sequence";
      return "";
    }
    const uint32_t h0 = N[node], ty = h0 & 0xffu;
    o << "    // record " << node << "\n";
    if (ty == RTL_QUAD) {
      G.quad(node, frame);
      node = N[node + 3];
    } else if (ty == RTL_QUADS) {
      const uint32_t cnt = h0 >> 8;
      for (uint32_t k = 0; k < cnt; ++k) G.quad(node + 4 + (size_t)k * RTL_QUAD_WORDS, frame);
      node = N[node + 1];
    } else if (ty == RTL_SPHERE) {
      G.sphere(node, frame);
      node = N[node + 3];
    } else if (ty == RTL_TRANSLATE || ty == RTL_ROTATE_Y) {
      G.xform(node);
      frame = (int)node;
      node = N[node + 3];
    } else if (ty == RTL_EXIT) {
      // frame_ray: the parent frame's ray, recomputed from the world ray through its chain
      frame = (int)N[node + 2];
      o << "    o = ro;\n    d = rd;\n";
      G.frame_changed();
      if (frame >= 0) {
        const uint32_t len = N[(size_t)frame + 2];
        const bool lng = (N[(size_t)frame] & RTL_XFORM_LONG) != 0u;
        for (uint32_t k = 0; k < len; ++k)
          G.xform(lng ? N[(size_t)N[(size_t)frame + 4] + k] : N[(size_t)frame + 4 + k]);
      }
      node = N[node + 3];
    } else if (ty == RTL_VOLUME) {
      // ConstantMedium (constant_medium.rs:41-95): the interpreter's boundary walks; the world
      // frame's volumes share one |rd| (constant_medium.rs:73 r.direction().length())
      const bool vt = gen_volume_two_hits(N, node, pre);
      if (frame < 0 && !wlen) {
        o << "    const double wlen = sqrt_nr(dot(rd, rd));\n";
        wlen = true;
      }
      o << "    h = volume_hit<COUNT, true, BVH, VOLI"
        << (vt ? ", VolTwo_" + std::to_string(node) : std::string()) << ">(P, " << node
        << "u, make_uint4(" << N[node] << "u, "
        << N[node + 1] << "u, " << N[node + 2] << "u, " << N[node + 3] << "u), ro, rd, tm, o, d, "
        << frame << ", tmin, closest, t, g, C" << (frame < 0 ? ", &wlen" : "") << ");\n"
        << "    closest = h ? t : closest;\n    code = h ? " << G.code(node, frame) << "u : code;\n";
      ++G.prims;
      node = N[node + 1];
    } else if (ty == RTL_BVH) {
      // BvhNode subtree [node, skip) per lane (rt_kernel.h traverse<UNI> RTL_BVH)
      o << "    if (BVH) {\n      double tb;\n      uint32_t bn = 0u;\n      int bf = -1;\n"
        << "      bool sub;\n";
      o << "      sub = bvh_subtree<true, COUNT, VOLB, BVH>(P, " << node << "u, " << N[node + 1]
        << "u, " << N[node + 3] << "u, ro, rd, tm, o, d, " << frame
        << ", tmin, closest, tb, bn, bf, g, C);\n";
      o << "      closest = sub ? tb : closest;\n      code = sub ? " << kBvhCode << "u : code;\n"
        << "      bhn = sub ? bn : bhn;\n      bhf = sub ? bf : bhf;\n    }\n";
      G.bvh = true;
      ++G.prims;
      node = N[node + 1];
    } else if (ty == RTL_DUP) {
      node = N[node + 1];
    } else if (ty == RTL_OTHER) {
      node = N[node + 1];
    } else if (ty == RTL_END) {
      break;
    } else {
      *why = "record type " + std::to_string(ty) + " is not generated";
      return "";
    }
    if (G.prims > kMaxPrims) {
      *why = "more than " + std::to_string(kMaxPrims) + " primitive tests per world query";
      return "";
    }
    if (G.frames.size() > kMaxFrames) {
      *why = "more than " + std::to_string(kMaxFrames) + " instance frames";
      return "";
    }
  }
  o << "    t_out = closest;\n"
       "    const bool hit = code != 0u;\n"
       "    uint32_t rn = (code & 0xffffffu) - 1u;\n"
       "    const uint32_t fid = code >> 24;\n"
       "    int fr = -1;\n";
  for (size_t id = 1; id < G.frames.size(); ++id)
    o << "    fr = fid == " << id << "u ? " << G.frames[id] << " : fr;\n";
  if (G.bvh)
    o << "    rn = code == " << kBvhCode << "u ? bhn : rn;\n"
      << "    fr = code == " << kBvhCode << "u ? bhf : fr;\n";
  o << "    hn = hit ? rn : hn;\n"
       "    hf = hit ? fr : hf;\n"
       "    return hit;\n"
       "  }\n";
  // The hit record's frame (rt_kernel.h TravInterpN::frame_in / frame_out): every frame the walk
  // can report, its chain unrolled with literals (the same translate/rotate arithmetic as
  // xform_in / xform_out); frames inside BVH subtrees take the interpreter's chain walk.
  std::ostringstream fi, fo;
  for (size_t id = 1; id < G.frames.size(); ++id) {
    const size_t f = (size_t)G.frames[id];
    const uint32_t len = N[f + 2];
    const bool lng = (N[f] & RTL_XFORM_LONG) != 0u;
    std::vector<size_t> chain;
    for (uint32_t k = 0; k < len; ++k) chain.push_back(lng ? N[(size_t)N[f + 4] + k] : N[f + 4 + k]);
    fi << "    " << (id > 1 ? "} else if" : "if") << " (hf == " << f << ") {\n";
    fo << "    " << (id > 1 ? "} else if" : "if") << " (hf == " << f << ") {\n";
    for (size_t x : chain) {
      if ((N[x] & 0xffu) == RTL_TRANSLATE)
        fi << "      translate_in(" << lit3(pd(N, x, 2), pd(N, x, 3), pd(N, x, 4)) << ", o);\n";
      else
        fi << "      rotate_y_in(" << lit(pd(N, x, 2)) << ", " << lit(pd(N, x, 3)) << ", o, d);\n";
    }
    for (size_t k = chain.size(); k-- > 0;) {
      const size_t x = chain[k];
      if ((N[x] & 0xffu) == RTL_TRANSLATE)
        fo << "      translate_out(" << lit3(pd(N, x, 2), pd(N, x, 3), pd(N, x, 4)) << ", p);\n";
      else
        fo << "      rotate_y_out(" << lit(pd(N, x, 2)) << ", " << lit(pd(N, x, 3)) << ", p, n);\n";
    }
  }
  // without BVH subtrees the frames above are all the walk can report
  const bool many = G.frames.size() > 1;
  const std::string more = G.bvh ? (many ? "    } else if (hf >= 0) {\n" : "    if (hf >= 0) {\n") : "";
  const std::string rest_in = G.bvh ? "      frame_ray(Nd, hf, wo, wd, o, d);\n    }\n" : (many ? "    }\n" : "");
  const std::string rest_out = G.bvh ? "      rtk::frame_out(Nd, hf, p, n);\n    }\n" : (many ? "    }\n" : "");
  o << "  template <class TP>\n"
       "  static __device__ __forceinline__ void frame_in(TP Nd, int hf, d3 wo, d3 wd, d3& o, d3& d) {\n"
       "    (void)Nd;\n    o = wo;\n    d = wd;\n"
    << fi.str() << more << rest_in << "  }\n"
    << "  template <class TP>\n"
       "  static __device__ __forceinline__ void frame_out(TP Nd, int hf, d3& p, d3& n) {\n"
       "    (void)Nd; (void)hf; (void)p; (void)n;\n"
    << fo.str() << more << rest_out << "  }\n";
  if (!gen_lights_pdf(F, o, why)) return "";
  // the scene's material kinds and light-list shape (rt_kernel.h kScene): shading code for what
  // the scene lacks is compiled out. RT_NO_SCENE_SET=1 (diagnostics, A/B) keeps every case.
  uint32_t sc = 0u;
  for (size_t m = 0; m + RTL_MAT_WORDS <= F.mats.size(); m += RTL_MAT_WORDS) {
    const uint32_t kind = F.mats[m] & 0xffu;
    if (kind == RT_MAT_METAL) sc |= RTL_SC_METAL;
    if (kind == RT_MAT_DIELECTRIC) sc |= RTL_SC_DIELECTRIC;
    if (kind == RT_MAT_DIFFUSE_LIGHT) sc |= RTL_SC_LIGHT;
  }
  if (F.hdr.n_lights) sc |= RTL_SC_LIGHTS;
  if (F.hdr.lights_nested) sc |= RTL_SC_LLIST;
  for (uint32_t off : F.light_offs) {
    const uint32_t ty = off < F.lights.size() ? (F.lights[off] & 0xffu) : 0u;
    if (ty == RTL_SPHERE) sc |= RTL_SC_LSPHERE;
    else if (ty != RTL_QUAD && ty != RTL_LLIST) sc |= RTL_SC_LOTHER;
  }
  const char* any = std::getenv("RT_NO_SCENE_SET");
  if (any && *any && *any != '0') sc = RTL_SC_ANY;
  char scb[64];
  std::snprintf(scb, sizeof scb, "  static constexpr uint32_t kScene = 0x%xu;\n", sc);
  o << scb << "};\n";
  return pre.str() + o.str();
}

Flags product_flags(const rtf::FlatScene& F, bool staged) {
  Flags f;
  f.vol = (F.hdr.has_volume | F.hdr.has_isotropic) != 0;
  f.tex = F.hdr.has_textures != 0;
  f.bvh = F.hdr.has_bvh != 0;
  f.staged = staged && !f.bvh;
  // rt_device.hip: BVH scenes whose volumes all sit outside BVH subtrees run the per-lane walker
  // without its volume branch, and without the two-walk interpreter when every boundary is a
  // one-walk sphere
  const bool novolb = f.bvh && f.vol && !F.hdr.volume_in_bvh;
  f.volb = novolb ? false : f.vol;
  f.voli = !(novolb && F.hdr.volumes_one_walk_spheres);
  return f;
}

std::string kernel_source(const std::string& walker, const Flags& f) {
  auto b = [](bool v) { return v ? "true" : "false"; };
  std::ostringstream src;
  src << "#include \"rt_kernel.h\"\nnamespace rtk {\n"
      << walker
      << "}  // namespace rtk\nusing namespace rtk;\n"
         "extern \"C\" __global__ __launch_bounds__(BlockOf<" << b(f.bvh) << ">::value, "
         "(MinWaves<" << b(f.vol) << ", " << b(f.tex) << ", " << b(f.bvh)
      << ", true>::value)) void rt_trace_jit(TraceParams P) {\n"
      << "  trace_body<false, " << b(f.vol) << ", " << b(f.tex) << ", " << b(f.bvh) << ", "
      << b(f.staged) << ", " << b(f.volb) << ", " << b(f.voli) << ", TravGen>(P);\n}\n";
  return src.str();
}

int compile(const std::string& src, const std::string& arch, std::vector<char>* code,
            std::string* log, bool use_cache) {
  // hiprtc provides the HIP device runtime and the fixed-width integer types itself: the
  // headers' <hip/hip_runtime.h> and <stdint.h> resolve to these stubs
  static const char* kStdint =
      "#pragma once\ntypedef unsigned char uint8_t; typedef unsigned short uint16_t;\n"
      "typedef unsigned int uint32_t; typedef unsigned long uint64_t; typedef signed char int8_t;\n"
      "typedef short int16_t; typedef int int32_t; typedef long int64_t;\n";
  std::vector<const char*> hs, hn;
  // diagnostics (register-allocation work without rebuilding the library): RT_JIT_SRC_DIR, a
  // ':'-separated list of directories, replaces the embedded headers by the files found there
  static thread_local std::vector<std::string> override_text;
  override_text.assign(kJitSrcCount, std::string());
  const char* src_dirs = std::getenv("RT_JIT_SRC_DIR");
  for (int k = 0; k < kJitSrcCount; ++k) {
    const char* text = kJitSrcText[k];
    if (src_dirs && *src_dirs) {
      std::istringstream dirs(src_dirs);
      for (std::string d; std::getline(dirs, d, ':');) {
        std::ifstream f(d + "/" + kJitSrcNames[k], std::ios::binary);
        if (!f) continue;
        std::ostringstream buf;
        buf << f.rdbuf();
        override_text[k] = buf.str();
        text = override_text[k].c_str();
        break;
      }
    }
    hs.push_back(text);
    hn.push_back(kJitSrcNames[k]);
  }
  hs.push_back(kStdint);
  hn.push_back("stdint.h");
  hs.push_back("#pragma once\n");
  hn.push_back("hip/hip_runtime.h");
  const std::string off = "--offload-arch=" + arch;
  // the ahead-of-time build's arithmetic flags (Makefile HIPFLAGS): contraction off, so every
  // fma is the one written in rt_kernel.h and the generated walker computes the same bits
  // No VGPR spills into AGPRs: the hiprtc a process binds to is whichever libhiprtc is loaded
  // first (PyTorch's bundled ROCm 7.0 comgr once torch is imported), and that compiler put 3
  // AGPRs on top of the 168 VGPRs of the 768-thread BVH kernel: 171 registers x 3 waves per SIMD
  // exceed the 512-entry file, so the CP rejected the dispatch (REGISTER_INVALID, reported as
  // HSA_STATUS_ERROR_INVALID_ISA) and aborted the queue. Spills then go to scratch instead.
  std::vector<const char*> opts = {off.c_str(), "-O3", "-std=c++17", "-ffp-contract=off",
                                   "-fno-gpu-flush-denormals-to-zero", "-mllvm",
                                   "-amdgpu-spill-vgpr-to-agpr=0"};
#ifndef RT_JIT_MLICM
  // No machine-level loop-invariant hoisting: it lifts the f64 literal constants of the math
  // inside the path loop (the log of ConstantMedium, sphere_uv's acos/atan2, polynomial
  // coefficients) out of the loop into VGPR pairs that stay live across every bounce, and the
  // register allocator then spills them rather than rematerialise them (final_scene: 168 VGPRs
  // + 24 spilled, cornell_smoke 128 + 10; without: 148 + 0 and 117 + 0). DESIGN.md §4.1b.
  opts.push_back("-mllvm");
  opts.push_back("-disable-machine-licm");
#endif
#ifndef RT_JIT_SLP
  // No SLP vectorisation: it packed the quad test's four accept compares (and the walks' hit
  // flags) into 16-bit lane vectors (v_cndmask 0/1, shifts, v_bitop3, a compare) instead of
  // combining them as lane masks; nothing in these kernels profits from it (the packed f32 box
  // arithmetic is written with vector types). C4 -1.3 %, C3 -0.4 %, C2 +-0, images identical
  // (profiles/r04_ab17_cN.log).
  opts.push_back("-fno-slp-vectorize");
#endif
  // build knobs of this library (ablation / occupancy variants, Makefile) apply to its
  // run-time kernels too
#define RTJ_STR2(x) #x
#define RTJ_STR(x) RTJ_STR2(x)
#ifdef RT_POOL_SI
  opts.push_back("-DRT_POOL_SI=" RTJ_STR(RT_POOL_SI));
#endif
#ifdef RT_MIN_WAVES
  opts.push_back("-DRT_MIN_WAVES=" RTJ_STR(RT_MIN_WAVES));
#endif
#ifdef RT_MIN_WAVES_BVH
  opts.push_back("-DRT_MIN_WAVES_BVH=" RTJ_STR(RT_MIN_WAVES_BVH));
#endif
#ifdef RT_MIN_WAVES_GEN
  opts.push_back("-DRT_MIN_WAVES_GEN=" RTJ_STR(RT_MIN_WAVES_GEN));
#endif
#ifdef RT_MIN_WAVES_GEN_VOL
  opts.push_back("-DRT_MIN_WAVES_GEN_VOL=" RTJ_STR(RT_MIN_WAVES_GEN_VOL));
#endif
#ifdef RT_BLOCK_BVH
  opts.push_back("-DRT_BLOCK_BVH=" RTJ_STR(RT_BLOCK_BVH));
#endif
#ifdef RT_PROF
  opts.push_back("-DRT_PROF");
#endif
#ifdef RT_ABL_TRAV2
  opts.push_back("-DRT_ABL_TRAV2");
#endif
#ifdef RT_ABL_NOLPDF
  opts.push_back("-DRT_ABL_NOLPDF");
#endif
#ifdef RT_ABL_LPDF2
  opts.push_back("-DRT_ABL_LPDF2");
#endif
#ifdef RT_ABL_HIT2
  opts.push_back("-DRT_ABL_HIT2");
#endif
#ifdef RT_ABL_TWICE_BVH
  opts.push_back("-DRT_ABL_TWICE_BVH=" RTJ_STR(RT_ABL_TWICE_BVH));
#endif
#ifdef RT_ABL_NOXS
  opts.push_back("-DRT_ABL_NOXS");
#endif
#ifdef RT_ABL_SEED2
  opts.push_back("-DRT_ABL_SEED2");
#endif
#ifdef RT_ABL_FRESH2
  opts.push_back("-DRT_ABL_FRESH2");
#endif
#ifdef RT_EXACT_PROBE
  opts.push_back("-DRT_EXACT_PROBE");
#endif
#ifdef RT_ABL_LEAF2
  opts.push_back("-DRT_ABL_LEAF2");
#endif
#ifdef RT_ABL_NOISE2
  opts.push_back("-DRT_ABL_NOISE2");
#endif
#ifdef RT_ABL_RUV2
  opts.push_back("-DRT_ABL_RUV2");
#endif
#ifdef RT_ABL_BUDGET
  opts.push_back("-DRT_ABL_BUDGET=" RTJ_STR(RT_ABL_BUDGET));
#endif
#ifdef RT_ABL_RNG2
  opts.push_back("-DRT_ABL_RNG2");
#endif
  // diagnostics: extra compiler options, space separated (register-allocation A/B)
  std::vector<std::string> extra;
  if (const char* e = std::getenv("RT_JIT_OPTS")) {
    std::istringstream in(e);
    for (std::string w; in >> w;) extra.push_back(w);
  }
  for (const std::string& w : extra) opts.push_back(w.c_str());
  // The code-object cache (cache_path): a translation unit compiled before with the same
  // headers, options and target is loaded instead of compiled again.
  const std::string cached = cache_path(src, hs, opts);
  if (!cached.empty() && use_cache) {
    std::ifstream f(cached, std::ios::binary);
    if (f) {
      code->assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
      if (!code->empty()) {
        *log = "code-object cache: " + cached;
        return 0;
      }
    }
  }
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, src.c_str(), "rt_trace_jit.hip", (int)hs.size(), hs.data(),
                          hn.data()) != HIPRTC_SUCCESS) {
    *log = "hiprtcCreateProgram failed";
    return RT_ERR_HIP;
  }
  const hiprtcResult rc = hiprtcCompileProgram(prog, (int)opts.size(), opts.data());
  size_t n = 0;
  hiprtcGetProgramLogSize(prog, &n);
  std::string plog(n, '\0');
  if (n) hiprtcGetProgramLog(prog, &plog[0]);
  if (rc != HIPRTC_SUCCESS) {
    hiprtcDestroyProgram(&prog);
    *log = "hiprtc: " + plog;
    return RT_ERR_HIP;
  }
  size_t code_size = 0;
  hiprtcGetCodeSize(prog, &code_size);
  code->resize(code_size);
  hiprtcGetCode(prog, code->data());
  hiprtcDestroyProgram(&prog);
  const char* wr = std::getenv("RT_JIT_CACHE_WRITE");
  if (!cached.empty() && wr && std::strcmp(wr, "1") == 0) {  // populate the cache (tools/jit_cache_fill.py)
    const std::string tmp = cached + ".tmp" + std::to_string((unsigned long)getpid());
    if (FILE* f = std::fopen(tmp.c_str(), "wb")) {
      const bool ok = std::fwrite(code->data(), 1, code->size(), f) == code->size();
      std::fclose(f);
      if (ok) std::rename(tmp.c_str(), cached.c_str());
      else std::remove(tmp.c_str());
    }
  }
  if (const char* dump = std::getenv("RT_JIT_DUMP")) {  // diagnostics: the code object as built
    if (FILE* f = std::fopen(dump, "wb")) {
      std::fwrite(code->data(), 1, code->size(), f);
      std::fclose(f);
    }
  }
  return 0;
}

namespace {
// The module cache: per (device, source) the kernel, the number of scenes holding it and the
// time of its last hand-out (for evicting the least recently used unheld modules).
struct Entry {
  Kernel k;
  int holds = 0;
  uint64_t used = 0;
};
std::mutex g_mu;
std::map<std::pair<int, std::string>, Entry> g_cache;
uint64_t g_tick = 0;

void evict_idle_locked() {
  for (;;) {
    int idle = 0;
    auto oldest = g_cache.end();
    for (auto it = g_cache.begin(); it != g_cache.end(); ++it) {
      if (it->second.holds > 0) continue;
      ++idle;
      if (oldest == g_cache.end() || it->second.used < oldest->second.used) oldest = it;
    }
    if (idle <= kIdleModules) return;
    int prev = -1;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(oldest->first.first);
    (void)hipModuleUnload(oldest->second.k.mod);
    if (prev >= 0) (void)hipSetDevice(prev);
    g_cache.erase(oldest);
  }
}
}  // namespace

void release_kernel(const Kernel& k) {
  if (!k.mod) return;
  std::lock_guard<std::mutex> lock(g_mu);
  for (auto& kv : g_cache)
    if (kv.second.k.mod == k.mod && kv.second.holds > 0) {
      --kv.second.holds;
      break;
    }
  evict_idle_locked();
}

int get_kernel(const std::string& walker, int device, const Flags& f, Kernel* out,
               std::string* log) {
  const std::string s = kernel_source(walker, f);
  std::lock_guard<std::mutex> lock(g_mu);
  // compile() reads RT_JIT_SRC_DIR's headers and RT_JIT_OPTS's options when set (diagnostics):
  // part of the module's identity, so an A/B in one process gets one module per setting
  const char* src_dirs = std::getenv("RT_JIT_SRC_DIR");
  const char* jit_opts = std::getenv("RT_JIT_OPTS");
  auto key = std::make_pair(device, s + "//" + (src_dirs ? src_dirs : "") + "//" +
                                        (jit_opts ? jit_opts : ""));
  auto it = g_cache.find(key);
  if (it != g_cache.end()) {
    ++it->second.holds;
    it->second.used = ++g_tick;
    *out = it->second.k;
    return 0;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) {
    *log = "hipGetDeviceProperties failed";
    return RT_ERR_HIP;
  }
  std::string arch = prop.gcnArchName;
  const size_t colon = arch.find(':');  // "gfx950:sramecc+:xnack-" -> gfx950
  if (colon != std::string::npos) arch.resize(colon);
  std::vector<char> code;
  int rc = compile(s, arch, &code, log);
  if (rc != 0) return rc;
  Kernel k;
  k.cached = log->rfind("code-object cache", 0) == 0;
  auto load = [&]() {
    if (k.mod) (void)hipModuleUnload(k.mod);
    k.mod = nullptr;
    k.fn = nullptr;
    const bool ok = hipModuleLoadData(&k.mod, code.data()) == hipSuccess &&
                    hipModuleGetFunction(&k.fn, k.mod, "rt_trace_jit") == hipSuccess;
    // a failed load leaves its error as the thread's last error ("device kernel image is
    // invalid"), which the render's launch check (hipGetLastError) would then report
    if (!ok) (void)hipGetLastError();
    return ok;
  };
  bool loaded = load();
  if (!loaded && k.cached) {
    // a cache entry that does not load (damaged, incompatible, or a transient failure such as
    // an out-of-memory error): compile the source for this process instead of leaving the scene
    // on the interpreter (a silent slowdown). The file is left alone: it pins the benchmark
    // kernels to the build-time compiler, and a transient failure must not
    // make every later process compile differently.
    const std::string path = log->substr(std::string("code-object cache: ").size());
    std::fprintf(stderr, "rt_jit: cached code object %s failed to load; recompiling (file kept)\n",
                 path.c_str());
    rc = compile(s, arch, &code, log, false);
    if (rc != 0) return rc;
    k.cached = false;
    *log = "recompiled (cached code object failed to load)";
    loaded = load();
  }
  if (!loaded) {
    *log = "hipModuleLoadData / hipModuleGetFunction failed";
    return RT_ERR_HIP;
  }
  if (hipFuncGetAttribute(&k.regs, HIP_FUNC_ATTRIBUTE_NUM_REGS, k.fn) != hipSuccess ||
      hipFuncGetAttribute(&k.max_threads, HIP_FUNC_ATTRIBUTE_MAX_THREADS_PER_BLOCK, k.fn) !=
          hipSuccess ||
      hipFuncGetAttribute(&k.static_lds, HIP_FUNC_ATTRIBUTE_SHARED_SIZE_BYTES, k.fn) != hipSuccess ||
      hipFuncGetAttribute(&k.scratch, HIP_FUNC_ATTRIBUTE_LOCAL_SIZE_BYTES, k.fn) != hipSuccess) {
    *log = "hipFuncGetAttribute failed on the scene-specialised kernel";
    return RT_ERR_HIP;
  }
  Entry e;
  e.k = k;
  e.holds = 1;
  e.used = ++g_tick;
  g_cache.emplace(key, e);
  *out = k;
  return 0;
}

}  // namespace rtj
