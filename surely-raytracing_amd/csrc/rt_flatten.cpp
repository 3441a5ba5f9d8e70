// rt_flatten.cpp — validate an rt_scene_blob and flatten it for the device.
//
// Input: the prefix-serialised object tree of the reference scene (HittableList / BvhNode /
// Sphere / Quad / Translate / RotateY / ConstantMedium, include/rt_mi355x.h). Output: one
// threaded pre-order word array (rt_layout.h) whose sequential walk reproduces the reference's
// recursive visiting order (hittable.rs:88-109, 216-236; transform.rs:57-135;
// constant_medium.rs:41-95), plus fp32 material / texture / Perlin / light tables.
// Shared subtrees (Arc<Object> clones, BVH span-1 duplicate leaves hittable.rs:161-162) are
// emitted once per reference, exactly as often as the reference would visit them.
#include "rt_flatten.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <memory>

#include <xmmintrin.h>

namespace rtf {

namespace {

struct Node {
  int tag = 0;
  int64_t mat = -1;
  int64_t moving = 0;
  double f[32] = {0};  // tag-specific payload (see read_node)
  double bbox[6] = {0};
  std::vector<std::unique_ptr<Node>> kids;
};

struct Reader {
  const uint64_t* s;
  uint64_t n, pos;
  bool err = false;
  std::string msg;
  int64_t i() {
    if (pos >= n) return fail("truncated blob"), 0;
    return (int64_t)s[pos++];
  }
  double f() {
    if (pos >= n) return fail("truncated blob"), 0.0;
    double d;
    std::memcpy(&d, &s[pos++], 8);
    return d;
  }
  void fail(const std::string& m) {
    if (!err) msg = m;
    err = true;
  }
};

// The axis-aligned quad test's planar coordinate is a(y) = fl(fl(y - q) * c), with y the hit
// point's coordinate along u or v, and it accepts when !(a < 0) & !(1 < a) (NaN accepts,
// object.rs:473). For finite q and finite c != 0, a(y) is monotone in y (both roundings are), so
// the accepted finite y form one interval [lo, hi] of doubles and the device compares y with
// those two bounds instead of forming a (rt_layout.h). lo/hi are found by bisection over the
// doubles' order; false (keep the general test) for any other q, c.
bool accept_interval(double q, double c, double& lo, double& hi) {
  if (!std::isfinite(q) || !std::isfinite(c) || c == 0.0) return false;
  // the device arithmetic: IEEE f64, round to nearest, no flush of subnormals (whatever the
  // calling process set in MXCSR)
  struct Csr {
    unsigned v = _mm_getcsr();
    Csr() { _mm_setcsr(v & ~0x8040u); }  // FTZ, DAZ off
    ~Csr() { _mm_setcsr(v); }
  } csr;
  auto a_of = [&](double y) {
    volatile double x = y - q;
    volatile double a = x * c;
    return (double)a;
  };
  auto key = [](double v) {  // order-preserving integer key (+0 and -0 share 0)
    int64_t b;
    std::memcpy(&b, &v, 8);
    return b >= 0 ? b : INT64_MIN - b;
  };
  auto val = [](int64_t k) {
    const int64_t b = k >= 0 ? k : INT64_MIN - k;
    double v;
    std::memcpy(&v, &b, 8);
    return v;
  };
  const int64_t kmin = key(-HUGE_VAL), kmax = key(HUGE_VAL);
  // the first key where a predicate that is monotone over [kmin, kmax] turns true (kmax + 1: never)
  auto first_true = [&](auto pred) {
    int64_t l = kmin, h = kmax + 1;
    while (l < h) {
      const int64_t m = l + (h - l) / 2;
      if (pred(val(m))) h = m; else l = m + 1;
    }
    return h;
  };
  int64_t klo, khi;
  if (c > 0.0) {  // a non-decreasing: a >= 0 from klo on, a <= 1 up to khi
    klo = first_true([&](double y) { return !(a_of(y) < 0.0); });
    khi = first_true([&](double y) { return 1.0 < a_of(y); }) - 1;
  } else {        // a non-increasing: a <= 1 from klo on, a >= 0 up to khi
    klo = first_true([&](double y) { return !(1.0 < a_of(y)); });
    khi = first_true([&](double y) { return a_of(y) < 0.0; }) - 1;
  }
  // y = q gives a = 0, so the interval holds q and its bounds are finite
  if (!(klo <= key(q) && key(q) <= khi) || klo <= kmin || khi >= kmax) return false;
  lo = val(klo);
  hi = val(khi);
  // the bounds and their neighbours outside, checked directly against the predicate
  auto acc = [&](double y) { const double a = a_of(y); return !(a < 0.0) && !(1.0 < a); };
  return acc(lo) && acc(hi) && !acc(val(klo - 1)) && !acc(val(khi + 1));
}

std::unique_ptr<Node> read_node(Reader& r, int depth) {
  if (depth > 256) {
    r.fail("object tree deeper than 256");
    return nullptr;
  }
  auto nd = std::make_unique<Node>();
  nd->tag = (int)r.i();
  auto bbox = [&]() {
    for (int k = 0; k < 6; ++k) nd->bbox[k] = r.f();
  };
  switch (nd->tag) {
    case RT_OBJ_LIST: {
      int64_t cnt = r.i();
      bbox();
      if (cnt < 0 || cnt > (1 << 24)) {
        r.fail("bad list length");
        return nullptr;
      }
      for (int64_t k = 0; k < cnt && !r.err; ++k) nd->kids.push_back(read_node(r, depth + 1));
      break;
    }
    case RT_OBJ_BVH:
      bbox();
      nd->kids.push_back(read_node(r, depth + 1));
      if (!r.err) nd->kids.push_back(read_node(r, depth + 1));
      break;
    case RT_OBJ_SPHERE:  // mat moving c3 radius cvec3
      nd->mat = r.i();
      nd->moving = r.i();
      for (int k = 0; k < 7; ++k) nd->f[k] = r.f();
      bbox();
      break;
    case RT_OBJ_QUAD:  // mat q3 u3 v3 n3 w3 d area
      nd->mat = r.i();
      for (int k = 0; k < 17; ++k) nd->f[k] = r.f();
      bbox();
      break;
    case RT_OBJ_TRANSLATE:  // offset3
      for (int k = 0; k < 3; ++k) nd->f[k] = r.f();
      bbox();
      nd->kids.push_back(read_node(r, depth + 1));
      break;
    case RT_OBJ_ROTATE_Y:  // sin cos
      nd->f[0] = r.f();
      nd->f[1] = r.f();
      bbox();
      nd->kids.push_back(read_node(r, depth + 1));
      break;
    case RT_OBJ_VOLUME:  // mat neg_inv_density
      nd->mat = r.i();
      nd->f[0] = r.f();
      bbox();
      nd->kids.push_back(read_node(r, depth + 1));
      break;
    default:
      r.fail("unknown object tag " + std::to_string(nd->tag));
      return nullptr;
  }
  if (r.err) return nullptr;
  for (auto& k : nd->kids)
    if (!k) {
      r.fail("bad child");
      return nullptr;
    }
  return nd;
}

// Structural equality of two object subtrees (the blob serialises a BvhNode's span-1 leaf
// (obj, obj), hittable.rs:161-162, as two copies of the same subtree).
bool same_tree(const Node& a, const Node& b) {
  if (a.tag != b.tag || a.mat != b.mat || a.moving != b.moving || a.kids.size() != b.kids.size())
    return false;
  if (std::memcmp(a.f, b.f, sizeof(a.f)) != 0 || std::memcmp(a.bbox, b.bbox, sizeof(a.bbox)) != 0)
    return false;
  for (size_t k = 0; k < a.kids.size(); ++k)
    if (!same_tree(*a.kids[k], *b.kids[k])) return false;
  return true;
}
// ConstantMedium draws a random number per boundary crossing (constant_medium.rs:75): a
// subtree holding one is not deterministic in its interval, so it is never elided.
bool has_volume_node(const Node& a) {
  if (a.tag == RT_OBJ_VOLUME) return true;
  for (auto& k : a.kids)
    if (has_volume_node(*k)) return true;
  return false;
}

// write an f64 payload value at double index k of the node starting at word p
inline void putd(std::vector<uint32_t>& w, size_t p, int k, double d) {
  std::memcpy(&w[p + 4 + 2 * (size_t)k], &d, 8);
}

struct Emitter {
  std::vector<uint32_t>& w;
  int64_t n_mats;
  std::string err;
  int status = RT_OK;
  uint32_t max_chain = 0;
  bool has_bvh = false, has_volume = false, volume_in_bvh = false, all_sphere_volumes = true;
  bool nested_volumes = false;
  int bvh_depth = 0;  // BVH subtrees enclosing the record being emitted
  size_t last_exit_end = (size_t)-1;  // end position of the most recent EXIT node
  size_t last_skip_target = (size_t)-1;

  // conservative bounds of the leaf records emitted (pre-relocation position), for rt_obvh.cpp
  std::vector<std::pair<size_t, PrimBox>> pbox;
  // transform chains longer than RTL_MAX_CHAIN (pre-relocation positions, root first)
  std::vector<std::vector<uint32_t>> long_chains;

  explicit Emitter(std::vector<uint32_t>& words, int64_t nm) : w(words), n_mats(nm) {}

  static void pad_box(PrimBox& b) {
    for (int k = 0; k < 3; ++k) {
      const double m = 1e-9 * (1.0 + std::max(std::fabs(b.lo[k]), std::fabs(b.hi[k])));
      b.lo[k] -= m;
      b.hi[k] += m;
    }
    b.valid = std::isfinite(b.lo[0] + b.lo[1] + b.lo[2] + b.hi[0] + b.hi[1] + b.hi[2]);
  }

  void fail(int code, const std::string& m) {
    if (status == RT_OK) {
      status = code;
      err = m;
    }
  }
  size_t push(uint32_t type, size_t n_words) {
    size_t pos = w.size();
    w.resize(pos + n_words, 0u);
    w[pos] = type;
    w[pos + 1] = 0xffffffffu;
    return pos;
  }
  void set_skip(size_t pos) {
    w[pos + 1] = (uint32_t)w.size();
    last_skip_target = w.size();
  }
  bool check_mat(int64_t m) {
    if (m < 0 || m >= n_mats) {
      fail(RT_ERR_BAD_BLOB, "material index out of range");
      return false;
    }
    return true;
  }
  void quad(const Node& n, bool light) {
    if (!check_mat(n.mat) && !light) return;
    size_t p = push(RTL_QUAD, light ? RTL_LQUAD_WORDS : RTL_QUAD_WORDS);
    const double* f = n.f;  // q 0-2, u 3-5, v 6-8, n 9-11, w 12-14, d 15, area 16
    const double u[3] = {f[3], f[4], f[5]}, v[3] = {f[6], f[7], f[8]}, wv[3] = {f[12], f[13], f[14]};
    // A = v x w, B = w x u (triple-product form of the planar coordinates, rt_layout.h)
    const double A[3] = {v[1] * wv[2] - v[2] * wv[1], v[2] * wv[0] - v[0] * wv[2],
                         v[0] * wv[1] - v[1] * wv[0]};
    const double B[3] = {wv[1] * u[2] - wv[2] * u[1], wv[2] * u[0] - wv[0] * u[2],
                         wv[0] * u[1] - wv[1] * u[0]};
    w[p + 2] = (uint32_t)(n.mat < 0 ? 0 : n.mat);
    const int g = light ? 0 : 6;  // general payload: d0 of a light record, d6 of a world record
    putd(w, p, g + 0, f[9]), putd(w, p, g + 1, f[10]), putd(w, p, g + 2, f[11]);
    putd(w, p, g + 3, f[15]);
    putd(w, p, g + 4, f[0]), putd(w, p, g + 5, f[1]), putd(w, p, g + 6, f[2]);
    putd(w, p, g + 7, f[16]);
    putd(w, p, g + 8, A[0]), putd(w, p, g + 9, A[1]), putd(w, p, g + 10, A[2]);
    putd(w, p, g + 12, B[0]), putd(w, p, g + 13, B[1]), putd(w, p, g + 14, B[2]);
    if (light) {
      putd(w, p, 16, u[0]), putd(w, p, 17, u[1]), putd(w, p, 18, u[2]);
      putd(w, p, 20, v[0]), putd(w, p, 21, v[1]), putd(w, p, 22, v[2]);
    }
    if (!light) {  // bounds of the four corners; the reference's Aabb spans q .. q + u + v only
      PrimBox b;
      const double q[3] = {f[0], f[1], f[2]};
      double c[4][3];
      for (int k = 0; k < 3; ++k) {
        c[0][k] = q[k], c[1][k] = q[k] + u[k], c[2][k] = q[k] + v[k], c[3][k] = (q[k] + u[k]) + v[k];
        b.lo[k] = std::min(std::min(c[0][k], c[1][k]), std::min(c[2][k], c[3][k]));
        b.hi[k] = std::max(std::max(c[0][k], c[1][k]), std::max(c[2][k], c[3][k]));
      }
      // Aabb::from_points(q, q + u + v).pad() (object.rs:427, 371-386, interval.rs:43-50)
      bool complete = true;
      for (int k = 0; k < 3; ++k) {
        double lo = std::min(c[0][k], c[3][k]), hi = std::max(c[0][k], c[3][k]);
        if (hi - lo < 0.0001) lo = lo - 0.0001 / 2., hi = hi + 0.0001 / 2.;
        for (int m = 1; m < 3; ++m) complete = complete && lo <= c[m][k] && c[m][k] <= hi;
      }
      b.ref_complete = complete;
      pad_box(b);
      pbox.push_back({p, b});
    }
    const int ax = light ? RTL_LQUAD_AXIS_D : 0;  // double index of the axis-aligned form
    // axis-aligned fast form (rt_layout.h): only when the exact-zero pattern holds
    auto single = [](const double* x) {
      int nz = -1;
      for (int c = 0; c < 3; ++c)
        if (x[c] != 0.0) {
          if (nz >= 0) return -1;
          nz = c;
        }
      return nz;
    };
    const int i = single(u), j = single(v);
    if (i < 0 || j < 0 || i == j) return;
    const int k = 3 - i - j;
    const double nk = f[9 + k];
    if (!(nk == 1.0 || nk == -1.0) || f[9 + i] != 0.0 || f[9 + j] != 0.0) return;
    if (f[15] != nk * f[k]) return;  // D = n.q = n_k q_k
    if (single(A) != i || single(B) != j) return;
    // a = (y_i - q_i) A_i and b = (y_j - q_j) B_j accept exactly on intervals of y_i and y_j
    double lo_i, hi_i, lo_j, hi_j;
    if (!accept_interval(f[i], A[i], lo_i, hi_i) || !accept_interval(f[j], B[j], lo_j, hi_j)) return;
    w[p] |= (uint32_t)(k + 1) << 8;
    putd(w, p, ax + 0, f[k]);
    if (i < j) {
      putd(w, p, ax + 1, lo_i), putd(w, p, ax + 2, hi_i), putd(w, p, ax + 3, lo_j);
      putd(w, p, ax + 4, hi_j);
    } else {
      putd(w, p, ax + 1, lo_j), putd(w, p, ax + 2, hi_j), putd(w, p, ax + 3, lo_i);
      putd(w, p, ax + 4, hi_i);
    }
  }
  void sphere(const Node& n, bool light) {
    if (!check_mat(n.mat) && !light) return;
    size_t p = push(RTL_SPHERE, RTL_SPHERE_WORDS);
    const double* f = n.f;  // c 0-2, radius 3, cvec 4-6
    w[p + 2] = (uint32_t)(n.mat < 0 ? 0 : n.mat);
    if (n.moving) w[p] |= RTL_SPHERE_MOVING;
    putd(w, p, 0, f[0]), putd(w, p, 1, f[1]), putd(w, p, 2, f[2]), putd(w, p, 3, f[3]);
    putd(w, p, 4, f[4]), putd(w, p, 5, f[5]), putd(w, p, 6, f[6]);
    putd(w, p, 7, 1.0 / f[3]);  // IEEE 1/r: outward = (p - c) / r by one residual step (rt_kernel.h)
    if (!light) {  // c +- r, and at c + cvec when moving (object.rs:88-105)
      PrimBox b;
      const double r = std::fabs(f[3]);
      for (int k = 0; k < 3; ++k) {
        const double c1 = n.moving ? f[k] + f[4 + k] : f[k];
        b.lo[k] = std::min(f[k], c1) - r;
        b.hi[k] = std::max(f[k], c1) + r;
      }
      b.ref_complete = true;
      pad_box(b);
      pbox.push_back({p, b});
    }
  }
  // RTL_VOLF_* when the boundary sequence starting at q has the one-walk form (rt_layout.h)
  uint32_t fusable_boundary(size_t q) const {
    auto ty = [&](size_t at) { return at < w.size() ? (w[at] & 0xffu) : 0xffu; };
    while (ty(q) == RTL_TRANSLATE || ty(q) == RTL_ROTATE_Y) q += RTL_XFORM_WORDS;
    uint32_t kind = 0;
    if (ty(q) == RTL_SPHERE) {
      kind = RTL_VOLF_SPHERE;
      q += RTL_SPHERE_WORDS;
    } else if (ty(q) == RTL_QUAD && RTL_QUAD_AXIS(w[q]) != 0u) {
      kind = RTL_VOLF_QUADS;
      q += RTL_QUAD_WORDS;
    } else if (ty(q) == RTL_QUADS) {
      const uint32_t cnt = w[q] >> 8;
      q += 4;
      for (uint32_t k = 0; k < cnt; ++k, q += RTL_QUAD_WORDS)
        if (ty(q) != RTL_QUAD || RTL_QUAD_AXIS(w[q]) == 0u) return 0u;
      kind = RTL_VOLF_QUADS;
    } else {
      return 0u;
    }
    while (ty(q) == RTL_EXIT) q += RTL_EXIT_WORDS;
    return ty(q) == RTL_END ? kind : 0u;
  }
  void exit_to(int parent) {
    // Consecutive EXITs collapse into one (restoring straight to the outermost parent) unless
    // a skip link targets the position between them.
    if (last_exit_end == w.size() && last_skip_target != w.size()) {
      w[w.size() - RTL_EXIT_WORDS + 2] = (uint32_t)parent;
      return;
    }
    size_t p = push(RTL_EXIT, RTL_EXIT_WORDS);
    w[p + 2] = (uint32_t)parent;
    last_exit_end = w.size();
  }
  void emit(const Node& n, int frame, std::vector<uint32_t>& chain, int in_volume) {
    if (status != RT_OK) return;
    switch (n.tag) {
      case RT_OBJ_LIST: {
        // Runs of >= 2 sibling quads become one QUADS batch (same visiting order; no skip
        // link can land inside a run because siblings of a list are never BVH boundaries).
        size_t i = 0;
        while (i < n.kids.size()) {
          size_t j = i;
          while (j < n.kids.size() && n.kids[j]->tag == RT_OBJ_QUAD) ++j;
#ifdef RT_NO_QUADS
          j = i;
#endif
          if (j - i >= 2) {
            size_t p = push(RTL_QUADS | (uint32_t)((j - i) << 8), 4);
            const size_t first_box = pbox.size();
            for (size_t k = i; k < j; ++k) quad(*n.kids[k], false);
            w[p + 1] = (uint32_t)w.size();
            PrimBox b = pbox[first_box].second;  // the batch: union of its quads' bounds
            for (size_t k = first_box + 1; k < pbox.size(); ++k) {
              const PrimBox& q = pbox[k].second;
              for (int c = 0; c < 3; ++c)
                b.lo[c] = std::min(b.lo[c], q.lo[c]), b.hi[c] = std::max(b.hi[c], q.hi[c]);
              b.valid = b.valid && q.valid;
              b.ref_complete = b.ref_complete && q.ref_complete;
            }
            pbox.push_back({p, b});
            i = j;
          } else {
            emit(*n.kids[i], frame, chain, in_volume);
            ++i;
          }
        }
        break;
      }
      case RT_OBJ_BVH: {
        has_bvh = true;
        size_t p = push(RTL_BVH, RTL_BVH_WORDS);
        for (int k = 0; k < 6; ++k) putd(w, p, k, n.bbox[k]);
        ++bvh_depth;
        emit(*n.kids[0], frame, chain, in_volume);
        if (same_tree(*n.kids[0], *n.kids[1]) && !has_volume_node(*n.kids[1])) {
          size_t d = push(RTL_DUP, RTL_DUP_WORDS);
          emit(*n.kids[1], frame, chain, in_volume);
          set_skip(d);
        } else {
          emit(*n.kids[1], frame, chain, in_volume);
        }
        --bvh_depth;
        set_skip(p);
        break;
      }
      case RT_OBJ_QUAD: quad(n, false); break;
      case RT_OBJ_SPHERE: sphere(n, false); break;
      case RT_OBJ_TRANSLATE:
      case RT_OBJ_ROTATE_Y: {
        bool tr = n.tag == RT_OBJ_TRANSLATE;
        size_t p = push(tr ? RTL_TRANSLATE : RTL_ROTATE_Y, RTL_XFORM_WORDS);
        chain.push_back((uint32_t)p);
        if (chain.size() > max_chain) max_chain = (uint32_t)chain.size();
        w[p + 2] = (uint32_t)chain.size();
        if (chain.size() <= RTL_MAX_CHAIN) {
          for (size_t k = 0; k < chain.size(); ++k) w[p + 4 + k] = chain[k];
        } else {  // a long chain: table appended after relocation (flatten)
          w[p] |= RTL_XFORM_LONG;
          w[p + 4] = (uint32_t)long_chains.size();
          long_chains.push_back(chain);
        }
        if (tr) {
          putd(w, p, 2, n.f[0]), putd(w, p, 3, n.f[1]), putd(w, p, 4, n.f[2]);
        } else {
          putd(w, p, 2, n.f[0]), putd(w, p, 3, n.f[1]);
        }
        emit(*n.kids[0], (int)p, chain, in_volume);
        chain.pop_back();
        exit_to(frame);
        w[p + 1] = (uint32_t)w.size();
        break;
      }
      case RT_OBJ_VOLUME: {
        if (in_volume > RTL_VOLUME_NEST) {
          fail(RT_ERR_UNSUPPORTED, "ConstantMedium boundaries nested deeper than " +
                                       std::to_string(RTL_VOLUME_NEST));
          return;
        }
        if (in_volume > 0 && bvh_depth > 0) {
          fail(RT_ERR_UNSUPPORTED, "ConstantMedium inside a BVH inside a ConstantMedium boundary");
          return;
        }
        if (in_volume > 0) nested_volumes = true;
        if (!check_mat(n.mat)) return;
        has_volume = true;
        if (bvh_depth > 0) volume_in_bvh = true;
        size_t p = push(RTL_VOLUME, RTL_VOLUME_WORDS);
        w[p + 2] = (uint32_t)n.mat;
        putd(w, p, 0, n.f[0]);
        emit(*n.kids[0], frame, chain, in_volume + 1);
        push(RTL_END, RTL_END_WORDS);
        set_skip(p);
        w[p] |= fusable_boundary(p + RTL_VOLUME_WORDS);
        if (!(w[p] & RTL_VOLF_SPHERE)) all_sphere_volumes = false;
        break;
      }
    }
  }
};

bool tex_needs_uv(const std::vector<uint32_t>& texs, uint32_t id, int depth) {
  if (depth > 64) return false;
  const uint32_t* t = &texs[(size_t)id * RTL_TEX_WORDS];
  if (t[0] == RT_TEX_IMAGE) return t[1] > 0 && t[2] > 0;
  if (t[0] == RT_TEX_CHECKER) return tex_needs_uv(texs, t[1], depth + 1) || tex_needs_uv(texs, t[2], depth + 1);
  return false;
}

}  // namespace

// Words of the record starting with header word h.
uint32_t record_words(uint32_t h) {
  switch (h & 0xffu) {
    case RTL_QUAD: return RTL_QUAD_WORDS;
    case RTL_SPHERE: return RTL_SPHERE_WORDS;
    case RTL_BVH: return RTL_BVH_WORDS;
    case RTL_TRANSLATE:
    case RTL_ROTATE_Y: return RTL_XFORM_WORDS;
    case RTL_EXIT: return RTL_EXIT_WORDS;
    case RTL_VOLUME: return RTL_VOLUME_WORDS;
    case RTL_DUP: return RTL_DUP_WORDS;
    default: return 4;  // END, QUADS header
  }
}

namespace {

// Move every BVH record to the front of the node array (the BVH region [0, bvh_words), staged
// in LDS by rt_trace) and make every link explicit (rt_layout.h): BVH records get their first
// child in word 2, every other record its pre-order successor in word 3. The visiting order,
// and with it every result, is unchanged: only the addresses move.
void relocate(std::vector<uint32_t>& w, uint32_t* root, uint32_t* bvh_words,
              std::vector<uint32_t>* map_out) {
  std::vector<size_t> pos;
  for (size_t p = 0; p < w.size(); p += record_words(w[p])) pos.push_back(p);
  std::vector<uint32_t> map(w.size() + 1, 0xffffffffu);
  uint32_t nb = 0;
  for (size_t p : pos)
    if ((w[p] & 0xffu) == RTL_BVH) map[p] = nb, nb += RTL_BVH_WORDS;
  uint32_t nm = nb;
  for (size_t p : pos)
    if ((w[p] & 0xffu) != RTL_BVH) map[p] = nm, nm += record_words(w[p]);
  map[w.size()] = nm;
  auto m = [&](uint32_t old) { return old == 0xffffffffu ? old : map[old]; };
  std::vector<uint32_t> out(w.size(), 0u);
  for (size_t p : pos) {
    const uint32_t h = w[p], sz = record_words(h), q = map[p];
    std::memcpy(&out[q], &w[p], sz * 4);
    const uint32_t type = h & 0xffu;
    if (type != RTL_QUAD && type != RTL_SPHERE && type != RTL_EXIT && type != RTL_END)
      out[q + 1] = m(w[p + 1]);  // skip
    if (type == RTL_BVH) {
      out[q + 2] = m((uint32_t)(p + sz));  // first child
    } else if (type != RTL_END) {
      out[q + 3] = m((uint32_t)(p + sz));  // pre-order successor
    }
    if ((type == RTL_TRANSLATE || type == RTL_ROTATE_Y) && !(h & RTL_XFORM_LONG))
      for (uint32_t k = 0; k < w[p + 2]; ++k) out[q + 4 + k] = m(w[p + 4 + k]);  // chain
    if (type == RTL_EXIT) out[q + 2] = m(w[p + 2]);  // parent frame
  }
  w.swap(out);
  *root = m(*root);
  *bvh_words = nb;
  map_out->swap(map);
}

// BVH records where the top-level walk hands a subtree to the per-lane walker (the world
// sequence and every ConstantMedium boundary sequence, as traverse<UNI> visits them)
std::vector<uint32_t> bvh_roots(const std::vector<uint32_t>& w, uint32_t root) {
  std::vector<uint32_t> roots, todo{root};
  size_t guard = 0;
  while (!todo.empty()) {
    uint32_t x = todo.back();
    todo.pop_back();
    while (x < w.size() && ++guard < (1u << 26)) {
      const uint32_t ty = w[x] & 0xffu;
      if (ty == RTL_END) break;
      if (ty == RTL_BVH) {
        roots.push_back(x);
        x = w[x + 1];
      } else if (ty == RTL_VOLUME) {
        todo.push_back(w[x + 3]);  // the boundary sequence
        x = w[x + 1];
      } else if (ty == RTL_QUADS || ty == RTL_DUP || ty == RTL_OTHER) {
        x = w[x + 1];
      } else {
        x = w[x + 3];  // QUAD, SPHERE: next; TRANSLATE / ROTATE_Y: child; EXIT: next
      }
    }
  }
  return roots;
}

}  // namespace

int flatten(const rt_scene_blob* blob, FlatScene* out, std::string* err) {
  if (!blob || !blob->slots || blob->n_slots < RT_BLOB_HEADER_SLOTS) {
    *err = "null or short blob";
    return RT_ERR_BAD_BLOB;
  }
  const uint64_t* s = blob->slots;
  if (s[0] != RT_BLOB_MAGIC || s[1] != RT_BLOB_VERSION || s[2] != blob->n_slots) {
    *err = "bad blob magic/version/size";
    return RT_ERR_BAD_BLOB;
  }
  uint64_t n = blob->n_slots;
  uint64_t n_tex = s[3], tex_off = s[4], n_mat = s[5], mat_off = s[6], n_perl = s[7],
           perl_off = s[8], world_off = s[9];
  int64_t lights_off = (int64_t)s[10];
  uint64_t n_texel = s[11];
  if (n_tex > (1u << 20) || n_mat > (1u << 20) || n_perl > 4096 ||
      tex_off + n_tex * RT_TEX_SLOTS > n || mat_off + n_mat * RT_MAT_SLOTS > n ||
      perl_off + n_perl * RT_PERLIN_SLOTS > n || world_off >= n ||
      (lights_off >= 0 && (uint64_t)lights_off >= n) || n_texel != blob->n_texels ||
      (n_texel > 0 && !blob->texels)) {
    *err = "blob header out of range";
    return RT_ERR_BAD_BLOB;
  }
  FlatScene& F = *out;
  F = FlatScene();
  auto setd = [](uint32_t* o, int k, double d) { std::memcpy(o + 4 + 2 * k, &d, 8); };
  auto rd_f = [&](uint64_t i) {
    double d;
    std::memcpy(&d, &s[i], 8);
    return d;
  };
  // textures
  F.texs.assign(n_tex * RTL_TEX_WORDS, 0u);
  for (uint64_t t = 0; t < n_tex; ++t) {
    uint64_t b = tex_off + t * RT_TEX_SLOTS;
    uint32_t* o = &F.texs[t * RTL_TEX_WORDS];
    int64_t kind = (int64_t)s[b];
    o[0] = (uint32_t)kind;
    switch (kind) {
      case RT_TEX_SOLID:
        setd(o, 0, rd_f(b + 1)), setd(o, 1, rd_f(b + 2)), setd(o, 2, rd_f(b + 3));
        break;
      case RT_TEX_CHECKER: {
        int64_t e = (int64_t)s[b + 2], d = (int64_t)s[b + 3];
        if (e < 0 || d < 0 || (uint64_t)e >= n_tex || (uint64_t)d >= n_tex) {
          *err = "checker texture index out of range";
          return RT_ERR_BAD_BLOB;
        }
        setd(o, 0, rd_f(b + 1)), o[1] = (uint32_t)e, o[2] = (uint32_t)d;
        break;
      }
      case RT_TEX_IMAGE: {
        int64_t w = (int64_t)s[b + 1], h = (int64_t)s[b + 2], off = (int64_t)s[b + 3];
        if (w < 0 || h < 0 || off < 0 || (w > 0 && h > 0 && (uint64_t)(off + w * h * 3) > n_texel)) {
          *err = "image texture out of range";
          return RT_ERR_BAD_BLOB;
        }
        o[1] = (uint32_t)w, o[2] = (uint32_t)h, o[3] = (uint32_t)off;
        break;
      }
      case RT_TEX_NOISE: {
        int64_t pi = (int64_t)s[b + 2];
        if (pi < 0 || (uint64_t)pi >= n_perl) {
          *err = "noise texture perlin index out of range";
          return RT_ERR_BAD_BLOB;
        }
        setd(o, 0, rd_f(b + 1)), o[1] = (uint32_t)pi;
        break;
      }
      default:
        *err = "unknown texture kind";
        return RT_ERR_BAD_BLOB;
    }
  }
  // checker cycles (the reference's Arc graph cannot form one; reject defensively)
  for (uint64_t t = 0; t < n_tex; ++t) {
    uint64_t id = t;
    int steps = 0;
    while (F.texs[id * RTL_TEX_WORDS] == RT_TEX_CHECKER && steps < 65) {
      id = F.texs[id * RTL_TEX_WORDS + 1];
      ++steps;
    }
    if (steps > 64) {
      *err = "checker texture nesting deeper than 64";
      return RT_ERR_UNSUPPORTED;
    }
  }
  // materials
  F.mats.assign(n_mat * RTL_MAT_WORDS, 0u);
  bool pdf_mats = false, textured = false, isotropic = false;
  for (uint64_t m = 0; m < n_mat; ++m) {
    uint64_t b = mat_off + m * RT_MAT_SLOTS;
    uint32_t* o = &F.mats[m * RTL_MAT_WORDS];
    int64_t kind = (int64_t)s[b];
    switch (kind) {
      case RT_MAT_LAMBERTIAN:
      case RT_MAT_DIFFUSE_LIGHT:
      case RT_MAT_ISOTROPIC: {
        int64_t t = (int64_t)s[b + 1];
        if (t < 0 || (uint64_t)t >= n_tex) {
          *err = "material texture index out of range";
          return RT_ERR_BAD_BLOB;
        }
        o[1] = (uint32_t)t;
        o[0] = (uint32_t)kind | (tex_needs_uv(F.texs, (uint32_t)t, 0) ? RTL_MATF_NEEDS_UV : 0u);
        if (kind != RT_MAT_DIFFUSE_LIGHT) pdf_mats = true;
        if (kind == RT_MAT_ISOTROPIC) isotropic = true;
        if (F.texs[(size_t)t * RTL_TEX_WORDS] != RT_TEX_SOLID) textured = true;
        break;
      }
      case RT_MAT_METAL:  // albedo3 fuzz
        o[0] = (uint32_t)kind;
        setd(o, 0, rd_f(b + 1)), setd(o, 1, rd_f(b + 2)), setd(o, 2, rd_f(b + 3));
        setd(o, 3, rd_f(b + 4));
        break;
      case RT_MAT_DIELECTRIC:  // ir tint3
        o[0] = (uint32_t)kind;
        setd(o, 3, rd_f(b + 1));
        setd(o, 0, rd_f(b + 2)), setd(o, 1, rd_f(b + 3)), setd(o, 2, rd_f(b + 4));
        {
          const double ir = rd_f(b + 1), inv = 1.0 / ir;
          const double rf = (1.0 - inv) / (1.0 + inv), rb = (1.0 - ir) / (1.0 + ir);
          setd(o, 4, inv), setd(o, 5, rf * rf), setd(o, 6, rb * rb);
        }
        break;
      default:
        *err = "unknown material kind";
        return RT_ERR_BAD_BLOB;
    }
  }
  // perlin tables
  F.perlin.assign(n_perl * RTL_PERLIN_BYTES, 0);
  for (uint64_t p = 0; p < n_perl; ++p) {
    uint64_t b = perl_off + p * RT_PERLIN_SLOTS;
    float* rv = (float*)&F.perlin[p * RTL_PERLIN_BYTES];
    for (int k = 0; k < 256; ++k) {
      rv[4 * k] = (float)rd_f(b + 3 * k);
      rv[4 * k + 1] = (float)rd_f(b + 3 * k + 1);
      rv[4 * k + 2] = (float)rd_f(b + 3 * k + 2);
      rv[4 * k + 3] = 0.0f;
    }
    uint8_t* perm = &F.perlin[p * RTL_PERLIN_BYTES + 4096];
    for (int k = 0; k < 768; ++k) {
      int64_t v = (int64_t)s[b + 768 + k];
      if (v < 0 || v > 255) {
        *err = "perlin permutation entry out of range";
        return RT_ERR_BAD_BLOB;
      }
      perm[k] = (uint8_t)v;
    }
  }
  // world
  Reader r{s, n, world_off};
  auto world = read_node(r, 0);
  if (r.err || !world) {
    *err = "world: " + r.msg;
    return RT_ERR_BAD_BLOB;
  }
  if (world->tag != RT_OBJ_LIST) {
    *err = "world must be a HittableList";
    return RT_ERR_BAD_BLOB;
  }
  Emitter em(F.nodes, (int64_t)n_mat);
  std::vector<uint32_t> chain;
  em.emit(*world, -1, chain, 0);
  em.push(RTL_END, RTL_END_WORDS);
  if (em.status != RT_OK) {
    *err = em.err;
    return em.status;
  }
  uint32_t root = 0, bvh_words = 0;
  std::vector<uint32_t> map;
  relocate(F.nodes, &root, &bvh_words, &map);
  const uint32_t rec_words = (uint32_t)F.nodes.size();
  // long transform chains (rt_layout.h RTL_XFORM_LONG): relocated tables after the records
  for (size_t p = 0; p < rec_words; p += record_words(F.nodes[p])) {
    const uint32_t h = F.nodes[p], ty = h & 0xffu;
    if ((ty == RTL_TRANSLATE || ty == RTL_ROTATE_Y) && (h & RTL_XFORM_LONG)) {
      const std::vector<uint32_t>& c = em.long_chains[F.nodes[p + 4]];
      F.nodes[p + 4] = (uint32_t)F.nodes.size();
      for (uint32_t x : c) F.nodes.push_back(map[x]);
    }
  }
  while (F.nodes.size() % 4) F.nodes.push_back(0u);
  uint32_t cbvh_word0 = 0, cbvh_words = 0, cbvh_stack = 0;
  {  // ordered BVHs of the product kernels (rt_obvh.cpp), appended after the records
    std::vector<PrimBox> boxes(rec_words);
    for (auto& pb : em.pbox)
      if (pb.first < map.size() && map[pb.first] < rec_words) boxes[map[pb.first]] = pb.second;
    build_ordered_bvhs(F.nodes, rec_words, boxes, bvh_roots(F.nodes, root), &cbvh_word0,
                       &cbvh_words, &cbvh_stack);
  }
  if (F.nodes.size() >= 0x7fffffffu) {
    *err = "scene too large";
    return RT_ERR_UNSUPPORTED;
  }
  // lights (HittablePDF over the lights object, pdf.rs:80-100)
  uint32_t n_lights = 0, is_list = 0, lights_nested = 0;
  if (lights_off >= 0) {
    Reader lr{s, n, (uint64_t)lights_off};
    auto lights = lr.err ? nullptr : read_node(lr, 0);
    if (lr.err || !lights) {
      *err = "lights: " + lr.msg;
      return RT_ERR_BAD_BLOB;
    }
    Emitter le(F.lights, (int64_t)n_mat);
    // Light entries: the top-level objects first, then the children of every nested list
    // (object.rs:57, 66: Object::List dispatches pdf_value / random to HittableList) as one
    // consecutive block per list, breadth first.
    std::vector<const Node*> ent;
    std::vector<int> level;
    std::vector<uint32_t> first;
    if (lights->tag == RT_OBJ_LIST) {
      is_list = 1;
      for (auto& k : lights->kids) ent.push_back(k.get()), level.push_back(1);
    } else {
      ent.push_back(lights.get()), level.push_back(1);
    }
    n_lights = (uint32_t)ent.size();
    first.assign(ent.size(), 0u);
    for (size_t e = 0; e < ent.size(); ++e) {
      if (ent[e]->tag != RT_OBJ_LIST || (e == 0 && !is_list && ent[e] == lights.get())) continue;
      if (ent[e]->kids.empty()) {
        *err = "empty HittableList inside the light list: the reference panics (hittable.rs:120)";
        return RT_ERR_EMPTY_LIGHTS;
      }
      if (level[e] > RTL_LIGHT_NEST) {
        *err = "light lists nested deeper than " + std::to_string(RTL_LIGHT_NEST);
        return RT_ERR_UNSUPPORTED;
      }
      first[e] = (uint32_t)ent.size();
      for (auto& k : ent[e]->kids) {
        ent.push_back(k.get()), level.push_back(level[e] + 1), first.push_back(0u);
      }
    }
    for (size_t e = 0; e < ent.size(); ++e) {
      const Node& nd = *ent[e];
      F.light_offs.push_back((uint32_t)F.lights.size());
      if (nd.tag == RT_OBJ_QUAD) {
        le.quad(nd, true);
      } else if (nd.tag == RT_OBJ_SPHERE) {
        le.sphere(nd, true);
      } else if (nd.tag == RT_OBJ_LIST && e < F.light_offs.size() && first[e] != 0u) {
        const size_t p = le.push(RTL_LLIST | (uint32_t)(nd.kids.size() << 8), RTL_LLIST_WORDS);
        F.lights[p + 1] = first[e];
        putd(F.lights, p, 0, 1. / (double)nd.kids.size());  // hittable.rs:116
        lights_nested = 1;
      } else {
        le.push(RTL_OTHER, 4);
      }
    }
    if (le.status != RT_OK) {
      *err = le.err;
      return le.status;
    }
    if (is_list && n_lights == 0) {
      // An empty HittableList light object panics in the reference exactly like render_par.
      is_list = 0;
    }
  }
  if (blob->n_texels) F.texels.assign(blob->texels, blob->texels + blob->n_texels);
  rtl_scene_header& h = F.hdr;
  h.root = root;
  h.bvh_words = bvh_words;
  h.n_node_words = (uint32_t)F.nodes.size();
  h.n_rec_words = rec_words;
  h.cbvh_word0 = cbvh_word0;
  h.cbvh_words = cbvh_words;
  h.cbvh_stack = cbvh_stack;
  h.n_mats = (uint32_t)n_mat;
  h.n_texs = (uint32_t)n_tex;
  h.n_perlins = (uint32_t)n_perl;
  h.n_lights = n_lights;
  h.lights_is_list = is_list;
  h.lights_nested = lights_nested;
  h.nested_volumes = em.nested_volumes;
  h.has_bvh = em.has_bvh;
  h.has_volume = em.has_volume;
  h.volume_in_bvh = em.volume_in_bvh;
  h.volumes_one_walk_spheres = em.has_volume && em.all_sphere_volumes;
  h.max_chain = em.max_chain;
  h.n_texel_bytes = (uint32_t)n_texel;
  h.pdf_materials = pdf_mats;
  h.has_textures = textured;
  h.has_isotropic = isotropic;
  return RT_OK;
}

}  // namespace rtf
