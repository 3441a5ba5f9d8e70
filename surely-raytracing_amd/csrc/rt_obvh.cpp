// rt_obvh.cpp — ordered BVHs for the product kernels (rt_layout.h "OBVH").
//
// BvhNode::hit (hittable.rs:216-236) returns the closest hit of its subtree. Which primitive
// wins depends on the visiting order only when candidates tie: for a quad (inclusive interval,
// object.rs:462) a later equal t replaces the record, for a sphere (strict, object.rs:161-166)
// it does not, and an AABB whose entry equals the current closest t is culled (object.rs:362-
// 364). Away from ties, every order finds the same record: the smallest candidate t.
//
// The reference's tree (random split axis, hittable.rs:150) is poor for traversal, and its
// fixed left-then-right order visits far subtrees before near ones. For a BVH subtree whose
// leaves are quads, quad batches and spheres (no instances, no ConstantMedium: no random draws
// during the walk), this file builds a second tree over the SAME leaf records: a BVH2 by the
// surface-area heuristic over conservative leaf bounds, written once per ray-direction octant
// as a threaded pre-order stream in which every node's near child (along its split axis for
// that octant) comes first. The kernel walks the octant's stream with closest-t culling and
// flags any lane whose result could depend on order (a candidate within 2^-30 relative of the
// running closest t, or of t_min); flagged lanes re-walk the reference subtree in the
// reference order (rt_kernel.h bvh_subtree), so images stay bit-identical to the reference
// order's (tests/test_gpu_parity.py compares against the op-counting build, which always walks
// the reference tree).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "rt_flatten.hpp"

namespace rtf {

namespace {

constexpr int kSahDepth = 40;  // SAH splits above this depth, median splits below (<= 40 + 20)

struct Leaf {
  uint32_t rec;
  PrimBox b;
  double c[3];
};

struct BNode {
  double lo[3], hi[3];
  int left = -1, right = -1;  // children (BNode indices); leaf: left = -1, leaf index in `right`
  int axis = 0;
};

double area(const double* lo, const double* hi) {
  const double x = hi[0] - lo[0], y = hi[1] - lo[1], z = hi[2] - lo[2];
  return 2.0 * (x * y + y * z + z * x);
}

struct Builder {
  std::vector<Leaf>& L;
  std::vector<BNode> nodes;
  explicit Builder(std::vector<Leaf>& l) : L(l) {}

  int build(int b, int e, int depth) {  // leaves [b, e)
    BNode n;
    for (int k = 0; k < 3; ++k) n.lo[k] = HUGE_VAL, n.hi[k] = -HUGE_VAL;
    for (int i = b; i < e; ++i)
      for (int k = 0; k < 3; ++k)
        n.lo[k] = std::min(n.lo[k], L[i].b.lo[k]), n.hi[k] = std::max(n.hi[k], L[i].b.hi[k]);
    const int id = (int)nodes.size();
    nodes.push_back(n);
    if (e - b == 1) {
      nodes[id].right = b;
      return id;
    }
    // SAH over every split position of the centroid order along each axis; past kSahDepth a
    // median split on the widest centroid axis bounds the depth
    double best = HUGE_VAL;
    int best_axis = 0, best_split = (b + e) / 2;
    std::vector<double> right_area(e - b + 1);
    if (depth >= kSahDepth) {
      double wmax = -1.0;
      for (int axis = 0; axis < 3; ++axis) {
        double lo = HUGE_VAL, hi = -HUGE_VAL;
        for (int i = b; i < e; ++i) lo = std::min(lo, L[i].c[axis]), hi = std::max(hi, L[i].c[axis]);
        if (hi - lo > wmax) wmax = hi - lo, best_axis = axis;
      }
    }
    for (int axis = 0; axis < 3 && depth < kSahDepth; ++axis) {
      std::stable_sort(L.begin() + b, L.begin() + e,
                       [axis](const Leaf& x, const Leaf& y) { return x.c[axis] < y.c[axis]; });
      double lo[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL}, hi[3] = {-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
      for (int i = e - 1; i > b; --i) {
        for (int k = 0; k < 3; ++k)
          lo[k] = std::min(lo[k], L[i].b.lo[k]), hi[k] = std::max(hi[k], L[i].b.hi[k]);
        right_area[i - b] = area(lo, hi) * (e - i);
      }
      for (int k = 0; k < 3; ++k) lo[k] = HUGE_VAL, hi[k] = -HUGE_VAL;
      for (int i = b; i < e - 1; ++i) {
        for (int k = 0; k < 3; ++k)
          lo[k] = std::min(lo[k], L[i].b.lo[k]), hi[k] = std::max(hi[k], L[i].b.hi[k]);
        const double cost = area(lo, hi) * (i + 1 - b) + right_area[i + 1 - b];
        if (cost < best) best = cost, best_axis = axis, best_split = i + 1;
      }
    }
    std::stable_sort(L.begin() + b, L.begin() + e, [best_axis](const Leaf& x, const Leaf& y) {
      return x.c[best_axis] < y.c[best_axis];
    });
    const int l = build(b, best_split, depth + 1);
    const int r = build(best_split, e, depth + 1);
    nodes[id].left = l;
    nodes[id].right = r;
    nodes[id].axis = best_axis;
    return id;
  }
};

float f32_down(double x) {
  float f = (float)x;
  if ((double)f > x) f = std::nextafter(f, -HUGE_VALF);
  return f;
}
float f32_up(double x) {
  float f = (float)x;
  if ((double)f < x) f = std::nextafter(f, HUGE_VALF);
  return f;
}

// end of the record / subtree starting at x in the relocated array (the walker's continuation)
bool subtree_end(const std::vector<uint32_t>& w, uint32_t x, uint32_t* end) {
  switch (w[x] & 0xffu) {
    case RTL_BVH:
    case RTL_DUP:
    case RTL_QUADS: *end = w[x + 1]; return true;
    case RTL_QUAD:
    case RTL_SPHERE: *end = w[x + 3]; return true;
    default: return false;
  }
}

// leaves of the reference subtree at x (BvhNode children, span-1 duplicates dropped)
bool collect(const std::vector<uint32_t>& w, uint32_t x, const std::vector<PrimBox>& boxes,
             std::vector<Leaf>& out, int depth) {
  if (depth > 256 || x >= w.size()) return false;
  const uint32_t ty = w[x] & 0xffu;
  if (ty == RTL_BVH) {
    const uint32_t c1 = w[x + 2];
    uint32_t c2;
    if (!collect(w, c1, boxes, out, depth + 1) || !subtree_end(w, c1, &c2) || c2 >= w.size())
      return false;
    if ((w[c2] & 0xffu) == RTL_DUP) return true;  // the same leaf again (hittable.rs:161-162)
    return collect(w, c2, boxes, out, depth + 1);
  }
  if (ty != RTL_QUADS && ty != RTL_QUAD && ty != RTL_SPHERE) return false;
  const PrimBox& b = boxes[x];
  if (!b.valid || !b.ref_complete) return false;
  Leaf lf;
  lf.rec = x;
  lf.b = b;
  for (int k = 0; k < 3; ++k) lf.c[k] = 0.5 * (b.lo[k] + b.hi[k]);
  out.push_back(lf);
  return true;
}

}  // namespace

void build_ordered_bvhs(std::vector<uint32_t>& w, uint32_t rec_words,
                        const std::vector<PrimBox>& boxes, const std::vector<uint32_t>& roots) {
  for (uint32_t root : roots) {
    std::vector<Leaf> leaves;
    if (!collect(w, root, boxes, leaves, 0) || leaves.empty() || leaves.size() > (1u << 20))
      continue;
    if (std::getenv("RT_OBVH_DEBUG")) {  // diagnostics: leaf count, distinct records
      std::vector<uint32_t> r;
      for (auto& l : leaves) r.push_back(l.rec);
      std::sort(r.begin(), r.end());
      std::fprintf(stderr, "obvh root %u: %zu leaves, %zu distinct\n", root, leaves.size(),
                   (size_t)(std::unique(r.begin(), r.end()) - r.begin()));
    }
    Builder B(leaves);
    B.build(0, (int)leaves.size(), 0);
    // one stream of 8-word entries per ray-direction octant, in pre-order with the near child
    // first; an internal entry carries its box as f32 (near, far) bound pairs for that octant
    const uint32_t n_entries = (uint32_t)B.nodes.size();
    while (w.size() % 4) w.push_back(0u);
    const uint32_t hdr = (uint32_t)w.size();
    const uint32_t streams_off = 4;
    w.resize(hdr + streams_off + (size_t)8 * n_entries * 8, 0u);
    w[hdr] = n_entries;
    w[hdr + 3] = streams_off;
    for (uint32_t oct = 0; oct < 8; ++oct) {
      uint32_t* S = &w[hdr + streams_off + (size_t)oct * n_entries * 8];
      uint32_t pos = 0;
      // pre-order with the near child first (recursion depth = tree depth <= kSahDepth + 20)
      struct Emit {
        const std::vector<BNode>& N;
        const std::vector<Leaf>& L;
        uint32_t* S;
        uint32_t oct;
        uint32_t& pos;
        void run(int i) {
          const BNode& n = N[i];
          uint32_t* E = S + (size_t)8 * pos++;
          if (n.left < 0) {
            E[0] = 0x80000000u;
            E[1] = L[n.right].rec;
          } else {
            const bool neg = (oct >> n.axis) & 1u;
            run(neg ? n.right : n.left);
            run(neg ? n.left : n.right);
            E[0] = pos;  // skip: the entry after the subtree
          }
          for (int a = 0; a < 3; ++a) {  // the node's (or leaf's) own box
            // conservative f32 bounds: the padded f64 box grown by 2^-18 (1 + |coord|) and
            // rounded outwards (rt_kernel.h obvh_walk's error budget)
            const double m = 0x1p-18 * (1.0 + std::max(std::fabs(n.lo[a]), std::fabs(n.hi[a])));
            const float lo = f32_down(n.lo[a] - m), hi = f32_up(n.hi[a] + m);
            const bool na = (oct >> a) & 1u;  // d_a < 0: the near bound is hi
            std::memcpy(&E[2 + 2 * a], na ? &hi : &lo, 4);
            std::memcpy(&E[3 + 2 * a], na ? &lo : &hi, 4);
          }
        }
      } em{B.nodes, leaves, S, oct, pos};
      em.run(0);
    }
    w[root + 3] = hdr;  // the reference BVH record points at its ordered tree
  }
  (void)rec_words;
}

}  // namespace rtf
