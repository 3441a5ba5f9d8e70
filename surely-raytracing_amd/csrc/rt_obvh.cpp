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
#include <array>
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

// A QUADS batch that is make_box's six sides (object.rs:509-560) in its order: z = max, x = max,
// z = min, x = min, y = max, y = min, every side axis-aligned in the batch's frame (rt_layout.h
// RTL_QUAD_AXIS: 3, 1, 3, 1, 2, 2) with the max side's plane above the min side's. Such a leaf is
// tagged RTL_LEAF_BOX in the ordered BVHs: obvh_leaf tests the three sides the ray faces in full
// and the other three only when their planes come within the tie window (rt_kernel.h).
bool make_box_batch(const std::vector<uint32_t>& w, uint32_t x) {
  if ((w[x] & 0xffu) != RTL_QUADS || (w[x] >> 8) != 6u) return false;
  static const uint32_t axis[6] = {3u, 1u, 3u, 1u, 2u, 2u};
  double qk[6];
  for (int f = 0; f < 6; ++f) {
    const size_t q = (size_t)x + 4 + (size_t)f * RTL_QUAD_WORDS;
    if (q + RTL_QUAD_WORDS > w.size() || (w[q] & 0xffu) != RTL_QUAD || RTL_QUAD_AXIS(w[q]) != axis[f])
      return false;
    const uint64_t bits = (uint64_t)w[q + 4] | (uint64_t)w[q + 5] << 32;  // d0 = q_k
    std::memcpy(&qk[f], &bits, 8);
  }
  return qk[0] > qk[2] && qk[1] > qk[3] && qk[4] > qk[5];
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
  lf.rec = x | (make_box_batch(w, x) ? RTL_LEAF_BOX : 0u);
  lf.b = b;
  for (int k = 0; k < 3; ++k) lf.c[k] = 0.5 * (b.lo[k] + b.hi[k]);
  out.push_back(lf);
  return true;
}

}  // namespace

// Outward-rounded f32 bounds of a node's box (the padded f64 box grown by 2^-18 (1 + |coord|)):
// rt_kernel.h obvh_walk / cbvh_walk's error budget.
void f32_box(const BNode& n, float lo[3], float hi[3]) {
  for (int a = 0; a < 3; ++a) {
    const double m = 0x1p-18 * (1.0 + std::max(std::fabs(n.lo[a]), std::fabs(n.hi[a])));
    lo[a] = f32_down(n.lo[a] - m);
    hi[a] = f32_up(n.hi[a] + m);
  }
}

// The compact copy of one tree (rt_layout.h CBVH) as words; false when it does not fit the
// format (16-bit references, internal-node depth <= RTL_CBVH_STACK).
bool compact_tree(const std::vector<BNode>& nodes, const std::vector<Leaf>& leaves,
                  std::vector<uint32_t>* out, uint32_t* root_ref, int* depth) {
  const size_t n_leaf = leaves.size();
  if (n_leaf == 0 || n_leaf > 0x7fffu) return false;
  if (n_leaf == 1) {  // a single leaf: the root reference is the leaf
    out->assign(4, 0u);
    (*out)[0] = leaves[0].rec;
    *root_ref = 0x8000u;
    *depth = 1;
    return true;
  }
  // internal nodes in pre-order (index 0 = the root), leaves in first-visit order
  std::vector<int> order, leaf_of(nodes.size(), -1), int_of(nodes.size(), -1);
  std::vector<uint32_t> leaf_recs;
  int max_depth = 0;
  struct Walk {
    const std::vector<BNode>& N;
    const std::vector<Leaf>& L;
    std::vector<int>& order;
    std::vector<int>& leaf_of;
    std::vector<int>& int_of;
    std::vector<uint32_t>& recs;
    int& max_depth;
    void run(int i, int depth) {
      if (N[i].left < 0) {
        leaf_of[i] = (int)recs.size();
        recs.push_back(L[N[i].right].rec);
        return;
      }
      max_depth = std::max(max_depth, depth);
      int_of[i] = (int)order.size();
      order.push_back(i);
      run(N[i].left, depth + 1);
      run(N[i].right, depth + 1);
    }
  } wk{nodes, leaves, order, leaf_of, int_of, leaf_recs, max_depth};
  wk.run(0, 1);
  const size_t n_int = order.size();
  if (n_int > 0x7fffu || max_depth > RTL_CBVH_STACK || leaf_recs.size() != n_leaf) return false;
  *depth = max_depth;
  auto ref = [&](int c) -> uint32_t {
    return nodes[c].left < 0 ? 0x8000u | (uint32_t)leaf_of[c] : (uint32_t)int_of[c];
  };
  const size_t words = (n_int * 12 + n_int + n_leaf + 3) & ~(size_t)3;
  out->assign(words, 0u);
  uint32_t* B = out->data();
  for (size_t k = 0; k < n_int; ++k) {
    const BNode& n = nodes[order[k]];
    const int ch[2] = {n.left, n.right};
    for (int c = 0; c < 2; ++c) {
      float lo[3], hi[3];
      f32_box(nodes[ch[c]], lo, hi);
      // per axis a: [lo_a child 0, lo_a child 1, hi_a child 0, hi_a child 1] (rt_layout.h CBVH)
      for (int a = 0; a < 3; ++a) {
        std::memcpy(&B[k * 12 + 4 * a + c], &lo[a], 4);
        std::memcpy(&B[k * 12 + 4 * a + 2 + c], &hi[a], 4);
      }
    }
    B[n_int * 12 + k] = ref(n.left) | ref(n.right) << 16;
  }
  for (size_t k = 0; k < n_leaf; ++k) B[n_int * 13 + k] = leaf_recs[k];
  *root_ref = 0u;
  return true;
}

void build_ordered_bvhs(std::vector<uint32_t>& w, uint32_t rec_words,
                        const std::vector<PrimBox>& boxes, const std::vector<uint32_t>& roots,
                        uint32_t* cbvh_word0, uint32_t* cbvh_words, uint32_t* cbvh_stack) {
  std::vector<uint32_t> cbvh;  // the compact region, appended after every ordered stream
  *cbvh_word0 = *cbvh_words = *cbvh_stack = 0u;
  for (uint32_t root : roots) {
    std::vector<Leaf> leaves;
    if (!collect(w, root, boxes, leaves, 0) || leaves.empty() || leaves.size() > (1u << 20))
      continue;
    if (std::getenv("RT_OBVH_DEBUG")) {  // diagnostics: leaf count, distinct records
      std::vector<uint32_t> r;
      for (auto& l : leaves) r.push_back(l.rec & ~RTL_LEAF_BOX);
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
    const uint32_t streams_off = 8;
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
          float lo[3], hi[3];  // the node's (or leaf's) own box, conservative f32 bounds
          f32_box(n, lo, hi);
          for (int a = 0; a < 3; ++a) {
            const bool na = (oct >> a) & 1u;  // d_a < 0: the near bound is hi
            std::memcpy(&E[2 + 2 * a], na ? &hi[a] : &lo[a], 4);
            std::memcpy(&E[3 + 2 * a], na ? &lo[a] : &hi[a], 4);
          }
        }
      } em{B.nodes, leaves, S, oct, pos};
      em.run(0);
    }
    w[root + 3] = hdr;  // the reference BVH record points at its ordered tree
    std::vector<uint32_t> blk;
    uint32_t root_ref = 0u;
    w[hdr + 1] = 0xffffffffu;
    // the two-wide compact tree (a 4-wide form walked in about half the steps but tested more
    // boxes and sorted them: 3.3 % slower at C4, profiles/r03_ab_bvh4_vs_bvh2_c4.log; removed)
    int depth = 0;
    if (!std::getenv("RT_NO_CBVH") &&
        compact_tree(B.nodes, leaves, &blk, &root_ref, &depth)) {
      w[hdr + 1] = (uint32_t)(cbvh.size() * 4);  // byte offset in the region
      w[hdr + 2] = root_ref;
      cbvh.insert(cbvh.end(), blk.begin(), blk.end());
      // per-lane stack bytes: cbvh_walk keeps one u32 per tree level
      *cbvh_stack = std::max(*cbvh_stack, 4u * (uint32_t)depth);
    }
  }
  if (!cbvh.empty()) {
    while (w.size() % 4) w.push_back(0u);
    *cbvh_word0 = (uint32_t)w.size();
    *cbvh_words = (uint32_t)cbvh.size();
    w.insert(w.end(), cbvh.begin(), cbvh.end());
  }
  (void)rec_words;
}

namespace {

uint64_t splitmix(uint64_t& x) {
  uint64_t z = (x += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
double u01(uint64_t& x) { return (double)(splitmix(x) >> 11) * 0x1p-53; }

// One compact tree (rt_layout.h CBVH) as the LDS walk sees it: nodes at byte 48 r, the reference
// pairs after the n_int nodes, the leaf records after those.
struct CTree {
  const uint8_t* base;  // the tree's block
  uint32_t n_int, n_leaf, root, bytes;
  float node(uint32_t byte) const {
    float f;
    std::memcpy(&f, base + byte, 4);
    return f;
  }
  uint32_t word(uint32_t byte) const {
    uint32_t w;
    std::memcpy(&w, base + byte, 4);
    return w;
  }
};

// The LDS walk of rt_kernel.h cbvh_walk_t for one ray with no closest hit (close_f = +inf: no
// box is culled by a hit, no stack entry dropped), recording its stack slots and region reads.
// TPOS: tmin >= 0 (the world walks); else the general box test of ConstantMedium boundaries.
void emulate_walk(const CTree& T, const double o[3], const double d[3], double tmin, bool tpos,
                  uint32_t stack_slots, WalkCheck& W, uint32_t tree_off) {
  auto fail = [&](const char* what) {
    if (W.errors++ == 0) W.first_error = what;
  };
  // the device's slab reciprocals (rt_kernel.h cbvh_walk_t): f32(rcp_nr1(d_a)), within an ulp of
  // 1/d_a, and NaN for d_a = +-0 (rcp_nr1's 0 * inf; a NaN slab time constrains nothing); the
  // octant from d's sign bit
  const double qnan = std::nan("");
  const double inv[3] = {d[0] == 0.0 ? qnan : 1.0 / d[0], d[1] == 0.0 ? qnan : 1.0 / d[1],
                         d[2] == 0.0 ? qnan : 1.0 / d[2]};
  const bool nx = std::signbit(d[0]), ny = std::signbit(d[1]), nz = std::signbit(d[2]);
  const float ix = (float)inv[0], iy = (float)inv[1], iz = (float)inv[2];
  const float ox = (float)o[0], oy = (float)o[1], oz = (float)o[2];
  const float nox = -(ox * ix), noy = -(oy * iy), noz = -(oz * iz);
  const float tmin_f = (float)(tmin - std::fabs(tmin) * 0x1p-20);
  const float close_f = HUGE_VALF;
  constexpr float kBoxRel = 0x1p-20f, kBoxPos = 1.0f + 0x1p-18f;
  const uint32_t onx = nx ? 8u : 0u, ony = ny ? 24u : 16u, onz = nz ? 40u : 32u;
  auto box = [&](float tnx, float tfx, float tny, float tfy, float tnz, float tfz, float& tn) {
    tn = std::fmax(std::fmax(tmin_f, tnx), std::fmax(tny, tnz));
    const float tf = std::fmin(std::fmin(close_f, tfx), std::fmin(tfy, tfz));
    return tpos ? tn <= tf * kBoxPos
                : std::fmaf(-std::fabs(tn), kBoxRel, tn) <= std::fmaf(std::fabs(tf), kBoxRel, tf);
  };
  auto entry = [](uint32_t child, float tn) {
    uint32_t b;
    std::memcpy(&b, &tn, 4);
    return child | (tn < 0.0f ? 0xff800000u : (b & 0xffff0000u));
  };
  auto read = [&](uint32_t byte, uint32_t n) {
    W.max_read = std::max<uint64_t>(W.max_read, (uint64_t)tree_off + byte + n);
    if (byte + n > T.bytes) fail("LDS walk read past its tree's block");
  };
  constexpr uint32_t kDone = 0xffffu;
  uint32_t stack[RTL_CBVH_STACK + 2];
  uint32_t ref = T.root, sp = 0;
  auto pop = [&]() -> uint32_t {
    const float cut = tpos ? close_f * kBoxPos : std::fmaf(std::fabs(close_f), kBoxRel, close_f);
    while (sp > 0) {
      const uint32_t e = stack[--sp];
      const uint32_t hb = e & 0xffff0000u;
      float tb;
      std::memcpy(&tb, &hb, 4);
      const bool drop = tpos ? (tb > cut) : (std::fmaf(-std::fabs(tb), kBoxRel, tb) > cut);
      if (!drop) return e & 0xffffu;
    }
    return kDone;
  };
  ++W.rays;
  for (uint64_t guard = 0; guard < 4ull * (T.n_int + T.n_leaf) + 8; ++guard) {
    while (ref < 0x8000u) {
      if (ref >= T.n_int) return fail("internal reference out of range");
      const uint32_t nb = ref * 48u;
      read(nb, 48u);
      read(T.n_int * 48u + 4u * ref, 4u);
      auto pair = [&](uint32_t off, float& a, float& b) {
        a = T.node(nb + off);
        b = T.node(nb + off + 4u);
      };
      float NX0, NX1, FX0, FX1, NY0, NY1, FY0, FY1, NZ0, NZ1, FZ0, FZ1;
      pair(onx, NX0, NX1), pair(onx ^ 8u, FX0, FX1);
      pair(ony, NY0, NY1), pair(ony ^ 8u, FY0, FY1);
      pair(onz, NZ0, NZ1), pair(onz ^ 8u, FZ0, FZ1);
      const uint32_t rr = T.word(T.n_int * 48u + 4u * ref);
      float tn0, tn1;
      const bool h0 = box(std::fmaf(NX0, ix, nox), std::fmaf(FX0, ix, nox), std::fmaf(NY0, iy, noy),
                          std::fmaf(FY0, iy, noy), std::fmaf(NZ0, iz, noz), std::fmaf(FZ0, iz, noz),
                          tn0);
      const bool h1 = box(std::fmaf(NX1, ix, nox), std::fmaf(FX1, ix, nox), std::fmaf(NY1, iy, noy),
                          std::fmaf(FY1, iy, noy), std::fmaf(NZ1, iz, noz), std::fmaf(FZ1, iz, noz),
                          tn1);
      const bool first0 = h0 && (!h1 || (tn0 <= tn1));
      const uint32_t r0 = rr & 0xffffu, r1 = rr >> 16;
      // the far child is stored to slot sp on every step (rt_kernel.h: no branch around the
      // store) and kept only when both children are hit
      W.max_store_slot = std::max(W.max_store_slot, sp);
      if (sp >= stack_slots || sp > RTL_CBVH_STACK) return fail("stack store past the lane's slots");
      stack[sp] = first0 ? entry(r1, tn1) : entry(r0, tn0);
      if (h0 && h1) ++sp;
      W.max_live = std::max(W.max_live, sp);
      ++W.steps;
      ref = (h0 || h1) ? (first0 ? r0 : r1) : pop();
    }
    if (ref == kDone) return;
    if ((ref & 0x7fffu) >= T.n_leaf) return fail("leaf reference out of range");
    read(T.n_int * 52u + 4u * (ref & 0x7fffu), 4u);
    ref = pop();
  }
  fail("walk did not end");
}

}  // namespace

WalkCheck check_compact_trees(const std::vector<uint32_t>& w, const rtl_scene_header& hdr,
                              uint32_t n_rays, uint64_t seed) {
  WalkCheck W;
  auto fail = [&](const std::string& what) {
    if (W.errors++ == 0) W.first_error = what;
  };
  // a leaf record the walks load: a QUAD / QUADS / SPHERE record inside the record region
  auto leaf_ok = [&](uint32_t rec) {
    rec &= ~RTL_LEAF_BOX;
    const uint32_t ty = rec < hdr.n_rec_words ? (w[rec] & 0xffu) : 0xffu;
    size_t end = 0;
    if (ty == RTL_QUADS) end = (size_t)rec + 4 + (size_t)(w[rec] >> 8) * RTL_QUAD_WORDS;
    else if (ty == RTL_QUAD) end = (size_t)rec + RTL_QUAD_WORDS;
    else if (ty == RTL_SPHERE) end = (size_t)rec + RTL_SPHERE_WORDS;
    return end != 0 && end <= hdr.n_rec_words;
  };
  uint64_t rng = seed ^ 0x5851F42D4C957F2Dull;
  if (hdr.cbvh_words == 0) return W;
  const size_t region0 = hdr.cbvh_word0, region_bytes = (size_t)hdr.cbvh_words * 4u;
  if (region0 % 4 != 0 || region0 + hdr.cbvh_words > w.size()) {
    fail("CBVH region outside the node array");
    return W;
  }
  const uint8_t* region = reinterpret_cast<const uint8_t*>(w.data() + region0);
  const uint32_t stack_slots = hdr.cbvh_stack / 4u;
  for (size_t p = 0; p < hdr.n_rec_words; p += record_words(w[p])) {
    if ((w[p] & 0xffu) != RTL_BVH || w[p + 3] == 0u) continue;
    const uint32_t ob = w[p + 3];
    if ((size_t)ob + 4 > w.size()) {
      fail("ordered-BVH header outside the node array");
      continue;
    }
    if (w[ob + 1] == 0xffffffffu) continue;  // no compact copy: walked from the global streams
    CTree T;
    const uint32_t n_entries = w[ob], off = w[ob + 1];
    T.n_int = n_entries ? (n_entries - 1u) >> 1 : 0u;
    T.n_leaf = T.n_int + 1u;
    T.root = w[ob + 2] & 0xffffu;
    const size_t words = T.n_int ? ((size_t)T.n_int * 13 + T.n_leaf + 3) & ~(size_t)3 : 4u;
    T.bytes = (uint32_t)(words * 4);
    ++W.trees;
    if (n_entries == 0 || (n_entries & 1u) == 0u || off % 16 != 0 || off + (size_t)T.bytes > region_bytes) {
      fail("compact tree block malformed or outside the CBVH region");
      continue;
    }
    T.base = region + off;
    // structure: every internal node and leaf reached exactly once from the root; depth
    std::vector<uint8_t> seen_int(T.n_int, 0), seen_leaf(T.n_leaf, 0);
    uint32_t depth = 0;
    bool ok = true;
    std::vector<std::pair<uint32_t, uint32_t>> todo = {{T.root, 1u}};
    while (!todo.empty() && ok) {
      const auto [r, dd] = todo.back();
      todo.pop_back();
      if (r >= 0x8000u) {
        const uint32_t li = r & 0x7fffu;
        if (r == 0xffffu || li >= T.n_leaf || seen_leaf[li]++) {
          fail("leaf reference invalid or reached twice");
          ok = false;
          break;
        }
        if (!leaf_ok(T.word(T.n_int * 52u + 4u * li))) {
          fail("leaf record is not a QUAD / QUADS / SPHERE record inside the record region");
          ok = false;
        }
        continue;
      }
      if (r >= T.n_int || seen_int[r]++) {
        fail("internal reference invalid or reached twice");
        ok = false;
        break;
      }
      depth = std::max(depth, dd);
      const uint32_t rr = T.word(T.n_int * 48u + 4u * r);
      todo.push_back({rr >> 16, dd + 1});
      todo.push_back({rr & 0xffffu, dd + 1});
    }
    if (!ok) continue;
    for (uint32_t k = 0; k < T.n_int; ++k) ok = ok && seen_int[k];
    for (uint32_t k = 0; k < T.n_leaf; ++k) ok = ok && seen_leaf[k];
    if (!ok) {
      fail("a node or leaf of the block is unreachable from the root");
      continue;
    }
    if (T.n_int == 0) depth = 1;  // a single leaf (rt_obvh.cpp compact_tree)
    W.max_depth = std::max(W.max_depth, depth);
    if (4u * depth > hdr.cbvh_stack) fail("tree deeper than the header's cbvh_stack");
    if (T.n_int == 0) continue;
    // the root box: both children of node 0
    double lo[3], hi[3];
    for (int a = 0; a < 3; ++a) {
      lo[a] = std::min(T.node(16u * a), T.node(16u * a + 4u));
      hi[a] = std::max(T.node(16u * a + 8u), T.node(16u * a + 12u));
    }
    for (uint32_t k = 0; k < n_rays; ++k) {
      double o[3], d[3];
      for (int a = 0; a < 3; ++a) {
        const double ext = hi[a] - lo[a];
        o[a] = lo[a] - 0.25 * ext + 1.5 * ext * u01(rng);
      }
      double n2 = 0.0;
      do {
        n2 = 0.0;
        for (int a = 0; a < 3; ++a) d[a] = 2.0 * u01(rng) - 1.0, n2 += d[a] * d[a];
      } while (n2 > 1.0 || n2 < 1e-6);
      if (k % 8 == 7) d[k / 8 % 3] = (k & 64) ? -0.0 : 0.0;  // a ray in a slab plane: 1/d = +-inf
      const bool tpos = (k & 1) == 0;
      emulate_walk(T, o, d, tpos ? 1e-4 : -HUGE_VAL, tpos, stack_slots, W, off);
    }
  }
  if (W.max_read > region_bytes) fail("LDS walk read past the CBVH region");
  return W;
}

}  // namespace rtf
