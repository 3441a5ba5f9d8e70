// rt_layout.h — device-resident scene layout (built by rt_flatten.cpp, read by rt_device.hip).
//
// The reference walks its object graph recursively (HittableList::hit hittable.rs:88-109,
// BvhNode::hit :216-236, Translate/RotateY::hit transform.rs:57-135). On the GPU the graph is
// flattened into ONE threaded pre-order word array: every node is followed in memory by its
// first child, and carries a `skip` link to the first node after its subtree. Traversal is a
// stack-free loop: "descend" = advance to the next node, "bbox miss" = follow skip. Visiting
// order is exactly the reference's depth-first, left-then-right order, so the interval
// shrinking (closest_so_far), tie behaviour and ConstantMedium RNG draw order are unchanged.
//
// Lists vanish (their children are simply consecutive). A Translate/RotateY node changes the
// lane's local ray; an EXIT node after its subtree restores the parent frame by re-applying the
// parent's transform chain to the world ray (same arithmetic as the recursive descent). The
// boundary of a ConstantMedium is a sub-sequence terminated by END, traversed twice with its
// own closest-hit state (constant_medium.rs:46-55).
//
// Word = 4 bytes; node offsets are word indices; every node starts 16-byte aligned.
//
// Addresses vs order (rt_flatten.cpp relocate): after emission every BVH record is moved to
// the front, the BVH region [0, bvh_words), which rt_trace stages in LDS; the other records
// keep their relative order after it. Links are therefore explicit: a BVH record holds its
// first child in word 2 (its skip in word 1), every other record its pre-order successor in
// word 3 ("next": where the walk continues after a primitive, and the child of an instance,
// volume or DUP). Quads of a QUADS batch stay contiguous.
#pragma once
#include <stdint.h>

#define RTL_END 0
#define RTL_QUAD 1
#define RTL_SPHERE 2
#define RTL_BVH 3
#define RTL_TRANSLATE 4
#define RTL_ROTATE_Y 5
#define RTL_EXIT 6
#define RTL_VOLUME 7
#define RTL_OTHER 8 /* light entry whose pdf_value is 0 (Object default arm, object.rs:295-311) */
#define RTL_LLIST 11 /* light table only: a HittableList nested in the light list (object.rs:57, 66):
                       [hdr | count << 8][first entry][0][0] d0 = 1.0 / count; its children are
                       the light entries [first, first + count) */
#define RTL_LLIST_WORDS 8
#define RTL_LIGHT_NEST 4 /* light lists nested at most this deep below the top-level list */
#define RTL_QUADS 9 /* batch of consecutive sibling quads: header word 0 = type | count << 8, then
                       `count` QUAD records; traversed in order, exactly like the list it replaces */
#define RTL_DUP 10  /* the right child of a BvhNode whose two children are the same deterministic
                       subtree (span-1 leaves, hittable.rs:161-162): [hdr][skip][0][0], then the
                       subtree. Re-testing it with [t_min, rec.t] (hittable.rs:223-228) reproduces
                       the left child's record exactly, so the renderer jumps to skip; the
                       op-counting build walks it, so counts stay the reference's. */
#define RTL_DUP_WORDS 4
/* header word 0: type | (flags << 8); word 1: skip (next node after the subtree).
 * Payloads are f64 (the reference computes in f64) starting at word 4, read as
 * 16-byte double2 pairs. dN = double index N counted from word 4. */
/* QUAD (36 words): [hdr][skip][mat][next] d0-1 n.xy | d2-3 n.z,D | d4-5 q.xy | d6-7 q.z,area |
 *   d8-9 A.xy | d10-11 A.z,0 | d12-13 B.xy | d14-15 B.z,0      with A = v x w, B = w x u, so
 *   the planar coordinates of object.rs:469-470, a = w.(pq x v) and b = w.(u x pq), are the
 *   same triple products evaluated as a = pq.A, b = pq.B (two dots instead of two crosses and
 *   two dots per test).                                                  object.rs:414-490
 * Light records (LQUAD) append d16-19 u.xyz,0 and d20-23 v.xyz,0 for Quad::random
 * (object.rs:503-506). */
/* World QUAD records (48 words) put an axis-aligned form FIRST, so one 64-byte scalar load
 * covers the header and everything the axis-aligned test reads, and the general payload after it:
 *   [hdr | axis << 8][skip][mat][next] d0-5 q_k, y0_lo, y1_lo, y0_hi, y1_hi, 0 | d6-21 general payload
 * (the QUAD layout above, read through X + RTL_QUAD_GEN). axis = k + 1 when the quad is
 * axis-aligned in its frame (u along axis i, v along axis j, normal along k; 0 = general). Then
 * n = +-e_k, D = +-q_k, and A, B each have one non-zero component, so the general test's
 *   t = (D - n.o) / (n.d) = (q_k - o_k) / d_k,   a = pq.A = pq_i A_i,   b = pq.B = pq_j B_j
 * hold bit for bit (the dropped terms are exact zeros), with pq_i = y_i - q_i, y = o + t d.
 * a = fl(fl(y_i - q_i) A_i) is monotone in y_i, so "a in [0, 1] or NaN" is "y_i in [y0, y1] or
 * NaN" for two doubles the flattener finds by bisection (rt_flatten.cpp accept_interval): the
 * device compares y with them instead of forming a and b. lo/hi = the in-plane axes in ascending
 * order: the accept test on (a, b) is symmetric, so only k varies per record. rt_flatten.cpp
 * verifies the zero pattern (and finite, non-zero q, C) before setting the form. */
#define RTL_QUAD_GEN 12
#define RTL_QUAD_WORDS 48
#define RTL_QUAD_AXIS(h) (((h) >> 8) & 0x3u)
/* Light QUAD records (64 words) = the general layout, u, v, then the axis-aligned form at
 * d24-28 (header axis bits as for world quads) for HittablePDF's hit test (object.rs:493). */
#define RTL_LQUAD_WORDS 64
#define RTL_LQUAD_AXIS_D 24
/* SPHERE (20 words): [hdr | moving][skip][mat][next] d0-3 c.xyz,r | d4-7 cvec.xyz,1/r
 *                                                                             object.rs:73-105 */
#define RTL_SPHERE_MOVING 0x100u
#define RTL_SPHERE_WORDS 20
/* BVH (16 words): [hdr][skip][child][obvh] d0-5 xmin xmax ymin ymax zmin zmax hittable.rs:135-187
 *   obvh: word offset of the subtree's ordered BVH (below), 0 = none (walk the reference tree).
 * OBVH (rt_obvh.cpp), for a BVH subtree whose leaves are QUAD / QUADS / SPHERE records: an SAH
 * BVH2 over the same leaf records, appended after the record region (n_rec_words):
 *   [n_entries][cbvh block][root ref][streams_off = 8][0][0][0][0]  (word offsets from the header)
 *   streams: 8 ray-direction octants (bit a set = d_a < 0, by sign bit) x n_entries x 8 words,
 *   each a threaded pre-order walk with the near child first. Internal entry:
 *   [skip][0][near_x][far_x][near_y][far_y][near_z][far_z] (f32 bounds of the node's box for the
 *   octant, outward-rounded with margin: box hit -> next entry, miss -> skip); leaf entry:
 *   [0x80000000][record][the leaf's own box, as above] (box hit -> test the record; then the
 *   next entry). Header words 1-2: the tree's block in the CBVH region (byte offset, 0xffffffff =
 *   none) and its root reference.
 * CBVH: the same trees, compact, for the walk from LDS (rt_kernel.h cbvh_walk): one contiguous
 *   region after the OBVHs (header cbvh_word0 / cbvh_words) of 16-byte aligned blocks, one per
 *   tree: n_int internal nodes of 48 bytes (both children's boxes as f32, outward-rounded as
 *   above, blocked per axis: [lo_x c0, lo_x c1, hi_x c0, hi_x c1, lo_y c0, ..., hi_z c1], so a
 *   lane reads its octant's near and far pair of an axis with one 8-byte load each), n_int u32
 *   child-reference pairs (ref0 | ref1 << 16;
 *   ref < 0x8000: internal node, else leaf index ref & 0x7fff), n_int + 1 u32 leaf records.
 *   Internal-node depth <= RTL_CBVH_STACK; the walk's per-lane LDS stack holds one u32 per
 *   level of the deepest tree (child reference | bf16 entry time << 16), header cbvh_stack.
 */
#define RTL_CBVH_STACK 32
/* Leaf record words of the OBVH streams and CBVH leaf arrays carry RTL_LEAF_BOX when the record is
 * a QUADS batch of make_box's six sides in its order (rt_obvh.cpp make_box_batch); the record's
 * word offset is the low 31 bits. */
#define RTL_LEAF_BOX 0x80000000u
#define RTL_BVH_WORDS 16
/* TRANSLATE / ROTATE_Y (16 words):
 *   [hdr][skip][chain_len][next] [chain0..3: transform nodes root->self] d2-5 p0 p1 p2 0
 *   translate: p = offset.xyz; rotate_y: p0 = sin, p1 = cos                  transform.rs */
#define RTL_XFORM_WORDS 16
#define RTL_MAX_CHAIN 4
/* A chain longer than RTL_MAX_CHAIN (transform.rs nests without a limit): header flag
 * RTL_XFORM_LONG, word 4 = word offset of the chain (chain_len words, root first) in a table
 * appended after the records. */
#define RTL_XFORM_LONG 0x100u
/* EXIT (4 words): [hdr][skip=unused][parent frame node or -1][next] */
#define RTL_EXIT_WORDS 4
/* VOLUME header flags: the boundary is [Translate|RotateY]* then one sphere, or one batch (or
 * one record) of axis-aligned quads, then EXITs and END; rt_trace then finds both boundary
 * hits (constant_medium.rs:46-55) in ONE walk (the closest-hit semantics of the two passes
 * reduce to "smallest candidate" and "smallest candidate >= t1 + 1e-4"). */
#define RTL_VOLF_SPHERE 0x100u
#define RTL_VOLF_QUADS 0x200u
/* VOLUME (8 words): [hdr][skip][mat][next] d0 neg_inv_density, d1 0; the boundary follows and an
 * END node terminates it                                                    constant_medium.rs */
#define RTL_VOLUME_WORDS 8
/* ConstantMedium records nested inside volume boundaries (constant_medium.rs:46-55 queries
 * `boundary.hit`, which may itself hold a ConstantMedium): walked at most this deep */
#define RTL_VOLUME_NEST 2
#define RTL_END_WORDS 4

/* material (20 words): [kind | flags(bit8: texture reads uv)][tex][0][0] d0-3 c.xyz, param,
 * d4-7 derived constants
 *   METAL: c = albedo, param = fuzz; DIELECTRIC: c = tint, param = ir, d4 = 1/ir,
 *   d5 / d6 = Schlick r0 for the front / back face ratio (material.rs:150-158, 166-191; the same
 *   IEEE divisions the reference performs per hit, done once on the host) */
/* Scene set (a walker's kScene, rt_kernel.h trace_body): material kinds and light-list shapes a
 * scene contains; a scene-specialised walker (rt_jit.cpp) clears the bits of what it lacks. */
#define RTL_SC_METAL 0x1u
#define RTL_SC_DIELECTRIC 0x2u
#define RTL_SC_LIGHT 0x4u       /* a DiffuseLight material                          */
#define RTL_SC_LIGHTS 0x8u      /* a non-empty light list                           */
#define RTL_SC_LLIST 0x10u      /* a HittableList nested in the light list         */
#define RTL_SC_LSPHERE 0x20u    /* a sphere in the light list                       */
#define RTL_SC_LOTHER 0x40u     /* a light that is neither quad, sphere nor list    */
#define RTL_SC_ANY 0xffffffffu
#define RTL_MAT_WORDS 20
#define RTL_MATF_NEEDS_UV 0x100u
/* texture (12 words): [kind][a][b][c] d0-3
 *   SOLID: d0-2 color; CHECKER: d0 inv_scale, a even, b odd;
 *   IMAGE: a width, b height, c byte offset into texels; NOISE: d0 scale, a perlin index */
#define RTL_TEX_WORDS 12
/* perlin table: ranvec 256 x float4 (x, y, z, 0; 4096 B: the turbulence is a radiance weight,
 * rt_kernel.h perlin_turb) + perm_x/y/z 3 x 256 bytes (768 B) */
#define RTL_PERLIN_BYTES (4096 + 768)

/* light entries: node-format QUAD / SPHERE / OTHER records in their own word array */
typedef struct rtl_scene_header {
  uint32_t root;          /* word offset of the world sequence                    */
  uint32_t n_node_words;  /* nodes                                                */
  uint32_t n_mats;
  uint32_t n_texs;
  uint32_t n_perlins;
  uint32_t n_lights;      /* 0 = empty light list                                 */
  uint32_t lights_is_list;/* 1: HittableList (random_int pick + 1/N average)      */
  uint32_t has_bvh;
  uint32_t has_volume;
  uint32_t max_chain;
  uint32_t n_texel_bytes;
  uint32_t pdf_materials; /* any Lambertian / Isotropic                           */
  uint32_t has_textures;  /* a material references a non-solid texture            */
  uint32_t bvh_words;     /* BVH region: node words [0, bvh_words) hold every BVH record */
  uint32_t volume_in_bvh; /* a ConstantMedium lies inside a BVH subtree                */
  uint32_t volumes_one_walk_spheres; /* every ConstantMedium boundary is a one-walk sphere */
  uint32_t has_isotropic; /* some material is Isotropic (also outside a ConstantMedium)  */
  uint32_t n_rec_words;   /* node words holding records; ordered BVHs follow (OBVH below) */
  uint32_t lights_nested; /* some light entry is a nested HittableList (RTL_LLIST)    */
  uint32_t nested_volumes;/* a ConstantMedium lies inside another one's boundary      */
  uint32_t cbvh_word0;    /* CBVH region (below): first node word, 0 = none            */
  uint32_t cbvh_words;    /* its size in words (a multiple of 4)                        */
  uint32_t cbvh_stack;    /* walk stack bytes per lane: 4 x the trees' largest depth     */
} rtl_scene_header;
