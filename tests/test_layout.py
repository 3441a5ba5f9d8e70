"""The flattened device layout (rt_flatten.cpp, rt_layout.h), host-only: BVH region, span-1
duplicate leaves (hittable.rs:161-162) and the one-walk ConstantMedium boundaries."""
import surely_rt as rt


def test_final_scene_bvh_region_and_duplicate_leaves():
    blob, _ = rt.preset_blob("final_scene", width=32, spp=4)
    st = rt.layout_stats(blob)
    # BvhNode::new over 400 boxes and 1000 spheres: 511 + 1023 nodes, of which
    # 112 + 24 have span 1 and test the same child twice
    assert st["bvh_records"] == 511 + 1023
    assert st["bvh_words"] == 16 * st["bvh_records"]
    assert st["dup_records"] == 112 + 24
    # fog (r = 5000) and the glass-ball medium: sphere boundaries, both one-walk
    assert st["volumes"] == 2 and st["volumes_one_walk_sphere"] == 2
    assert st["bvh_words"] * 4 <= 152 * 1024  # the whole region fits the LDS stage


def test_cornell_smoke_boxes_are_one_walk():
    blob, _ = rt.preset_blob("cornell_smoke", width=32, spp=4)
    st = rt.layout_stats(blob)
    assert st["bvh_records"] == 0 and st["bvh_words"] == 0 and st["dup_records"] == 0
    assert st["volumes"] == 2 and st["volumes_one_walk_quads"] == 2


def test_cornell_box_layout():
    blob, _ = rt.preset_blob("cornell_box", width=32, spp=4)
    st = rt.layout_stats(blob)
    assert st["volumes"] == 0 and st["bvh_records"] == 0
    assert st["lights"] == 2  # the light quad and the glass sphere (main.rs:485-494)


def test_non_fusable_boundaries_keep_two_walks():
    sc = rt.Scene(3)
    white = sc.lambertian((0.7, 0.7, 0.7))
    balls = sc.hittable_list(sc.sphere((0, 0, 0), 1.0, white), sc.sphere((1, 0, 0), 1.0, white))
    general = sc.quad((0, 0, 0), (1, 0.5, 0), (0, 0, 1), white)  # not axis-aligned
    world = sc.hittable_list(sc.constant_medium(balls, 0.5, (1, 1, 1)),
                             sc.constant_medium(sc.create_bvh(sc.hittable_list(
                                 sc.sphere((3, 0, 0), 0.5, white), sc.sphere((4, 0, 0), 0.5, white))),
                                 0.5, (1, 1, 1)),
                             sc.constant_medium(sc.hittable_list(general), 0.5, (1, 1, 1)),
                             sc.constant_medium(sc.translate(sc.sphere((0, 5, 0), 1.0, white),
                                                             (1, 1, 1)), 0.5, (1, 1, 1)))
    blob = sc.serialize(world, None)
    st = rt.layout_stats(blob)
    assert st["volumes"] == 4
    # two spheres, a BVH and a general quad are walked twice; an instanced sphere is one-walk
    assert st["volumes_one_walk_sphere"] == 1 and st["volumes_one_walk_quads"] == 0


def test_span1_duplicates_are_marked():
    sc = rt.Scene(9)
    white = sc.lambertian((0.7, 0.7, 0.7))
    lst = sc.hittable_list(*[sc.sphere((k, 0, 0), 0.3, white) for k in range(5)])
    blob = sc.serialize(sc.hittable_list(sc.create_bvh(lst)), None)
    st = rt.layout_stats(blob)
    # 5 objects: span 5 -> (2, 3); 3 -> (1, 2): five BvhNodes, one of span 1
    assert st["bvh_records"] == 5 and st["dup_records"] == 1


def test_ordered_bvhs_for_primitive_leaf_subtrees():
    """rt_obvh.cpp: final_scene's two BVH subtrees (400 ground boxes = quad batches; 1000 spheres
    under Translate(RotateY)) get ordered BVHs; a BVH whose leaves hold instances does not."""
    blob, cam = rt.preset_blob("final_scene", width=32, spp=4)
    assert rt.layout_stats(blob)["ordered_bvhs"] == 2
    sc = rt.Scene(21)
    white = sc.lambertian((0.73, 0.73, 0.73))
    items = sc.hittable_list(sc.translate(sc.make_box((0, 0, 0), (1, 1, 1), white), (2, 0, 0)),
                             sc.sphere((0, 0, 0), 0.5, white), sc.sphere((0, 2, 0), 0.5, white))
    world = sc.hittable_list(sc.create_bvh(items))
    st = rt.layout_stats(sc.serialize(world, None))
    assert st["bvh_records"] > 0 and st["ordered_bvhs"] == 0


def test_compact_bvhs_fit_the_lds_budget():
    """rt_obvh.cpp / rt_layout.h CBVH: both final_scene trees also get the compact copy that
    cbvh_walk reads from LDS (48-byte two-child nodes, u16 references), and with the per-lane
    stacks of a 768-thread workgroup (one u32 per tree level: final_scene's trees are 10 and 12
    levels deep, so at most 16 x 4 bytes), the f64 sample sums and the Perlin table it fits the
    CU's 160 KiB."""
    blob, cam = rt.preset_blob("final_scene", width=32, spp=4)
    st2 = rt.layout_stats(blob)
    assert st2["compact_bvhs"] == st2["ordered_bvhs"] == 2
    n_leaves = 400 + 1000
    n_int = n_leaves - 2
    assert n_int * 52 + n_leaves * 4 <= st2["compact_bvh_bytes"] <= n_int * 52 + n_leaves * 4 + 32
    stacks, sums, perlin = 16 * 768 * 4, 768 * 24, 4864
    assert st2["compact_bvh_bytes"] + stacks + sums + perlin + 512 <= 160 * 1024
