"""Render-level properties of the CPU oracle, and its statistical agreement with the only
outputs the reference ships (final_images/*.png, tests/golden/final_images_stats.json)."""
import json
from pathlib import Path

import numpy as np
import pytest

import oracle_lib as O
import surely_rt as rt

GOLD = json.loads((Path(__file__).parent / "golden" / "final_images_stats.json").read_text())


def _decode(u8):
    """Approximate inverse of color.rs linear_to_gamma at the byte's bin centre."""
    g = (u8.astype(np.float64) + 0.5) / 256.0
    return np.where(g <= 12.92 * 0.0031308, g / 12.92, ((g + 0.055) / 1.055) ** 2.4)


@pytest.mark.parametrize("name,tol_mean,tol_blocks", [
    ("book3.png", 0.04, 0.05),
    ("mixed_pdf.png", 0.04, 0.05),
    # cornell_smoke renders under the semantics register; the agreement
    # with the published image supports those decisions
    ("cornell_smoke.png", 0.05, 0.08),
])
def test_matches_reference_render_statistics(name, tol_mean, tol_blocks):
    m = GOLD[name]
    W = 120
    blob, cam = rt.preset_blob(m["preset"], variant=m["variant"], width=W, spp=100, depth=m["depth"])
    acc, _ = O.render(blob, cam, rt.make_opts(cam, seed=1), precision=64)
    lin = _decode(rt.write_color(acc, cam.samples_per_pixel))
    ref = np.array(m["block10_linear"])
    assert lin.mean() == pytest.approx(ref.mean(), rel=tol_mean)
    blocks = lin.reshape(10, W // 10, 10, W // 10, 3).mean(axis=(1, 3))
    rel = np.abs(blocks - ref) / np.maximum(ref, 0.02)
    assert rel.mean() < tol_blocks, rel.mean()


def test_thread_count_and_chunking_invariance():
    """The pool's 3-row chunks (render.rs:171) never change results: samples are keyed by
    (pixel, sample), not by thread or scheduling order."""
    blob, cam = rt.preset_blob("cornell_box", width=45, spp=9)
    a, oa = O.render(blob, cam, rt.make_opts(cam, seed=4), threads=1)
    b, ob = O.render(blob, cam, rt.make_opts(cam, seed=4), threads=7)
    assert np.array_equal(a, b) and oa == ob


def test_row_tiling_and_strata_in_oracle():
    blob, cam = rt.preset_blob("cornell_smoke", width=30, spp=16, depth=10)
    full, _ = O.render(blob, cam, rt.make_opts(cam, seed=2))
    part, _ = O.render(blob, cam, rt.make_opts(cam, seed=2, row_begin=1, row_step=3,
                                               n_rows=len(range(1, 30, 3))))
    assert np.array_equal(part, full[1::3])
    a, _ = O.render(blob, cam, rt.make_opts(cam, seed=2, sj_begin=0, sj_count=1))
    b, _ = O.render(blob, cam, rt.make_opts(cam, seed=2, sj_begin=1, sj_count=3))
    np.testing.assert_allclose(a + b, full, rtol=1e-6, atol=1e-6)


def test_accumulate_adds_into_buffer():
    """render.rs:189 adds into a caller-owned, pre-zeroed buffer; rt flags: 0 = accumulate."""
    blob, cam = rt.preset_blob("quads", width=16, spp=4)
    base, _ = O.render(blob, cam, rt.make_opts(cam))
    acc = np.full_like(base, 2.0)
    O.render(blob, cam, rt.make_opts(cam, flags=0), accum=acc)
    np.testing.assert_allclose(acc, base + 2.0, rtol=1e-6)


def test_f32_precision_study_shows_self_intersection():
    """Why the device computes in f64: at fp32 the reference's fixed
    t_min = 1e-4 (render.rs:267) lets refracted rays re-hit the glass sphere's surface, so far
    more paths run into the depth limit and the image darkens."""
    blob, cam = rt.preset_blob("cornell_box", width=100, spp=16)
    a64, o64 = O.render(blob, cam, rt.make_opts(cam), precision=64)
    a32, o32 = O.render(blob, cam, rt.make_opts(cam), precision=32)
    assert o32["depth_cutoff"] > 10 * max(1, o64["depth_cutoff"])
    assert o32["dielectric"] > 1.1 * o64["dielectric"]
    assert a32.mean() < a64.mean()


def test_reference_semantics_flag_in_oracle():
    blob, cam = rt.preset_blob("quads", width=8, spp=1)
    with pytest.raises(RuntimeError):
        O.render(blob, cam, rt.make_opts(cam, flags=rt.RT_FLAG_OVERWRITE | rt.RT_FLAG_SEMANTICS_REFERENCE))
    # Isotropic scattering_pdf = 0 under reference semantics: fog then only absorbs (S2)
    sc = rt.Scene(1)
    light = sc.diffuse_light((4, 4, 4))
    fog = sc.constant_medium(sc.sphere((0, 0, 0), 2, sc.dielectric(1.5)), 0.5, (1, 1, 1))
    lq = sc.quad((-1, 3, -1), (2, 0, 0), (0, 0, 2), light)
    blob = sc.serialize(sc.hittable_list(fog, lq), sc.hittable_list(
        sc.quad((-1, 3, -1), (2, 0, 0), (0, 0, 2), light)))
    cam = rt.camera_new(1.0, 24, 16, 10, 40, (0, 0, 8), (0, 0, 0), (0, 1, 0), 0, 0, (0, 0, 0))
    book2, _ = O.render(blob, cam, rt.make_opts(cam))
    ref, _ = O.render(blob, cam, rt.make_opts(cam, flags=rt.RT_FLAG_OVERWRITE | rt.RT_FLAG_SEMANTICS_REFERENCE))
    assert book2.sum() > ref.sum()


def _book2_region_means(render, W, spp, seeds):
    """Linear region means (raw sums / spp) of final_scene at W x W for each scene-build seed.
    render(blob, cam, opts) -> accum [n_rows, W, 3]; only the row bands the regions cover are
    rendered."""
    m = GOLD["book2.png"]
    s = 800.0 / W
    regions = m["regions"]
    rows = sorted({j for cx, cy, r in regions.values()
                   for j in range(max(0, int((cy - r) / s) - 1), min(W, int((cy + r) / s) + 2))})
    out = {k: [] for k in regions}
    for seed in seeds:
        blob, cam = rt.preset_blob("final_scene", width=W, spp=spp, depth=m["depth"],
                                   build_seed=seed)
        img = np.zeros((W, W, 3))
        k = 0
        while k < len(rows):  # contiguous bands
            e = k
            while e + 1 < len(rows) and rows[e + 1] == rows[e] + 1:
                e += 1
            acc = render(blob, cam, rt.make_opts(cam, seed=1, row_begin=rows[k], n_rows=e - k + 1))
            img[rows[k]:rows[e] + 1] = acc / cam.samples_per_pixel
            k = e + 1
        yy, xx = np.mgrid[0:W, 0:W]
        for name, (cx, cy, r) in regions.items():
            mask = ((xx + 0.5) * s - cx) ** 2 + ((yy + 0.5) * s - cy) ** 2 < r * r
            out[name].append(img[mask].mean(0))
    return {k: np.array(v) for k, v in out.items()}


def _check_book2(means):
    """Each region's linear mean must agree with book2.png's within 3 standard deviations of the
    scene-build seed spread (the reference's own scene is one unseeded draw of the same random
    geometry) plus 2 % + 1e-3 for the 8-bit quantisation of the PNG and residual noise."""
    ref = GOLD["book2.png"]["region_linear"]
    bad = {}
    for name, v in means.items():
        mu, sd = v.mean(0), v.std(0, ddof=1)
        r = np.array(ref[name])
        tol = 3.0 * sd + 0.02 * r + 1e-3
        if np.any(np.abs(mu - r) > tol):
            bad[name] = (mu.round(5).tolist(), r.tolist(), tol.round(5).tolist())
    assert not bad, bad


def test_final_scene_matches_book2_regions():
    """BASELINE C4's scene against the reference's own final_images/book2.png (800x800, 10000
    spp, depth 40, main.rs:603-712 with selector 9, main.rs:726): the oracle under the semantics
    register (App. A S1: empty light list -> material PDF alone, the book-2 estimator the image
    was rendered with; S2; S3: earth texture absent -> its disk is not compared) renders
    final_scene at 200x200, 256 spp, for four scene-build seeds, and the linear means of five
    fixed objects' disks (tests/golden/final_images_stats.json "regions": motion blur, glass,
    fuzz-1.0 metal, the subsurface ConstantMedium, Perlin turbulence) match the image's."""
    means = _book2_region_means(
        lambda blob, cam, opts: O.render(blob, cam, opts, precision=64)[0], 200, 256, (1, 2, 3, 4))
    _check_book2(means)
