"""The C-ABI libraries load and export every symbol their headers declare; blob validation
(host-only, no GPU) accepts reference scenes and rejects malformed ones with a status code."""
import ctypes as C
import re
from pathlib import Path

import numpy as np
import pytest

import surely_rt as rt

REPO = Path(__file__).resolve().parent.parent


def _declared(header: str):
    text = (REPO / "include" / header).read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b((?:rt|rth)_[a-z0-9_]+)\s*\(", text)))


@pytest.mark.parametrize("header,lib", [("rt_mi355x.h", "librtmi355x.so"),
                                        ("rt_host.h", "librthost.so"),
                                        ("rt_gather.h", "librtgather.so")])
def test_exports_every_declared_symbol(header, lib):
    names = _declared(header)
    assert len(names) >= 7
    so = C.CDLL(str(REPO / "build" / lib))
    missing = [n for n in names if not hasattr(so, n)]
    assert not missing, missing


def test_abi_version_and_error_string():
    lib = rt.device_lib()
    assert lib.rt_abi_version() == 3
    assert isinstance(lib.rt_last_error(), bytes)


def test_validate_accepts_all_presets():
    lib = rt.device_lib()
    for name in ["cornell_box", "cornell_smoke", "final_scene", "quads", "simple_light",
                 "two_spheres", "two_perlin_spheres", "random_balls", "three_spheres", "earth"]:
        blob, cam = rt.preset_blob(name, width=32, spp=4)
        assert lib.rt_scene_validate(blob.ref()) == rt.RT_OK, (name, lib.rt_last_error())


def test_validate_rejects_malformed_blobs():
    lib = rt.device_lib()
    blob, _ = rt.preset_blob("cornell_box", width=32, spp=4)
    bad = blob.slots.copy()
    bad[0] = 0  # magic
    assert lib.rt_scene_validate(rt.Blob(bad, blob.texels).ref()) == rt.RT_ERR_BAD_BLOB
    bad = blob.slots.copy()
    bad[2] = bad[2] + 1  # size mismatch
    assert lib.rt_scene_validate(rt.Blob(bad, blob.texels).ref()) == rt.RT_ERR_BAD_BLOB
    bad = blob.slots[: int(blob.slots[9]) + 3].copy()  # truncated world tree
    bad[2] = bad.size
    assert lib.rt_scene_validate(rt.Blob(bad, blob.texels).ref()) == rt.RT_ERR_BAD_BLOB
    bad = blob.slots.copy()
    w = int(bad[9])
    bad[w] = 99  # unknown object tag
    assert lib.rt_scene_validate(rt.Blob(bad, blob.texels).ref()) == rt.RT_ERR_BAD_BLOB
    assert "tag" in lib.rt_last_error().decode()


def test_validate_rejects_out_of_range_material():
    sc = rt.Scene(1)
    m = sc.lambertian((0.5, 0.5, 0.5))
    world = sc.hittable_list(sc.sphere((0, 0, 0), 1, m))
    blob = sc.serialize(world)
    slots = blob.slots.copy()
    w = int(slots[9])
    # LIST [tag n bbox6] then SPHERE [tag mat ...]
    slots[w + 8 + 1] = 1000
    lib = rt.device_lib()
    assert lib.rt_scene_validate(rt.Blob(slots, blob.texels).ref()) == rt.RT_ERR_BAD_BLOB


def test_nested_constant_medium_depth_limit():
    """ConstantMedium boundaries may hold ConstantMedium records (constant_medium.rs:46-55);
    the device walks them RTL_VOLUME_NEST = 2 levels deep and reports a deeper nesting as
    RT_ERR_UNSUPPORTED instead of rendering it wrongly."""
    sc = rt.Scene(1)
    glass = sc.dielectric(1.5)
    vol = sc.constant_medium(sc.sphere((0, 0, 0), 1, glass), 0.5, (1, 1, 1))
    for depth in range(1, 4):
        vol = sc.constant_medium(sc.hittable_list(sc.sphere((0, 0, 0), 1 + depth, glass), vol),
                                 0.5, (1, 1, 1))
        blob = sc.serialize(sc.hittable_list(vol))
        want = rt.RT_OK if depth <= 2 else rt.RT_ERR_UNSUPPORTED
        assert rt.device_lib().rt_scene_validate(blob.ref()) == want, depth


def test_product_path_fails_loudly_without_library(tmp_path):
    """No CPU fallback: with the HIP library absent, loading the render path raises."""
    with pytest.raises(RuntimeError, match="HIP library is required"):
        rt.load_device_lib(tmp_path / "librtmi355x.so")


def test_gather_row_layout_host_functions():
    """rt_gather_rows / rt_gather_max_rows (host-only): the cyclic tiling of bench.py and
    surely_rt.parallel (rank r renders rows r, r + N, ...), padded to ceil(H / N)."""
    from surely_rt.parallel import cyclic_rows, gather_lib, max_rows

    g = gather_lib()
    for H in (1, 7, 800, 2160):
        for N in (1, 2, 3, 8):
            assert g.rt_gather_max_rows(H, N) == max_rows(H, N)
            assert sum(g.rt_gather_rows(H, N, r) for r in range(N)) == H
            for r in range(N):
                assert g.rt_gather_rows(H, N, r) == cyclic_rows(H, r, N)[2]
    assert g.rt_gather_rows(5, 0, 0) == 0 and g.rt_gather_max_rows(0, 4) == 0
