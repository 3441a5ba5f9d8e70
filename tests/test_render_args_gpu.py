"""rt_render's argument checks (include/rt_mi355x.h status codes; rt_device.hip
render_device_rows): a row range outside the image, a bad row step or stratum range, a depth
beyond the 24-bit field, and sizes beyond the 32-bit pixel/sample keys or the lane-key fields
are refused with RT_ERR_INVALID_ARG / RT_ERR_UNSUPPORTED before anything is launched, and the
scene stays usable. The reference has no such limits (it panics or loops on absurd input,
render.rs:144-216); these are the boundary's."""
import numpy as np
import pytest

import surely_rt as rt

pytestmark = pytest.mark.gpu


def test_render_rejects_out_of_range_arguments(gpu_available):
    blob, cam = rt.preset_blob("cornell_box", width=32, spp=4)
    ds = rt.DeviceScene(blob)
    try:
        ref, _ = ds.render(cam, rt.make_opts(cam, seed=3))

        def code(c, o):
            with pytest.raises(rt.RtError) as e:
                ds.render(c, o)
            return e.value.code

        H, S = cam.image_height, cam.sqrt_spp
        # rows 30, 32: the second lies outside a 32-row image
        assert code(cam, rt.make_opts(cam, row_begin=H - 2, row_step=2, n_rows=2)) == \
            rt.RT_ERR_INVALID_ARG
        bad_step = rt.make_opts(cam, n_rows=1)
        bad_step.row_step = 0
        assert code(cam, bad_step) == rt.RT_ERR_INVALID_ARG
        # stratum rows [1, 1 + S) exceed the S stratum rows
        assert code(cam, rt.make_opts(cam, sj_begin=1, sj_count=S)) == rt.RT_ERR_INVALID_ARG
        deep = rt.RtCamera.from_buffer_copy(cam)
        deep.max_depth = 1 << 24  # the depth word keeps 24 bits beside the special-value state
        assert code(deep, rt.make_opts(deep)) == rt.RT_ERR_INVALID_ARG
        wide = rt.RtCamera.from_buffer_copy(cam)
        wide.image_width, wide.image_height = 70000, 1  # x is a 16-bit lane-key field
        assert code(wide, rt.make_opts(wide, n_rows=1)) == rt.RT_ERR_UNSUPPORTED
        dense = rt.RtCamera.from_buffer_copy(cam)
        dense.sqrt_spp = dense.samples_per_pixel = 40000  # s_j, s_i fields: sqrt_spp <= 32768
        assert code(dense, rt.make_opts(dense, n_rows=1)) == rt.RT_ERR_UNSUPPORTED
        # the refused calls left nothing behind: the same render again, bit for bit
        again, _ = ds.render(cam, rt.make_opts(cam, seed=3))
        assert np.array_equal(again, ref)
    finally:
        ds.close()
