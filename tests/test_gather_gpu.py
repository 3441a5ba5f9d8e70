"""The C-ABI framebuffer gather (include/rt_gather.h, librtgather.so): RCCL over xGMI for one
process per GPU, the C counterpart of bench.py's torch.distributed gather.

On the one-GPU test box: the de-interleave of three ranks' cyclic shares (rendered one after the
other with rt_render_device) must give the single-render frame bit for bit, and an RCCL
communicator of one rank must gather a frame through ncclGather unchanged."""
import os

import numpy as np
import pytest

import surely_rt as rt

pytestmark = pytest.mark.gpu


def test_deinterleave_of_three_shares_is_the_frame(gpu_available):
    from hip_buf import DevBuf
    from surely_rt.parallel import cyclic_rows, gather_lib, max_rows

    blob, cam = rt.preset_blob("cornell_box", width=61, spp=16)
    H, W, N = cam.image_height, cam.image_width, 3
    ds = rt.DeviceScene(blob)
    full, _ = ds.render(cam, rt.make_opts(cam, seed=5))
    m = max_rows(H, N)
    gathered = DevBuf((N, m, W, 3))
    frame = DevBuf((H, W, 3))
    try:
        for r in range(N):
            b, s, n = cyclic_rows(H, r, N)
            part, _ = ds.render(cam, rt.make_opts(cam, seed=5, row_begin=b, row_step=s, n_rows=n))
            host = gathered.download()
            host[r, :n] = part
            gathered.upload(host)
        assert gather_lib().rt_gather_deinterleave(gathered.ptr, N, W, H, frame.ptr, None) == 0
        assert np.array_equal(frame.download(), full)
    finally:
        gathered.free()
        frame.free()
        ds.close()


@pytest.mark.timeout(180)
def test_rccl_gather_of_one_rank(gpu_available):
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    from hip_buf import DevBuf
    from surely_rt.parallel import RcclFrameGather

    blob, cam = rt.preset_blob("cornell_box", width=48, spp=9)
    H, W = cam.image_height, cam.image_width
    ds = rt.DeviceScene(blob)
    local = DevBuf((H, W, 3))
    scratch = DevBuf((H, W, 3))
    frame = DevBuf((H, W, 3))
    comm = RcclFrameGather(RcclFrameGather.unique_id(), world=1, rank=0, device=0)
    try:
        ds.render_device(cam, rt.make_opts(cam, seed=2), local.ptr)
        comm.gather(local.ptr, W, H, scratch.ptr, frame.ptr)
        ref, _ = ds.render(cam, rt.make_opts(cam, seed=2))
        assert np.array_equal(frame.download(), ref)
    finally:
        comm.close()
        for b in (local, scratch, frame):
            b.free()
        ds.close()
