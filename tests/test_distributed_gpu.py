"""The multi-rank path with the HIP library: two processes joined by a gloo
process group each render their cyclic rows with librtmi355x.so on the box's GPU (device 0) and
gather the frame to rank 0 (surely_rt.parallel.gather_frame, the helper bench.py drives over
RCCL on N GPUs). The gathered frame must equal a single-process render bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    from pathlib import Path

    import torch

    repo = Path(__file__).resolve().parent.parent
    sys.path.insert(0, str(repo / "surely-raytracing_amd"))
    import surely_rt as rt
    from surely_rt.parallel import cyclic_rows, gather_frame, max_rows

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        blob, cam = rt.preset_blob("cornell_box", width=64, spp=16)
        H, W = cam.image_height, cam.image_width
        b, s, n = cyclic_rows(H, rank, world)
        ds = rt.DeviceScene(blob, device=0)
        part, _ = ds.render(cam, rt.make_opts(cam, seed=3, row_begin=b, row_step=s, n_rows=n))
        local = torch.zeros((max_rows(H, world), W, 3), dtype=torch.float32)
        local[:n] = torch.from_numpy(part)
        frame = gather_frame(local, H, rank, world)
        if rank == 0:
            full, _ = ds.render(cam, rt.make_opts(cam, seed=3))
            q.put(bool(np.array_equal(frame.numpy(), full)))
        ds.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gloo_ranks_render_with_hip_and_gather(gpu_available, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5) is True
