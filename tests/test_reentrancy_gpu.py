"""Re-entrancy of one device scene ("re-entrant per distinct output buffer"; the
reference's render_par_lights takes &HittableList and may run concurrently, render.rs:144-150).

Renders of ONE rt_scene issued on two HIP streams at once, and from two host threads at once,
each into its own buffer, must give their serial images bit for bit (include/rt_mi355x.h: every
render call takes its own slot of pool-queue word, counters and workspace)."""
import threading

import numpy as np
import pytest

import surely_rt as rt

pytestmark = pytest.mark.gpu

CASES = [("cornell_box", dict(width=400, spp=256)),
         ("final_scene", dict(width=200, spp=64, depth=12))]


@pytest.mark.parametrize("name,kw", CASES)
def test_two_streams_render_one_scene_concurrently(gpu_available, name, kw):
    from hip_buf import DevBuf, Stream

    blob, cam = rt.preset_blob(name, **kw)
    ds = rt.DeviceScene(blob)
    seeds = (11, 12)
    serial = [ds.render(cam, rt.make_opts(cam, seed=s))[0] for s in seeds]
    assert not np.array_equal(serial[0], serial[1])
    ones = np.ones(serial[0].shape, np.float32)
    # accumulate mode, serially: ones + the render's sums (rounded once, from f64)
    serial_acc = [ds.render(cam, rt.make_opts(cam, seed=s, flags=0), accum=ones.copy())[0]
                  for s in seeds]
    streams = [Stream(), Stream()]
    bufs = [DevBuf(serial[0].shape), DevBuf(serial[0].shape)]
    try:
        # three rounds back to back, nothing synchronised in between: both streams' renders are
        # in flight together, and each stream reuses its own slot in stream order
        for _ in range(3):
            for s, st, b in zip(seeds, streams, bufs):
                ds.render_device(cam, rt.make_opts(cam, seed=s), b.ptr, st.handle)
        for st in streams:
            st.sync()
        for b, ref in zip(bufs, serial):
            assert np.array_equal(b.download(), ref)
        # accumulate mode on both streams at once: each buffer gets its own render added
        for b in bufs:
            b.upload(ones)
        for s, st, b in zip(seeds, streams, bufs):
            ds.render_device(cam, rt.make_opts(cam, seed=s, flags=0), b.ptr, st.handle)
        # a synchronous render with stats meanwhile (its own slot, third stream = NULL)
        again, stt = ds.render(cam, rt.make_opts(cam, seed=seeds[0]))
        assert np.array_equal(again, serial[0]) and stt.samples == cam.image_width * cam.image_height * cam.samples_per_pixel
        for st in streams:
            st.sync()
        for b, ref in zip(bufs, serial_acc):
            assert np.array_equal(b.download(), ref)
    finally:
        for b in bufs:
            b.free()
        for st in streams:
            st.destroy()
        ds.close()


@pytest.mark.parametrize("name,kw", CASES[:1])
def test_two_host_threads_render_one_scene(gpu_available, name, kw):
    blob, cam = rt.preset_blob(name, **kw)
    ds = rt.DeviceScene(blob)
    seeds = (21, 22)
    serial = {s: ds.render(cam, rt.make_opts(cam, seed=s))[0] for s in seeds}
    got: dict[int, list] = {s: [] for s in seeds}
    errors: list[BaseException] = []

    def work(s):
        try:
            for _ in range(4):
                acc, st = ds.render(cam, rt.make_opts(cam, seed=s))
                got[s].append((acc, st.samples))
        except BaseException as e:  # surfaced in the main thread
            errors.append(e)

    th = [threading.Thread(target=work, args=(s,)) for s in seeds]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    ds.close()
    assert not errors, errors
    for s in seeds:
        assert len(got[s]) == 4
        for acc, n in got[s]:
            assert np.array_equal(acc, serial[s])
            assert n == cam.image_width * cam.image_height * cam.samples_per_pixel


def test_per_thread_default_stream_from_two_threads(gpu_available):
    """hipStreamPerThread has one handle value but is a different stream in each host thread
    (ADVICE r4): a render must not take a slot whose previous render, issued by another thread
    on "the same" handle, may still be running. Each thread issues four renders back to back on
    hipStreamPerThread without synchronising, then checks its buffer."""
    from hip_buf import DevBuf, hip

    blob, cam = rt.preset_blob("cornell_box", width=400, spp=256)
    ds = rt.DeviceScene(blob)
    seeds = (31, 32)
    serial = {s: ds.render(cam, rt.make_opts(cam, seed=s))[0] for s in seeds}
    per_thread = 2  # hipStreamPerThread (hip_runtime_api.h)
    bufs = {s: DevBuf(serial[s].shape) for s in seeds}
    errors: list[BaseException] = []
    got: dict[int, np.ndarray] = {}

    def work(s):
        try:
            for _ in range(4):
                ds.render_device(cam, rt.make_opts(cam, seed=s), bufs[s].ptr, per_thread)
            assert hip().hipStreamSynchronize(per_thread) == 0
            got[s] = bufs[s].download()
        except BaseException as e:  # surfaced in the main thread
            errors.append(e)

    th = [threading.Thread(target=work, args=(s,)) for s in seeds]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    for b in bufs.values():
        b.free()
    ds.close()
    assert not errors, errors
    for s in seeds:
        assert np.array_equal(got[s], serial[s])
