"""rt_render from several host threads at once (a renderer serving requests:
include/rt.h promises a thread-safe library).

ctypes drops the GIL around every foreign call, so the Python threads below
are real concurrent callers of rt_render / rt_render_u8: they share the
per-device scene cache (concurrent misses of one scene, LRU eviction with
more scenes than it keeps), the render contexts (the device's NULL-stream
context and the non-blocking ones), the host worker pool of the fan-out
(interleaved shards on device 0 from several callers at once) and the
per-stream tile orders; one thread also calls rt_cache_clear between its
renders.  Every frame must equal the same call made alone, bit for bit.
"""
from __future__ import annotations

from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest
import torch  # noqa: F401  (before rtclj: conftest.gpu_lib)

pytestmark = pytest.mark.gpu


def _jobs():
    from rtclj import raytracing as R, scenes
    from rtclj._lib import RT_FLAG_SHARDS_ON_DEVICE0, RT_FLAG_REALM
    cover = scenes.cover(11)
    small = scenes.cover(4, seed=7)
    ref = R.Scene.from_bodies(R.hittables)
    jobs = [
        (cover, scenes.cover_camera(96, 54), 96, 54, dict(spp=4, seed=2)),
        (ref, R.camera(64, 36, **R.REFERENCE_CAMERA), 64, 36, dict(spp=3, seed=5)),
        (cover, scenes.cover_camera(80, 45), 80, 45,
         dict(spp=2, seed=3, n_devices=3, flags=RT_FLAG_SHARDS_ON_DEVICE0)),
        (ref, R.camera(48, 27, **R.REFERENCE_CAMERA), 48, 27, dict(spp=2, seed=9, u8=True)),
        (small, scenes.cover_camera(40, 23), 40, 23, dict(spp=5, seed=4, flags=RT_FLAG_REALM)),
        (cover, scenes.cover_camera(72, 40), 72, 40,
         dict(spp=2, seed=6, n_devices=2, flags=RT_FLAG_SHARDS_ON_DEVICE0, u8=True, rows=(5, 37))),
        # five scenes in all: more than the 4 a device caches (LRU eviction under load)
        (scenes.cover(6, seed=1), scenes.cover_camera(56, 32), 56, 32, dict(spp=3, seed=8)),
        (scenes.cover(3, seed=9), scenes.cover_camera(32, 18), 32, 18, dict(spp=6, seed=1)),
    ]
    return jobs


def test_concurrent_renders_equal_serial(gpu_lib):
    from rtclj import raytracing as R
    from rtclj._lib import lib
    jobs = _jobs()
    lib.rt_cache_clear()
    expect = [R.render(sc, cam, w, h, **kw) for sc, cam, w, h, kw in jobs]
    lib.rt_cache_clear()

    def worker(t):
        bad = []
        for i in range(5):
            k = (t + i) % len(jobs)
            sc, cam, w, h, kw = jobs[k]
            got = R.render(sc, cam, w, h, **kw)
            if not np.array_equal(got, expect[k]):
                bad.append((t, i, k))
            if t == 0 and i % 2 == 1:
                lib.rt_cache_clear()   # drops what is idle; in-flight renders keep theirs
        return bad

    with ThreadPoolExecutor(max_workers=6) as ex:
        bad = [b for r in ex.map(worker, range(6)) for b in r]
    assert not bad, bad
    # the library is still whole afterwards: a serial call of each job
    assert all(np.array_equal(R.render(sc, cam, w, h, **kw), e) for (sc, cam, w, h, kw), e in zip(jobs, expect))
    lib.rt_cache_clear()


def test_frames_in_flight_equal_render(gpu_lib):
    """rt_render_submit .. rt_render_wait: every job submitted before any is
    waited on (eight frames in flight: more contexts than the NULL stream's,
    shards of several frames interleaved on device 0, streamed split units),
    then waited on in reverse order; each frame equals rt_render's, bit for
    bit, and its statistics are rt_render's."""
    from rtclj import raytracing as R
    from rtclj._lib import lib
    jobs = _jobs()
    lib.rt_cache_clear()
    expect, est = [], []
    for sc, cam, w, h, kw in jobs:
        st = {}
        expect.append(R.render(sc, cam, w, h, stats=st, **kw))
        est.append(st)
    frames = [R.render_async(sc, cam, w, h, **kw) for sc, cam, w, h, kw in jobs]
    for k in reversed(range(len(jobs))):
        st = {}
        got = frames[k].wait(stats=st)
        assert np.array_equal(got, expect[k]), k
        assert (st["segments"], st["samples"], st["n_devices"]) == \
            (est[k]["segments"], est[k]["samples"], est[k]["n_devices"]), k
        assert st["kernel_ms"] > 0 and st["total_ms"] >= st["wait_ms"]
    with pytest.raises(RuntimeError):
        frames[0].wait()
    lib.rt_cache_clear()


def test_frames_in_flight_from_threads(gpu_lib):
    """Several threads, each keeping two frames in flight (submit the next,
    then wait on the previous: a renderer's frame loop), against rt_render
    called alone; one thread clears the cache between frames."""
    from rtclj import raytracing as R
    from rtclj._lib import lib
    jobs = _jobs()
    lib.rt_cache_clear()
    expect = [R.render(sc, cam, w, h, **kw) for sc, cam, w, h, kw in jobs]

    def worker(t):
        bad, prev = [], None
        for i in range(6):
            k = (t + i) % len(jobs)
            sc, cam, w, h, kw = jobs[k]
            f = (k, R.render_async(sc, cam, w, h, **kw))
            if prev is not None and not np.array_equal(prev[1].wait(), expect[prev[0]]):
                bad.append((t, i, prev[0]))
            prev = f
            if t == 0 and i % 2 == 1:
                lib.rt_cache_clear()
        if not np.array_equal(prev[1].wait(), expect[prev[0]]):
            bad.append((t, "last", prev[0]))
        return bad

    with ThreadPoolExecutor(max_workers=4) as ex:
        bad = [b for r in ex.map(worker, range(4)) for b in r]
    assert not bad, bad
    lib.rt_cache_clear()


def test_submit_errors_and_dropped_frame(gpu_lib):
    """rt_render's argument errors come from rt_render_submit (no frame is
    made); rt_render_wait(NULL) is an argument error; a frame dropped without
    a wait is waited on by its finaliser and the library stays whole."""
    import ctypes as C
    from rtclj import raytracing as R, scenes
    from rtclj._lib import RTError, lib, rt_params
    sc = scenes.cover(4, seed=3)
    cam = scenes.cover_camera(32, 18)
    with pytest.raises(RTError, match="rt_render_submit: bad width"):
        R.render_async(sc, cam, 32, 18, spp=-1)
    with pytest.raises(RTError, match="rt_render_submit: bad row range"):
        R.render_async(sc, cam, 32, 18, spp=1, rows=(10, 40))
    p = rt_params(width=32, height=18, row_begin=0, row_end=18, spp=1, max_depth=5, seed=1, row_tile=8)
    out = np.empty((18, 32, 3), np.float32)
    code = lib.rt_render_submit(C.byref(sc.c), C.byref(cam), C.byref(p),
                                out.ctypes.data_as(C.POINTER(C.c_float)), out.size, None)
    assert code < 0 and b"NULL frame" in lib.rt_last_error()
    assert lib.rt_render_wait(None, None) < 0 and b"NULL frame" in lib.rt_last_error()
    f = R.render_async(sc, cam, 32, 18, spp=2, seed=4)
    del f
    assert np.array_equal(R.render_async(sc, cam, 32, 18, spp=2, seed=4).wait(),
                          R.render(sc, cam, 32, 18, spp=2, seed=4))
