"""The adaptive tile schedule (rt_set_schedule, include/rt.h): rt_launch on a
persistent scene dispatches tiles longest first by the previous launch's
durations.  The order must be a permutation of the launch's tiles and never
change a bit of the output: every launch here writes into a NaN-filled buffer
(a tile skipped or run twice would leave NaNs or be caught by the equality)
and is compared with rt_render of the same frame (fresh scene: plain order),
itself pinned to the oracle by test_gpu_parity.py.
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env(gpu_lib):
    import torch
    from rtclj import scenes
    from rtclj._lib import check, lib
    sc = scenes.cover(11)
    ds = C.c_void_p()
    check(lib.rt_scene_upload(0, C.byref(sc.c), C.byref(ds)))
    yield sc, ds, torch
    lib.rt_scene_free(ds)


def _launch(env, cam, w, h, spp, stream=None, seed=1, rows=None, row_tile=0, tile_first=0, tile_step=0,
            sample_begin=0, dll=None, ds=None):
    sc, ds0, torch = env
    from rtclj._lib import check, lib, rt_params
    ds = ds if ds is not None else ds0
    dll = dll if dll is not None else lib
    r0, r1 = rows or (0, h)
    p = rt_params(width=w, height=h, row_begin=r0, row_end=r1, spp=spp, max_depth=50, seed=seed,
                  sample_begin=sample_begin, row_tile=row_tile, tile_first=tile_first, tile_step=tile_step)
    n = check(lib.rt_rows_out(C.byref(p)))
    s = stream or torch.cuda.current_stream()
    with torch.cuda.stream(s):
        out = torch.full((n * w * 3,), float("nan"), dtype=torch.float32, device="cuda")
    s.synchronize()
    rc = dll.rt_launch(ds, C.byref(cam), C.byref(p), C.c_void_p(out.data_ptr()), None, C.c_void_p(s.cuda_stream))
    assert rc == 0, dll.rt_last_error()
    s.synchronize()
    return out.cpu().numpy().reshape(n, w, 3)


def _render(sc, cam, w, h, spp, **kw):
    from rtclj import raytracing as R
    return R.render(sc, cam, w, h, spp=spp, max_depth=50, **kw)


@pytest.mark.parametrize("v", [0, 5, 12, 16, 18, 11, 22, 24, 26])
def test_repeated_launches_are_bit_identical(env, v):
    from rtclj import scenes
    from rtclj._lib import diag_lib, lib
    sc = env[0]
    w, h, spp = 333, 187, 6                       # ragged tiles at both edges
    cam = scenes.cover_camera(w, h)
    want = _render(sc, cam, w, h, spp)
    dll = lib if v in (0, 5, 12, 16, 18, 24, 26) else diag_lib()
    ds = env[1]
    if dll is not lib:                            # the diagnostic build's own device scene
        ds = C.c_void_p()
        from rtclj._lib import check
        check(dll.rt_scene_upload(0, C.byref(sc.c), C.byref(ds)))
    old = dll.rt_set_variant(v)
    try:
        for k in range(4):                        # launch 0 plain, then scheduled by the previous launch
            got = _launch(env, cam, w, h, spp, dll=dll, ds=ds)
            assert not np.isnan(got).any(), k
            assert np.array_equal(got, want), k
    finally:
        dll.rt_set_variant(old)
        if dll is not lib:
            dll.rt_scene_free(ds)


def test_schedule_off_matches_on(env):
    from rtclj import scenes
    from rtclj._lib import lib
    w, h, spp = 256, 144, 8
    cam = scenes.cover_camera(w, h)
    on = [_launch(env, cam, w, h, spp) for _ in range(2)]
    old = lib.rt_set_schedule(1)
    try:
        off = _launch(env, cam, w, h, spp)
    finally:
        lib.rt_set_schedule(old)
    assert np.array_equal(on[0], off) and np.array_equal(on[1], off)


def test_same_shape_other_camera_seed_and_samples(env):
    """The order recorded for one frame is reused by the next launch of the
    same shape with another camera, seed and sample range: still exact."""
    from rtclj import raytracing as R
    from rtclj import scenes
    sc = env[0]
    w, h = 200, 112
    cam_a = scenes.cover_camera(w, h)
    cam_b = R.camera(w, h, 30.0, (10.0, 3.0, -4.0), (0.0, 0.5, 0.0), (0.0, 1.0, 0.0), 0.0, 10.0)
    _launch(env, cam_a, w, h, 4)
    got = _launch(env, cam_b, w, h, 5, seed=7)
    assert np.array_equal(got, _render(sc, cam_b, w, h, 5, seed=7))
    got = _launch(env, cam_b, w, h, 4, seed=7, sample_begin=4)
    assert np.array_equal(got, _render(sc, cam_b, w, h, 4, seed=7, sample_begin=4))


def test_shape_changes_and_row_shards(env):
    """Alternating shapes re-key the record; interleaved row-tile shards (the
    multi-GPU split) keep their own tile count."""
    from rtclj import scenes
    sc = env[0]
    for w, h in ((160, 90), (96, 54), (160, 90), (1, 1), (160, 90)):
        cam = scenes.cover_camera(w, h)
        assert np.array_equal(_launch(env, cam, w, h, 3), _render(sc, cam, w, h, 3)), (w, h)
    w, h = 180, 101
    cam = scenes.cover_camera(w, h)
    full = _render(sc, cam, w, h, 4)
    for _ in range(2):
        parts = [_launch(env, cam, w, h, 4, row_tile=8, tile_first=f, tile_step=3) for f in range(3)]
        for f, part in enumerate(parts):
            rows = np.concatenate([np.arange(t, min(t + 8, h)) for t in range(8 * f, h, 24)])
            assert np.array_equal(part, full[rows]), f


def test_streams_keep_separate_records(env):
    """Two streams launching the same scene concurrently: each has its own
    record, and more streams than the record holds run unscheduled."""
    from rtclj import scenes
    torch = env[2]
    sc = env[0]
    w, h = 240, 135
    cam = scenes.cover_camera(w, h)
    want = _render(sc, cam, w, h, 4)
    streams = [torch.cuda.Stream() for _ in range(10)]
    for _ in range(2):
        for s in streams:
            assert np.array_equal(_launch(env, cam, w, h, 4, stream=s), want)
    # concurrent: enqueue on both streams before synchronising either
    from rtclj._lib import check, lib, rt_params
    _, ds, _ = env
    p = rt_params(width=w, height=h, row_begin=0, row_end=h, spp=4, max_depth=50, seed=1)
    outs = []
    for s in streams[:2]:
        with torch.cuda.stream(s):
            o = torch.full((h * w * 3,), float("nan"), dtype=torch.float32, device="cuda")
        outs.append(o)
    torch.cuda.synchronize()
    for _ in range(3):
        for s, o in zip(streams[:2], outs):
            check(lib.rt_launch(ds, C.byref(cam), C.byref(p), C.c_void_p(o.data_ptr()), None,
                                C.c_void_p(s.cuda_stream)))
    torch.cuda.synchronize()
    for o in outs:
        assert np.array_equal(o.cpu().numpy().reshape(h, w, 3), want)


@pytest.mark.parametrize("spp", [1, 3, 9, 8191, 8193])
def test_large_and_small_spp_launches(env, spp):
    """One launch per frame at any spp (the fixed-point sums need no rounds):
    rt_launch on a persistent scene == rt_render, at spp around the
    multiply-high / integer-division switch of the pool index."""
    from rtclj import scenes
    sc = env[0]
    w, h = (150, 77) if spp < 100 else (10, 9)
    cam = scenes.cover_camera(w, h)
    want = _render(sc, cam, w, h, spp)
    for _ in range(2):
        got = _launch(env, cam, w, h, spp)
        assert not np.isnan(got).any()
        assert np.array_equal(got, want)


@pytest.fixture
def split_env(monkeypatch):
    """RTCLJ_SPLIT forces rt_launch's sample split (read at every launch)."""
    def set_split(k):
        if k is None:
            monkeypatch.delenv("RTCLJ_SPLIT", raising=False)
        else:
            monkeypatch.setenv("RTCLJ_SPLIT", str(k))
    yield set_split
    monkeypatch.delenv("RTCLJ_SPLIT", raising=False)


@pytest.mark.parametrize("spp", [1, 2, 7, 37, 100, 8193])
def test_sample_split_is_bit_exact(env, split_env, spp):
    """Every split of the tiles' samples over workgroups (contiguous sample
    ranges, integer pixel sums added by finalize_kernel) gives the unsplit
    frame's bits, including splits > spp (clamped), spp = 1 and per-split
    counts on both sides of the multiply-high limit."""
    from rtclj import scenes
    sc = env[0]
    w, h = (90, 53) if spp < 1000 else (9, 8)
    cam = scenes.cover_camera(w, h)
    split_env(1)
    want = _launch(env, cam, w, h, spp)
    assert not np.isnan(want).any()
    for k in (2, 3, 5, 64, 1000):
        split_env(k)
        for _ in range(2):   # the second launch runs the adaptive order of the split units
            got = _launch(env, cam, w, h, spp)
            assert np.array_equal(got, want), (spp, k)
    split_env(None)          # the automatic choice (a small frame: split)
    assert np.array_equal(_launch(env, cam, w, h, spp), want)
    assert np.array_equal(_render(sc, cam, w, h, spp), want)


def test_sample_split_shards_realm_and_stripes(env, split_env):
    """Split launches of interleaved row-tile shards, of a sample stripe
    (sample_begin) and of realm semantics: the unsplit bits."""
    from rtclj import scenes
    from rtclj._lib import RT_FLAG_REALM
    sc = env[0]
    w, h = 120, 67
    cam = scenes.cover_camera(w, h)
    split_env(1)
    full = _render(sc, cam, w, h, 12)
    stripe = _launch(env, cam, w, h, 5, sample_begin=7)
    realm = _render(sc, cam, w, h, 6, flags=RT_FLAG_REALM)
    for k in (4, 12):
        split_env(k)
        for f in range(3):
            part = _launch(env, cam, w, h, 12, row_tile=8, tile_first=f, tile_step=3)
            rows = np.concatenate([np.arange(t, min(t + 8, h)) for t in range(8 * f, h, 24)])
            assert np.array_equal(part, full[rows]), (k, f)
        assert np.array_equal(_launch(env, cam, w, h, 5, sample_begin=7), stripe), k
        assert np.array_equal(_render(sc, cam, w, h, 6, flags=RT_FLAG_REALM), realm), k


def test_streamed_frames_in_flight_are_bit_exact(env):
    """RT_FLAG_STREAMED (include/rt.h): C1's 8-GPU shard and 4-GPU shard
    launched as frames in flight -- round-robin over two streams, each stream
    its own output buffer, tile-order record and split sums, never
    synchronised in between -- equal rt_render's rows of the same frame, every
    frame.  The flag changes the sample split (two rounds of workgroups, at
    least 2 splits), never a bit."""
    from rtclj import scenes
    from rtclj._lib import RT_FLAG_STREAMED, check, lib, rt_params
    from rtclj.shard import shard_params, shard_rows
    sc, ds, torch = env
    w, h, spp = 1200, 675, 24
    cam = scenes.cover_camera(w, h)
    full = _render(sc, cam, w, h, spp)
    for world in (8, 4):
        rank = world - 1
        p = rt_params(**shard_params(world, rank, w, h, spp, 50, 1, "strong"))
        p.flags |= RT_FLAG_STREAMED
        n = check(lib.rt_rows_out(C.byref(p)))
        streams = [torch.cuda.Stream() for _ in range(2)]
        frames = []
        for f in range(6):
            s = streams[f % 2]
            with torch.cuda.stream(s):
                out = torch.full((n * w * 3,), float("nan"), dtype=torch.float32, device="cuda")
            rc = lib.rt_launch(ds, C.byref(cam), C.byref(p), C.c_void_p(out.data_ptr()), None,
                               C.c_void_p(s.cuda_stream))
            assert rc == 0, lib.rt_last_error()
            frames.append(out)
        torch.cuda.synchronize()
        want = full[shard_rows(h, 8, rank, world)]
        for f, out in enumerate(frames):
            got = out.cpu().numpy().reshape(n, w, 3)
            assert np.array_equal(got, want), (world, f)
    # rt_render is one frame per call: the flag is rt_launch's only
    from rtclj import raytracing as R
    from rtclj._lib import RTError
    with pytest.raises(RTError):
        R.render(sc, cam, 64, 36, spp=2, flags=RT_FLAG_STREAMED)



def test_cost_balanced_splits_are_bit_exact(env, split_env, monkeypatch):
    """Split launches in the recorded order run the units the previous
    launch's plan_kernel dealt by tile cost (a heavy tile gets more, shorter
    sample ranges; units the clamps leave over exit): the unsplit bits, with
    the plan on and off (RTCLJ_SPLIT_PLAN=0), across spp changes that keep
    the unit count (a plan made for spp 24 run at spp 7: some units empty)
    and that change it (the plan is then not used)."""
    from rtclj import scenes
    sc = env[0]
    w, h = 200, 112
    cam = scenes.cover_camera(w, h)
    split_env(1)
    want = {spp: _launch(env, cam, w, h, spp) for spp in (24, 7, 5)}
    for plan in ("1", "0"):
        monkeypatch.setenv("RTCLJ_SPLIT_PLAN", plan)
        split_env(4)
        for spp in (24, 24, 24, 7, 7, 24):
            got = _launch(env, cam, w, h, spp)
            assert np.array_equal(got, want[spp]), (plan, spp)
        split_env(8)
        for spp in (24, 24, 5, 24, 24):   # spp 5: 5 splits, another unit count
            got = _launch(env, cam, w, h, spp)
            assert np.array_equal(got, want[spp]), (plan, spp)
    monkeypatch.delenv("RTCLJ_SPLIT_PLAN")
