"""Tile sharing: the launch's last workgroups, dispatched
once every tile has been, join the tiles still running and claim batches of
their samples from the tile's shared counter until it is spent; a shared
tile's integer pixel sums meet in a per-tile buffer.  Integer sums do not
depend on who ran which sample, so every frame must equal the oracle's fp32
mirror (MODE_MIRROR32 | DIRECT) bit for bit, with helpers actually joining
(rt_steal_stats) -- by default, and with the knobs (RTCLJ_STEAL_MIN,
RTCLJ_THIEVES; read at every launch) at their extremes.
"""
import ctypes as C

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


def _mirror(sc, cam, w, h, spp, seed, rows=None):
    out, _, _, _ = oracle.render(oracle.MODE_MIRROR32 | oracle.DIRECT, sc.sphere.astype(np.float64), sc.kind,
                                 sc.mat.astype(np.float64), cam.as_list(), cam.defocus, w, h, spp, 50,
                                 seed=seed, rows=rows)
    return out


def _shard_rows(h, tile, first, step):
    return np.concatenate([np.arange(t, min(t + tile, h)) for t in range(tile * first, h, tile * step)])


@pytest.fixture(autouse=True)
def share_always(monkeypatch):
    """These frames have few tiles: rt_launch would split their samples
    instead of sharing them (RTCLJ_SPLIT=1 keeps every tile whole); and a
    launch in the recorded tile order shares only with
    RTCLJ_SHARE_RECORDED=1 (by default only plain-order launches do)."""
    monkeypatch.setenv("RTCLJ_SPLIT", "1")
    monkeypatch.setenv("RTCLJ_SHARE_RECORDED", "1")


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


def _launch(env, cam, p, stream):
    """rt_launch into a NaN-filled buffer; the frame and rt_steal_stats."""
    from rtclj._lib import check, lib
    sc, ds, torch = env
    n = check(lib.rt_rows_out(C.byref(p)))
    with torch.cuda.stream(stream):
        out = torch.full((n * p.width * 3,), float("nan"), dtype=torch.float32, device="cuda")
    stream.synchronize()
    check(lib.rt_launch(ds, C.byref(cam), C.byref(p), C.c_void_p(out.data_ptr()), None,
                        C.c_void_p(stream.cuda_stream)))
    st = (C.c_uint64 * 2)()
    check(lib.rt_steal_stats(ds, C.c_void_p(stream.cuda_stream), st))
    return out.cpu().numpy().reshape(n, p.width, 3), (int(st[0]), int(st[1]))


def test_default_steals_on_a_frame_of_few_tiles(env):
    """6 tiles x 600 spp on a device that holds ~1,500 workgroups: 6 owners,
    the helpers join them (claims of 128 in the first launch's plain order,
    up to 1,024 in the recorded order); every launch equals the mirror."""
    from rtclj import scenes
    from rtclj._lib import rt_params
    sc, ds, torch = env
    w, h, spp, seed = 24, 16, 600, 5
    cam = scenes.cover_camera(w, h)
    want = _mirror(sc, cam, w, h, spp, seed)
    s = torch.cuda.Stream()
    p = rt_params(width=w, height=h, row_begin=0, row_end=h, spp=spp, max_depth=50, seed=seed)
    for k in range(3):
        got, st = _launch(env, cam, p, s)
        assert np.array_equal(got, want), k
        assert st[0] > 0 and 0 < st[1] < w * h * spp, (k, st)


def test_recorded_order_does_not_share_by_default(env, monkeypatch):
    """By default only a launch without a tile-cost record (plain order)
    shares its tiles: the first launch of a shape has helpers joining, the
    next ones (recorded longest-first order) none -- every frame equal to
    the mirror."""
    from rtclj import scenes
    from rtclj._lib import rt_params
    sc, ds, torch = env
    monkeypatch.delenv("RTCLJ_SHARE_RECORDED")
    w, h, spp, seed = 24, 16, 600, 6
    cam = scenes.cover_camera(w, h)
    want = _mirror(sc, cam, w, h, spp, seed)
    s = torch.cuda.Stream()
    p = rt_params(width=w, height=h, row_begin=0, row_end=h, spp=spp, max_depth=50, seed=seed)
    steals = []
    for k in range(3):
        got, st = _launch(env, cam, p, s)
        assert np.array_equal(got, want), k
        steals.append(st[0])
    assert steals[0] > 0 and steals[1] == steals[2] == 0, steals


@pytest.mark.parametrize("knobs", [dict(RTCLJ_STEAL_MIN="1"), dict(RTCLJ_STEAL_MIN="100000"),
                                   dict(RTCLJ_BATCH_MAX="65536", RTCLJ_STEAL_MIN="1"),
                                   dict(RTCLJ_THIEVES="1"), dict(RTCLJ_THIEVES="16"), dict(RTCLJ_THIEVES="0")])
def test_forced_sharing_is_bit_exact(env, monkeypatch, knobs):
    """Helpers that join any tile with an unclaimed sample, helpers that
    join nothing, claims of up to 65,536 samples (an eighth of what is
    left), one / sixteen helpers per workgroup slot, and none (owners
    still claim batch by batch from the shared word): on a frame of few
    tiles, an interleaved row-tile shard and frames of tiny pools, every
    frame equals the mirror."""
    from rtclj import scenes
    from rtclj._lib import rt_params
    sc, ds, torch = env
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    s = torch.cuda.Stream()
    for w, h, spp, rt, tf, ts in ((40, 24, 300, 0, 0, 0), (200, 112, 40, 8, 1, 3), (33, 9, 1, 0, 0, 0),
                                  (17, 20, 7, 0, 0, 0)):
        cam = scenes.cover_camera(w, h)
        want = _mirror(sc, cam, w, h, spp, 3)
        if ts:
            want = want[_shard_rows(h, rt, tf, ts)]
        p = rt_params(width=w, height=h, row_begin=0, row_end=h, spp=spp, max_depth=50, seed=3,
                      row_tile=rt, tile_first=tf, tile_step=ts)
        steals = 0
        for k in range(2):   # plain order, then the recorded one
            got, st = _launch(env, cam, p, s)
            assert np.array_equal(got, want), (w, h, spp, k)
            steals += st[0]
        if spp >= 40 and knobs == dict(RTCLJ_STEAL_MIN="1"):   # (2 batches of 256 < every such pool)
            assert steals > 0, (w, h, spp)


def test_epoch_wrap_keeps_shared_tiles_exact(env, monkeypatch):
    """The 16-bit launch epoch of a stream's tile words wraps after 65,535
    sharing launches: rt_launch then re-zeroes the words and the owner table
    (trace.hip, the epoch's set-up), so no word left by a launch 65,535
    earlier looks current.  The stream's epoch starts at 65,528
    (RTCLJ_EPOCH_START) and 16 launches cross the wrap, alternating spp on
    one shape (the stale-owner race of a helper joining a tile published
    with another spp) and shapes, with helpers joining any tile: every frame
    equals the mirror, with no NaN (an unwritten tile)."""
    from rtclj import scenes
    from rtclj._lib import check, lib, rt_params
    sc, _, torch = env
    monkeypatch.setenv("RTCLJ_EPOCH_START", "65528")
    monkeypatch.setenv("RTCLJ_STEAL_MIN", "1")
    ds = C.c_void_p()   # a fresh scene: its stream entries start at the knob's epoch
    check(lib.rt_scene_upload(0, C.byref(sc.c), C.byref(ds)))
    try:
        s = torch.cuda.Stream()
        cases = [(24, 16, 600), (24, 16, 100), (24, 16, 300), (40, 24, 120)]
        want = {}
        for w, h, spp in cases:
            want[(w, h, spp)] = _mirror(sc, scenes.cover_camera(w, h), w, h, spp, 9)
        steals = 0
        for k in range(16):
            w, h, spp = cases[k % 3] if k % 5 != 4 else cases[3]
            cam = scenes.cover_camera(w, h)
            p = rt_params(width=w, height=h, row_begin=0, row_end=h, spp=spp, max_depth=50, seed=9)
            got, st = _launch((sc, ds, torch), cam, p, s)
            assert not np.isnan(got).any(), (k, w, h, spp)
            assert np.array_equal(got, want[(w, h, spp)]), (k, w, h, spp)
            steals += st[0]
        assert steals > 0
    finally:
        torch.cuda.synchronize()
        lib.rt_scene_free(ds)
