"""Drain compaction: once a wave's batches are spent, a
wave holding at most RTCLJ_COMPACT paths writes them (13 words each) into
its traversal stack's LDS and leaves; its sibling waves' free lanes take
them and run them to the end.  A path carries everything it needs (origin,
direction, throughput, RNG state, pool pixel, depth left, the body it
leaves) and the colour sums are integers, so every frame must equal the
oracle's fp32 mirror (MODE_MIRROR32 | DIRECT) bit for bit whoever finishes which
path -- at every threshold, with and without tile sharing and sample splits,
on pools smaller than a workgroup's 256 lanes (fewer waves start) and on
C4's 8-body-leaf traversal (u8 stack: smaller posts).
"""
import ctypes as C

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


def _mirror(sc, cam, w, h, spp, depth, seed):
    out, _, _, _ = oracle.render(oracle.MODE_MIRROR32 | oracle.DIRECT, sc.sphere.astype(np.float64), sc.kind,
                                 sc.mat.astype(np.float64), cam.as_list(), cam.defocus, w, h, spp, depth,
                                 seed=seed)
    return out


def _frame(gpu_lib, ds, cam, w, h, spp, depth, seed):
    import torch
    from rtclj._lib import check, lib, rt_params
    p = rt_params(width=w, height=h, row_begin=0, row_end=h, spp=spp, max_depth=depth, seed=seed)
    out = torch.full((h * w * 3,), float("nan"), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    check(lib.rt_launch(ds, C.byref(cam), C.byref(p), C.c_void_p(out.data_ptr()), None, None))
    torch.cuda.synchronize()
    return out.cpu().numpy().reshape(h, w, 3)


@pytest.fixture(scope="module")
def cover(gpu_lib):
    from rtclj import scenes
    from rtclj._lib import check, lib
    sc = scenes.cover(11)
    ds = C.c_void_p()
    check(lib.rt_scene_upload(0, C.byref(sc.c), C.byref(ds)))
    yield sc, ds
    lib.rt_scene_free(ds)


@pytest.mark.parametrize("knobs", [dict(RTCLJ_COMPACT="64"), dict(RTCLJ_COMPACT="16"), dict(RTCLJ_COMPACT="1"),
                                   dict(RTCLJ_COMPACT="5", RTCLJ_SPLIT="1"),
                                   dict(RTCLJ_COMPACT="16", RTCLJ_SPLIT="1", RTCLJ_STEAL_MIN="1", RTCLJ_SHARE_RECORDED="1"),
                                   dict(RTCLJ_COMPACT="16", RTCLJ_STEAL="0"),
                                   dict(RTCLJ_COMPACT="0"), dict(RTCLJ_TH4="2"), dict(RTCLJ_COMPACT="1", RTCLJ_TH4="2")])
def test_compaction_is_bit_exact(gpu_lib, cover, monkeypatch, knobs):
    """Thresholds 64 (clamped: posts as full as the stack slice holds, 22 on
    this scene's tree), 16, 1 and 5; tiles kept whole and shared
    (RTCLJ_SPLIT=1, helpers joining any tile), sharing off, compaction off;
    frames of many small pools, few large ones (sample splits by default) and
    pools of 1..255 samples: each launched twice (plain order, then the
    recorded one), every frame equal to the mirror.  These small frames run
    22 by default; RTCLJ_TH4=2 moves them to 28 (8 x 4-pixel pools)."""
    from rtclj import scenes
    sc, ds = cover
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    for w, h, spp, depth in ((96, 40, 24, 50), (24, 16, 500, 50), (33, 9, 3, 50), (17, 20, 1, 50),
                             (40, 24, 64, 3)):
        cam = scenes.cover_camera(w, h)
        want = _mirror(sc, cam, w, h, spp, depth, 9)
        for k in range(2):
            got = _frame(gpu_lib, ds, cam, w, h, spp, depth, 9)
            assert np.array_equal(got, want), (w, h, spp, depth, k)


@pytest.mark.parametrize("v", [18, 24, 26])
def test_compaction_on_the_eight_wave_traversals(gpu_lib, monkeypatch, v):
    """C4's 1000-body scene in 8- and 16-wave workgroups -- the 8-body-leaf
    tree with a u8 stack (half the room per post; the scene's resolved
    variant) and the 4-body compact image (24; 26, its default launch): a
    strip at depth 64 equals the mirror with compaction on (the default) and
    at threshold 3."""
    from rtclj import scenes
    from rtclj._lib import check, lib
    sc = scenes.cover_c4()
    ds = C.c_void_p()
    check(lib.rt_scene_upload(0, C.byref(sc.c), C.byref(ds)))
    old = lib.rt_set_variant(v)
    try:
        assert old >= 0
        w, h, spp, depth = 64, 16, 12, 64
        cam = scenes.cover_camera(w, h)
        want = _mirror(sc, cam, w, h, spp, depth, 4)
        for thr in (None, "3"):
            if thr:
                monkeypatch.setenv("RTCLJ_COMPACT", thr)
            got = _frame(gpu_lib, ds, cam, w, h, spp, depth, 4)
            assert np.array_equal(got, want), thr
    finally:
        lib.rt_set_variant(old)
        lib.rt_scene_free(ds)
