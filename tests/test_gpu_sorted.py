"""Direction-coherent waves (diagnostic variants 20 / 21, trace.hip's sorted_kernel;
measured slower than the default, profiles/r04/sorted_waves/):
512-thread workgroups whose 8 waves advance in lock step and deal the
workgroup's paths to the waves by key before every ray-color level (20:
fresh samples, then the 8 direction octants; 21: live paths packed only).
The paths move between lanes through LDS, but each is computed with the same
fp32 ops, and the pixel sums are integers: every frame must equal the
oracle's fp32 mirror (MODE_MIRROR32 | DIRECT) bit for bit, with the same segment
count -- whole tiles, sample splits, interleaved shards, realm semantics,
ragged tiles, depth 1 and the recorded tile order.
"""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


def _mirror(sc, cam, w, h, spp, depth, seed, realm=False, rows=None):
    mode = (oracle.MODE_REALM32 if realm else oracle.MODE_MIRROR32) | oracle.DIRECT   # the kernel's default samplers
    out, _, segs, _ = oracle.render(mode, sc.sphere.astype(np.float64), sc.kind, sc.mat.astype(np.float64),
                                    cam.as_list(), cam.defocus, w, h, spp, depth, seed=seed, rows=rows)
    return out, segs


@pytest.fixture(params=[20, 21])
def sorted_variant(request, gpu_lib):
    """The diagnostic build (lib/librtclj_diag.so: the sorted kernels were
    measured slower than the default and are not in the product library,
    profiles/r04/sorted_waves/) with variant 20 or 21 selected."""
    from rtclj._lib import diag_lib
    dll = diag_lib()
    old = dll.rt_set_variant(request.param)
    assert old >= 0, dll.rt_last_error()
    yield dll
    dll.rt_set_variant(old)


@pytest.mark.parametrize("w,h,spp,depth", [(72, 40, 7, 50), (200, 112, 16, 50), (33, 17, 3, 50), (9, 10, 100, 50),
                                           (64, 36, 5, 1), (40, 24, 64, 3)])
def test_sorted_cover_frames_bit_exact(sorted_variant, w, h, spp, depth):
    """Frames of few tiles (sample splits), of many (whole tiles), ragged in
    both directions, depth 1 and 3; each rendered twice (the second launch
    in the recorded tile order)."""
    from rtclj import raytracing as R, scenes
    sc = scenes.cover(11)
    cam = scenes.cover_camera(w, h)
    ref, segs = _mirror(sc, cam, w, h, spp, depth, 4)
    for k in range(2):
        st = {}
        g = R.render(sc, cam, w, h, spp=spp, max_depth=depth, seed=4, stats=st, library=sorted_variant)
        assert np.array_equal(g, ref), (w, h, spp, depth, k)
        assert st["segments"] == segs


def test_sorted_reference_scene_realm_and_shards(sorted_variant):
    """The reference's five bodies under -main and realm semantics, and the
    8-shard interleaved fan-out (RT_FLAG_SHARDS_ON_DEVICE0) bit-identical."""
    from rtclj import raytracing as R
    from rtclj._lib import RT_FLAG_REALM, RT_FLAG_SHARDS_ON_DEVICE0
    sc = R.Scene.from_bodies(R.hittables)
    w, h = 160, 90
    cam = R.camera(w, h, **R.REFERENCE_CAMERA)
    ref, _ = _mirror(sc, cam, w, h, 16, 50, 2)
    dll = sorted_variant
    assert np.array_equal(R.render(sc, cam, w, h, spp=16, seed=2, library=dll), ref)
    rr, _ = _mirror(sc, cam, w, h, 8, 50, 2, realm=True)
    assert np.array_equal(R.render(sc, cam, w, h, spp=8, seed=2, flags=RT_FLAG_REALM, library=dll), rr)
    sh = R.render(sc, cam, w, h, spp=16, seed=2, n_devices=8, flags=RT_FLAG_SHARDS_ON_DEVICE0, library=dll)
    assert np.array_equal(sh, ref)


def test_sorted_deep_paths_fall_back(gpu_lib):
    """A path's depth left travels in 10 bits: max_depth > 1023 runs the
    default traversal (same bits)."""
    from rtclj import raytracing as R, scenes
    from rtclj._lib import diag_lib
    dll = diag_lib()
    sc = scenes.cover(11)
    w, h = 24, 16
    cam = scenes.cover_camera(w, h)
    ref, _ = _mirror(sc, cam, w, h, 2, 1500, 3)
    old = dll.rt_set_variant(20)
    try:
        assert np.array_equal(R.render(sc, cam, w, h, spp=2, max_depth=1500, seed=3, library=dll), ref)
    finally:
        dll.rt_set_variant(old)


def test_sorted_c1_rows(sorted_variant):
    """C1 at full size and spp (1200 x 675 x 100): rows across the frame
    (sky, field, the r = 1 bodies, the ground) equal the mirror."""
    from rtclj import raytracing as R, scenes
    sc = scenes.cover(11)
    w, h = 1200, 675
    cam = scenes.cover_camera(w, h)
    g = R.render(sc, cam, w, h, spp=100, seed=1, library=sorted_variant)
    for r in (40, 196, 300, 470, 640):
        ref, _ = _mirror(sc, cam, w, h, 100, 50, 1, rows=(r, r + 1))
        assert np.array_equal(g[r], ref[0]), r
