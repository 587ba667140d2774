"""BASELINE.json's configurations at their own sizes on the GPU, and the
fp64 reference-semantics pin of the benchmark workload.

The kernel's default draws vec3a's two samplers loop-free (the same
distributions, a fixed number of uniforms; include/rt.h
RT_FLAG_REJECTION_SAMPLERS), so its paths after the first scatter are
independent of MODE_REF64's, which draws by the reference's rejection loops:
against REF64 the default is held to oracle/pin.py's BOUNDS_INDEPENDENT (SURVEY.md §8c's
bounds for a render against the reference's own unseeded one), and the
kernel with RT_FLAG_REJECTION_SAMPLERS -- the same draws as REF64 -- to the
same-draw BOUNDS.  Bit-exact checks compare each with its own fp32 mirror
(MODE_MIRROR32 | DIRECT, MODE_MIRROR32).

  C1 cover 1200x675, 100 spp, depth 50: the kernel's frame against the
     oracle's MODE_REF64 (the Clojure path in double) on every 8th row at
     full spp, and the segments per sample within 2e-3 of REF64's, with
     either samplers;
  C2 3840x2160, 500 spp (484 bodies): the whole frame, deterministic,
     finite, in range, sixteen rows spread over the frame (sky, the field,
     the near ground) and two through the r = 1 glass body bit-exact
     against the fp32 mirror at full spp;
  C3 3840x2160, 1000 spp, row tiles over 8 GPUs + host gather: rt_render's
     8-way fan-out (RT_FLAG_SHARDS_ON_DEVICE0 puts the 8 shards on this box's
     one GPU) bit-identical to the 1-shard frame, and two whole rows and two
     64-pixel strips of the gathered frame (four shards) bit-exact against the
     fp32 mirror at full spp;
  C4 7680x4320, 2000 spp, depth 64, 1000 bodies: the whole frame's
     properties, a row band re-rendered alone equal to the frame's rows, and
     eight 64-pixel strips bit-exact against the mirror at full spp; and C4's own
     kernel (variant 26: the compact 4-body image, u8 stack, 1024-thread
     workgroups, two per CU) against MODE_REF64 on every 270th row: with the
     rejection samplers at 16 and 64 spp (the same-draw bounds), with the
     default samplers at 64 spp (the independent-draw bounds).

Every full frame's segments per sample (one hit-anything call each,
raytracing.clj:48) must match the fp64 reference-semantics value of its
config's scene, camera and depth (tests/golden/segs_ref64.json, from
tests/golden/make_segs.py: MODE_REF64 over every row, ~1e-4 relative
standard error) within oracle/pin.py's 2e-3: a systematic shift of the
shading or the traversal fails there, not only in the images.

The scene cache of rt_render (include/rt.h) is checked here too: a repeat
call hits it, a changed body misses it, and neither changes a bit.
"""
import json
import os
from pathlib import Path

import numpy as np
import pytest

import oracle
from oracle.pin import BOUNDS, BOUNDS_INDEPENDENT, compare, within

pytestmark = pytest.mark.gpu

NT = min(16, os.cpu_count() or 1)   # the GPU box's CPU share
# the fp32 mirror of the kernel's default contract (loop-free samplers)
KERNEL32 = oracle.MODE_MIRROR32 | oracle.DIRECT
SEGS = json.loads((Path(__file__).resolve().parent / "golden" / "segs_ref64.json").read_text())["configs"]


def _oracle(mode, sc, cam, w, h, spp, depth, rows=None, row_step=1, cols=None):
    out, _, segs, smp = oracle.render(mode, sc.sphere.astype(np.float64), sc.kind, sc.mat.astype(np.float64),
                                      cam.as_list(), cam.defocus, w, h, spp, depth, seed=1, rows=rows,
                                      row_step=row_step, nthreads=NT, cols=cols)
    return out, segs, smp


def _props(img, st, config):
    """Finite, in [0, 1], and segments per sample within 2e-3 (relative) of
    the config's fp64 reference-semantics value."""
    assert np.isfinite(img).all() and img.min() >= 0.0 and img.max() <= 1.0 + 1e-6
    ref = SEGS[config]["segments_per_sample"]
    got = st["segments"] / st["samples"]
    assert abs(got - ref) / ref <= BOUNDS["seg_rel"], (config, got, ref)


def _launch_rows(sc, cam, w, h, spp, depth, row_tile, tile_first, tile_step, flags=0):
    """rt_launch of an interleaved row selection on a fresh device scene ->
    (rows array, segments, samples)."""
    import ctypes as C
    import torch
    from rtclj._lib import check, lib, rt_params
    p = rt_params(width=w, height=h, row_begin=0, row_end=h, spp=spp, max_depth=depth, seed=1,
                  row_tile=row_tile, tile_first=tile_first, tile_step=tile_step, flags=flags)
    n = check(lib.rt_rows_out(C.byref(p)))
    ds = C.c_void_p()
    check(lib.rt_scene_upload(0, C.byref(sc.c), C.byref(ds)))
    try:
        out = torch.full((n * w * 3,), float("nan"), dtype=torch.float32, device="cuda")
        cnt = torch.zeros(2, dtype=torch.int64, device="cuda")
        s = torch.cuda.current_stream()
        check(lib.rt_launch(ds, C.byref(cam), C.byref(p), C.c_void_p(out.data_ptr()), C.c_void_p(cnt.data_ptr()),
                            C.c_void_p(s.cuda_stream)))
        torch.cuda.synchronize()
    finally:
        lib.rt_scene_free(ds)
    c = cnt.cpu().tolist()
    return out.cpu().numpy().reshape(n, w, 3), c[0], c[1]


_C1_REF64 = {}


@pytest.mark.parametrize("samplers", ["direct", "rejection"])
def test_c1_against_fp64_reference_semantics(gpu_lib, samplers):
    from rtclj import raytracing as R
    from rtclj import scenes
    from rtclj._lib import RT_FLAG_REJECTION_SAMPLERS
    flags = RT_FLAG_REJECTION_SAMPLERS if samplers == "rejection" else 0
    sc = scenes.cover(11)
    w, h, spp = 1200, 675, 100
    cam = scenes.cover_camera(w, h)
    st = {}
    g = R.render(sc, cam, w, h, spp=spp, max_depth=50, seed=1, stats=st, flags=flags)
    _props(g, st, "c1")
    # every 8th row on its own (1-row tiles, stride 8): the frame's rows, and
    # the segment count of exactly those rows
    rows, segs32, smp32 = _launch_rows(sc, cam, w, h, spp, 50, row_tile=1, tile_first=0, tile_step=8, flags=flags)
    assert np.array_equal(rows, g[::8])
    if not _C1_REF64:
        _C1_REF64["r"] = _oracle(oracle.MODE_REF64, sc, cam, w, h, spp, 50, row_step=8)
    ref, segs, smp = _C1_REF64["r"]
    assert ref.shape == (85, w, 3) and smp == smp32
    s = compare(ref, segs / smp, rows, segs32 / smp32, by=4)
    ok = within(s, BOUNDS_INDEPENDENT if samplers == "direct" else BOUNDS)
    assert all(ok.values()), (ok, s)


def test_c2_full_frame(gpu_lib):
    from rtclj import raytracing as R
    from rtclj import scenes
    sc = scenes.cover(11)
    w, h, spp = 3840, 2160, 500
    cam = scenes.cover_camera(w, h)
    st, st2 = {}, {}
    a = R.render(sc, cam, w, h, spp=spp, max_depth=50, seed=1, stats=st)
    b = R.render(sc, cam, w, h, spp=spp, max_depth=50, seed=1, stats=st2)
    assert np.array_equal(a, b)
    assert st["samples"] == w * h * spp and st2["scene_cached"] == 1
    _props(a, st, "c2")
    # rows 180, 540, ..., 1980: sky, the field, the r = 1 bodies, the ground
    ref, segs, smp = _oracle(KERNEL32, sc, cam, w, h, spp, 50, rows=(180, h), row_step=360)
    assert ref.shape[0] == 6
    bad = [r for k, r in enumerate(range(180, h, 360)) if not np.array_equal(a[r], ref[k])]
    # ten more: the sky's top row, the horizon band, the field's middle
    # distance and the near ground down to the last row
    for r in (0, 90, 700, 860, 1010, 1230, 1440, 1660, 1880, 2159):
        g, _, _ = _oracle(KERNEL32, sc, cam, w, h, spp, 50, rows=(r, r + 1))
        if not np.array_equal(a[r], g[0]):
            bad.append(r)
    # and two rows through the r = 1 glass body at (0, 1, 0) (it spans rows
    # ~161-1080 around column 1920; row 626 is its centre): refraction, total
    # internal reflection and Schlick draws over a wide run of pixels
    for r in (400, 626):
        g, _, _ = _oracle(KERNEL32, sc, cam, w, h, spp, 50, rows=(r, r + 1))
        if not np.array_equal(a[r], g[0]):
            bad.append(r)
    assert not bad, bad


def test_c3_eight_shard_fan_out(gpu_lib):
    from rtclj import raytracing as R
    from rtclj import scenes
    from rtclj._lib import RT_FLAG_SHARDS_ON_DEVICE0
    sc = scenes.cover(11)
    w, h, spp = 3840, 2160, 1000
    cam = scenes.cover_camera(w, h)
    st1, st8 = {}, {}
    one = R.render(sc, cam, w, h, spp=spp, max_depth=50, seed=1, n_devices=1, stats=st1)
    eight = R.render(sc, cam, w, h, spp=spp, max_depth=50, seed=1, n_devices=8,
                     flags=RT_FLAG_SHARDS_ON_DEVICE0, stats=st8)
    assert st8["n_devices"] == 8
    assert np.array_equal(one, eight)
    assert st1["samples"] == st8["samples"] == w * h * spp and st1["segments"] == st8["segments"]
    _props(one, st1, "c2")   # C3 renders C2's scene, camera and depth
    # the gathered frame directly against the fp32 mirror at its full 1000
    # spp: two whole rows from different shards (8-row tiles: rows 626 and
    # 1507 are tiles 78 and 188, shards 6 and 4) -- the r = 1 glass body's
    # centre row and the near field -- and 64-pixel strips of shards 0 and 7
    bad = []
    for r, c0, c1 in ((626, 0, w), (1507, 0, w), (3, 1900, 1964), (2159, 3776, 3840)):
        ref, _, _ = _oracle(KERNEL32, sc, cam, w, h, spp, 50, rows=(r, r + 1), cols=(c0, c1))
        if not np.array_equal(eight[r, c0:c1], ref[0, c0:c1]):
            bad.append((r, c0))
    assert not bad, bad


def test_c4_full_frame(gpu_lib):
    from rtclj import raytracing as R
    from rtclj import scenes
    sc = scenes.cover_c4()
    assert len(sc) == 1000
    w, h, spp, depth = 7680, 4320, 2000, 64
    cam = scenes.cover_camera(w, h)
    st = {}
    img = R.render(sc, cam, w, h, spp=spp, max_depth=depth, seed=1, stats=st)
    assert img.shape == (h, w, 3) and st["samples"] == w * h * spp
    _props(img, st, "c4")
    # a band rendered alone (row_begin offset, other tiling) == the frame's rows
    band = R.render(sc, cam, w, h, spp=spp, max_depth=depth, seed=1, rows=(2100, 2116))
    assert np.array_equal(band, img[2100:2116])
    # eight 64-pixel strips spread over the frame, full spp, against the fp32
    # mirror: the r = 1 glass (centre row 1252, column 3840), lambertian
    # (1043, 3199) and metal (1629, 5001) bodies, sky, the field, the near
    # ground and the frame's last row and columns
    bad = []
    for r, c0 in ((1252, 3808), (1043, 3168), (1629, 4970), (200, 6000), (2600, 2500), (2200, 5800),
                  (3800, 1000), (4319, 7616)):
        ref, _, _ = _oracle(KERNEL32, sc, cam, w, h, spp, depth, rows=(r, r + 1), cols=(c0, c0 + 64))
        if not np.array_equal(img[r, c0:c0 + 64], ref[0, c0:c0 + 64]):
            bad.append((r, c0))
    assert not bad, bad


def test_c4_against_fp64_reference_semantics(gpu_lib):
    """C4's kernel instantiation -- 1000 bodies, depth 64, variant 26 (the
    compact 4-body image, u8 stack, 1024-thread workgroups on 8x8-pixel
    pools), the r = 1000 ground's self-hit guard at depth 64 -- against the
    Clojure path in double (hittable.clj:10-23, raytracing.clj:45-58):
      * with RT_FLAG_REJECTION_SAMPLERS (REF64's own draws) on rows 0, 270,
        ..., 4050 of the 7680x4320 frame at 16 and at 64 spp, with the
        same-draw bounds;
      * with the default loop-free samplers on the same rows at 64 spp, with
        the independent-draw bounds (measured on the CPU mirror: block means
        mean |d| 0.058, max 0.33 in 2 x 16 blocks; per-pixel 2.8);
    (spp reduced from 2000 so that MODE_REF64's linear scan over 1000 bodies
    finishes in seconds; the kernel's arithmetic does not depend on spp;
    oracle/pin.py)."""
    import ctypes as C
    from rtclj import scenes
    from rtclj._lib import RT_FLAG_REJECTION_SAMPLERS, check, lib
    sc = scenes.cover_c4()
    w, h, spp, depth = 7680, 4320, 16, 64
    cam = scenes.cover_camera(w, h)
    ds = C.c_void_p()
    check(lib.rt_scene_upload(0, C.byref(sc.c), C.byref(ds)))
    try:
        # the scene resolves to the 8-body-leaf tree; its launches run the
        # 4-body compact image in 16-wave workgroups (variant 26), two per CU
        assert lib.rt_resolve_variant(ds) == 18
        from rtclj._lib import rt_params
        p = rt_params(width=w, height=h, row_begin=0, row_end=h, spp=2000, max_depth=depth, seed=1)
        o = (C.c_int * 4)()
        check(lib.rt_launch_occupancy(ds, C.byref(p), o))
        assert o[3] == 26 and o[0] * 256 // 1024 == 2, list(o)
    finally:
        lib.rt_scene_free(ds)
    fails, refs = [], {}
    for samplers, spp, step, by in (("rejection", 16, 270, 4), ("rejection", 64, 270, 4), ("direct", 64, 270, 2)):
        flags = RT_FLAG_REJECTION_SAMPLERS if samplers == "rejection" else 0
        rows, segs32, smp32 = _launch_rows(sc, cam, w, h, spp, depth, row_tile=1, tile_first=0, tile_step=step,
                                           flags=flags)
        if (spp, step) not in refs:
            refs[spp, step] = _oracle(oracle.MODE_REF64, sc, cam, w, h, spp, depth, row_step=step)
        ref, segs, smp = refs[spp, step]
        n = (h + step - 1) // step
        assert ref.shape == rows.shape == (n, w, 3) and smp == smp32 == n * w * spp
        s = compare(ref, segs / smp, rows, segs32 / smp32, by=by)
        ok = within(s, BOUNDS if samplers == "rejection" else BOUNDS_INDEPENDENT)
        if not all(ok.values()):
            fails.append((samplers, spp, ok, s))
    assert not fails, fails


def test_scene_cache_hits_and_invalidates(gpu_lib):
    from rtclj import raytracing as R
    from rtclj import scenes
    from rtclj._lib import lib
    lib.rt_cache_clear()
    sc = scenes.cover(11)
    w, h = 200, 112
    cam = scenes.cover_camera(w, h)
    s1, s2, s3, s4 = {}, {}, {}, {}
    a = R.render(sc, cam, w, h, spp=8, seed=2, stats=s1)
    b = R.render(sc, cam, w, h, spp=8, seed=2, stats=s2)
    assert s1["scene_cached"] == 0 and s2["scene_cached"] == 1 and np.array_equal(a, b)
    # a changed body (same count) misses the cache and renders its own scene
    sph = sc.sphere.copy()
    sph[-1, 1] += 0.25                     # lift the r = 1 metal body
    moved = R.Scene(sph, sc.kind, sc.mat)
    c = R.render(moved, cam, w, h, spp=8, seed=2, stats=s3)
    assert s3["scene_cached"] == 0 and not np.array_equal(a, c)
    ref_c, _, _, _ = oracle.render(KERNEL32, moved.sphere.astype(np.float64), moved.kind,
                                   moved.mat.astype(np.float64), cam.as_list(), cam.defocus, w, h, 8, 50, seed=2,
                                   nthreads=NT)
    assert np.array_equal(c, ref_c)
    # a material change alone misses too
    mat = sc.mat.copy()
    mat[0, :3] = (0.7, 0.1, 0.1)
    d = R.render(R.Scene(sc.sphere, sc.kind, mat), cam, w, h, spp=8, seed=2, stats=s4)
    assert s4["scene_cached"] == 0 and not np.array_equal(a, d)
    # the original is still cached (LRU of 4) and still renders the same bits
    e = R.render(sc, cam, w, h, spp=8, seed=2, stats=s1)
    assert s1["scene_cached"] == 1 and np.array_equal(a, e)
    assert lib.rt_cache_clear() == 3
