"""GPU parity: the HIP kernel (through the C ABI) vs the oracle.

The fp32 kernel follows an explicit arithmetic contract that
oracle/rt_oracle.cpp's MODE_MIRROR32 restates op for op, so the expected
result is bit-for-bit equality: with the kernel's default loop-free samplers
against MODE_MIRROR32 | DIRECT (KERNEL32), with RT_FLAG_REJECTION_SAMPLERS
(vec3a.clj:74-86's rejection loops) against MODE_MIRROR32.  The stated tolerance is the
floor the test enforces: >= 99.5 % of pixels within 1e-4 absolute per
channel and image-mean |diff| <= 1e-5; the bit-exact fraction is asserted
separately at >= 99.5 %.
"""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

TOL_ABS = 1e-4
TOL_FRAC = 0.995


PRODUCT_VARIANTS = (0, 5, 12, 16, 18, 22, 24, 26, 28)
# the fp32 mirrors of the kernel's default contract (loop-free samplers), main and realm semantics
KERNEL32 = oracle.MODE_MIRROR32 | oracle.DIRECT
KERNEL_REALM32 = oracle.MODE_REALM32 | oracle.DIRECT
SAMPLERS = ("direct", "rejection")


def _flags(samplers):
    from rtclj._lib import RT_FLAG_REJECTION_SAMPLERS
    return RT_FLAG_REJECTION_SAMPLERS if samplers == "rejection" else 0


def _mode(samplers, realm=False):
    """The oracle mode mirroring the kernel with these samplers."""
    base = oracle.MODE_REALM32 if realm else oracle.MODE_MIRROR32
    return base | (oracle.DIRECT if samplers == "direct" else 0)


class variant:
    """Select kernel variant v for the block: in the product library when it
    holds v, else in the diagnostic build.  `as` gives the library to pass to
    R.render(library=...)."""

    def __init__(self, v):
        from rtclj._lib import diag_lib, lib
        self.v = v
        self.lib = lib if v in PRODUCT_VARIANTS else diag_lib()

    def __enter__(self):
        self.old = self.lib.rt_set_variant(self.v)
        assert self.old >= 0, self.lib.rt_last_error()
        return self.lib

    def __exit__(self, *exc):
        self.lib.rt_set_variant(self.old)


def _ref_scene():
    from rtclj import raytracing as R
    return R.Scene.from_bodies(R.hittables)


def _mirror(scene, cam, w, h, spp, depth, seed=1, rows=None, sample_begin=0, mode=KERNEL32):
    out, _, segs, smp = oracle.render(mode, scene.sphere.astype(np.float64), scene.kind,
                                      scene.mat.astype(np.float64), cam.as_list(), cam.defocus, w, h, spp, depth,
                                      seed=seed, rows=rows, sample_begin=sample_begin)
    return out, segs, smp


def _assert_parity(gpu, ref, label):
    assert gpu.shape == ref.shape, label
    assert np.isfinite(gpu).all(), label
    d = np.abs(gpu.astype(np.float64) - ref.astype(np.float64))
    px_ok = (d.max(axis=-1) <= TOL_ABS).mean()
    exact = (gpu == ref).all(axis=-1).mean()
    assert px_ok >= TOL_FRAC, f"{label}: only {px_ok:.4%} pixels within {TOL_ABS}"
    assert d.mean() <= 1e-5, f"{label}: mean |diff| {d.mean():.3g}"
    assert exact >= TOL_FRAC, f"{label}: bit-exact pixels {exact:.4%}"
    return exact


@pytest.mark.parametrize("samplers", SAMPLERS)
def test_reference_scene_matches_mirror(gpu_lib, samplers):
    from rtclj import raytracing as R
    sc = _ref_scene()
    cam = R.camera(400, 225, **R.REFERENCE_CAMERA)
    st = {}
    gpu = R.render(sc, cam, 400, 225, spp=16, max_depth=50, seed=7, stats=st, flags=_flags(samplers))
    ref, segs, smp = _mirror(sc, cam, 400, 225, 16, 50, seed=7, mode=_mode(samplers))
    _assert_parity(gpu, ref, "reference scene 400x225x16")
    assert st["samples"] == smp == 400 * 225 * 16
    assert st["segments"] == segs, (st["segments"], segs)


@pytest.mark.parametrize("samplers", SAMPLERS)
def test_cover_scene_matches_mirror(gpu_lib, samplers):
    from rtclj import scenes
    from rtclj import raytracing as R
    sc = scenes.cover(11)
    cam = scenes.cover_camera(200, 112)
    st = {}
    gpu = R.render(sc, cam, 200, 112, spp=8, max_depth=50, seed=3, stats=st, flags=_flags(samplers))
    ref, segs, smp = _mirror(sc, cam, 200, 112, 8, 50, seed=3, mode=_mode(samplers))
    _assert_parity(gpu, ref, "cover 200x112x8")
    assert st["segments"] == segs


@pytest.mark.parametrize("w,h", [(37, 21), (1, 1), (64, 8), (17, 40)])
def test_ragged_sizes(gpu_lib, w, h):
    from rtclj import raytracing as R
    sc = _ref_scene()
    cam = R.camera(w, h, **R.REFERENCE_CAMERA)
    gpu = R.render(sc, cam, w, h, spp=4, max_depth=10, seed=11)
    ref, _, _ = _mirror(sc, cam, w, h, 4, 10, seed=11)
    _assert_parity(gpu, ref, f"ragged {w}x{h}")


@pytest.mark.parametrize("depth", [0, 1, 2, 64])
def test_depth_edges(gpu_lib, depth):
    from rtclj import raytracing as R
    sc = _ref_scene()
    cam = R.camera(64, 36, **R.REFERENCE_CAMERA)
    gpu = R.render(sc, cam, 64, 36, spp=4, max_depth=depth, seed=5)
    ref, _, _ = _mirror(sc, cam, 64, 36, 4, depth, seed=5)
    _assert_parity(gpu, ref, f"depth {depth}")
    if depth == 0:
        assert not gpu.any()  # ray-color depth <= 0 -> black (raytracing.clj:46-47)


def test_spp_zero_is_black(gpu_lib):
    from rtclj import raytracing as R
    cam = R.camera(16, 9, **R.REFERENCE_CAMERA)
    assert not R.render(_ref_scene(), cam, 16, 9, spp=0).any()


def test_empty_scene_is_sky(gpu_lib):
    from rtclj import raytracing as R
    sc = R.Scene(np.zeros((0, 4)), np.zeros(0), np.zeros((0, 4)))
    cam = R.camera(32, 18, **R.REFERENCE_CAMERA)
    gpu = R.render(sc, cam, 32, 18, spp=2, max_depth=50)
    ref, segs, _ = _mirror(sc, cam, 32, 18, 2, 50)
    _assert_parity(gpu, ref, "empty scene")
    assert segs == 32 * 18 * 2


def test_body_without_material_is_black(gpu_lib):
    from rtclj import hittable
    from rtclj import raytracing as R
    bodies = [hittable.sphere((0, 0, -1.2), 0.5)] + R.hittables
    sc = R.Scene.from_bodies(bodies)
    cam = R.camera(48, 27, **R.REFERENCE_CAMERA)
    gpu = R.render(sc, cam, 48, 27, spp=4, max_depth=20, seed=2)
    ref, _, _ = _mirror(sc, cam, 48, 27, 4, 20, seed=2)
    _assert_parity(gpu, ref, "RT_NONE body")


def test_no_defocus_and_seed_changes_image(gpu_lib):
    from rtclj import raytracing as R
    sc = _ref_scene()
    cam = R.camera(64, 36, 20.0, (-2, 2, 1), (0, 0, -1), (0, 1, 0), 0.0, 3.4)
    assert cam.defocus == 0
    a = R.render(sc, cam, 64, 36, spp=4, seed=1)
    b = R.render(sc, cam, 64, 36, spp=4, seed=2)
    ref, _, _ = _mirror(sc, cam, 64, 36, 4, 50, seed=1)
    _assert_parity(a, ref, "no defocus")
    assert not np.array_equal(a, b)


def test_row_tiles_and_sample_stripes_compose(gpu_lib):
    """Interleaved row-tile shards and sample stripes reproduce the full frame
    (RNG keyed by (seed, pixel, sample): independent of sharding)."""
    import ctypes as C
    from rtclj import raytracing as R
    from rtclj._lib import check, lib, rt_params
    sc = _ref_scene()
    w, h = 80, 45
    cam = R.camera(w, h, **R.REFERENCE_CAMERA)
    full = R.render(sc, cam, w, h, spp=8, seed=9)
    # rows [10, 45) in one call == the same rows of the full frame
    part = R.render(sc, cam, w, h, spp=8, seed=9, rows=(10, 45))
    assert np.array_equal(part, full[10:45])
    # sample stripes 0-3 and 4-7, recombined, agree with 8 spp up to fp32 re-association
    s0 = R.render(sc, cam, w, h, spp=4, seed=9)
    s1 = R.render(sc, cam, w, h, spp=4, seed=9, sample_begin=4)
    assert np.allclose((s0 + s1) / 2, full, atol=2e-6)
    # interleaved row-tile shards: the row selection covers every row once ...
    for step in (2, 3, 8):
        rows = []
        for first in range(step):
            p = rt_params(width=w, height=h, row_begin=0, row_end=h, row_tile=8, tile_first=first, tile_step=step)
            rows.append(check(lib.rt_rows_out(C.byref(p))))
        assert sum(rows) == h
    # ... and the multi-GPU fan-out + host gather reproduces the frame bit for bit
    from rtclj._lib import RT_FLAG_SHARDS_ON_DEVICE0
    for nshards, tile in ((2, 8), (3, 8), (8, 4), (5, 16)):
        st = {}
        sharded = R.render(sc, cam, w, h, spp=8, seed=9, n_devices=nshards, row_tile=tile,
                           flags=RT_FLAG_SHARDS_ON_DEVICE0, stats=st)
        assert st["n_devices"] == min(nshards, -(-h // tile))
        assert np.array_equal(sharded, full), (nshards, tile)


@pytest.mark.parametrize("samplers", SAMPLERS)
@pytest.mark.parametrize("v", [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 16, 17, 18, 19, 22, 24, 26, 28])
def test_every_variant_is_bit_exact(gpu_lib, v, samplers):
    """Kernel variants (product and diagnostic builds: table in LDS / scalar
    cache, simple / grouped / packed scan, BVH traversals, stats builds) all
    give the mirror's bits, with either samplers."""
    from rtclj import scenes
    from rtclj import raytracing as R
    sc = scenes.cover(11)
    w, h, spp = 72, 40, 7
    cam = scenes.cover_camera(w, h)
    with variant(v) as dll:
        st = {}
        g = R.render(sc, cam, w, h, spp=spp, seed=4, stats=st, library=dll, flags=_flags(samplers))
        if v in (3, 6, 7, 10, 13, 17, 19):
            import ctypes as C
            d = (C.c_uint64 * 32)()
            assert dll.rt_debug_stats(d) == 0 and d[0] > 0 and d[5] > 0
    ref, segs, _ = _mirror(sc, cam, w, h, spp, 50, seed=4, mode=_mode(samplers))
    assert np.array_equal(g, ref), f"variant {v}"
    assert st["segments"] == segs


@pytest.mark.parametrize("spp", [1, 2, 3, 4, 5, 63, 100, 8191, 8192, 12288])
def test_edge_spp(gpu_lib, spp):
    """spp around the pool's index arithmetic: multiply-high division up to
    8191 samples per pixel, exact integer division above (the round-1
    multiply-high was inexact there)."""
    from rtclj import raytracing as R
    sc = _ref_scene()
    w, h = (40, 22) if spp <= 100 else (9, 10)   # 9 x 10: a ragged tile in both directions
    cam = R.camera(w, h, **R.REFERENCE_CAMERA)
    st = {}
    g = R.render(sc, cam, w, h, spp=spp, max_depth=20, seed=8, stats=st)
    ref, segs, smp = _mirror(sc, cam, w, h, spp, 20, seed=8)
    assert np.array_equal(g, ref), spp
    assert st["segments"] == segs and st["samples"] == smp == w * h * spp


def test_max_spheres_and_too_many(gpu_lib):
    from rtclj import raytracing as R
    from rtclj._lib import RT_MAX_SPHERES
    from rtclj import RTError
    rng = np.random.default_rng(0)
    n = RT_MAX_SPHERES
    sph = np.zeros((n, 4), np.float32)
    sph[:, 0] = rng.uniform(-40, 40, n)
    sph[:, 1] = rng.uniform(-1, 3, n)
    sph[:, 2] = rng.uniform(-60, -5, n)
    sph[:, 3] = 0.1
    kind = rng.integers(0, 3, n).astype(np.int32)
    mat = np.column_stack([rng.uniform(0, 1, (n, 3)), np.where(kind == 2, 1.5, 0.3)]).astype(np.float32)
    sc = R.Scene(sph, kind, mat)
    cam = R.camera(32, 18, 40.0, (0, 1, 3), (0, 1, -10), (0, 1, 0), 0.0, 10.0)
    gpu = R.render(sc, cam, 32, 18, spp=2, max_depth=8, seed=1)
    ref, _, _ = _mirror(sc, cam, 32, 18, 2, 8, seed=1)
    _assert_parity(gpu, ref, "8192 spheres")
    big = R.Scene(np.zeros((n + 1, 4)), np.zeros(n + 1), np.zeros((n + 1, 4)))
    with pytest.raises(RTError) as ei:
        R.render(big, cam, 8, 8, spp=1)
    assert ei.value.code == -3


def test_bad_material_rejected(gpu_lib):
    from rtclj import raytracing as R
    from rtclj import RTError
    sc = R.Scene(np.array([[0, 0, -1, 0.5]]), np.array([7]), np.zeros((1, 4)))
    cam = R.camera(8, 8, **R.REFERENCE_CAMERA)
    with pytest.raises(RTError) as ei:
        R.render(sc, cam, 8, 8, spp=1)
    assert ei.value.code == -2


@pytest.mark.parametrize("samplers", SAMPLERS)
def test_gpu_matches_committed_mirror_fixture(gpu_lib, samplers):
    """Committed golden vectors, bit-exact: tests/golden/mirror_small_direct.npz
    (the default samplers) and mirror_small.npz (RT_FLAG_REJECTION_SAMPLERS),
    main and realm semantics."""
    from pathlib import Path
    from rtclj import raytracing as R
    from rtclj import realm, scenes
    name = "mirror_small_direct.npz" if samplers == "direct" else "mirror_small.npz"
    f = np.load(Path(__file__).parent / "golden" / name)
    fl = _flags(samplers)
    st = {}
    g = R.render(_ref_scene(), R.camera(48, 27, **R.REFERENCE_CAMERA), 48, 27, spp=8, seed=3, stats=st, flags=fl)
    assert np.array_equal(g, f["reference_48x27_spp8_seed3"]) and st["segments"] == f["segments"][0]
    g = R.render(scenes.cover(11), scenes.cover_camera(32, 18), 32, 18, spp=4, seed=5, stats=st, flags=fl)
    assert np.array_equal(g, f["cover_32x18_spp4_seed5"]) and st["segments"] == f["segments"][1]
    g = realm.render(R.Scene.from_bodies(realm.hittables), realm.camera(48, 27), 48, 27, spp=8, max_depth=50,
                     seed=3, stats=st, flags=fl)
    assert np.array_equal(g, f["realm_48x27_spp8_seed3"]) and st["segments"] == f["segments"][2]


@pytest.mark.parametrize("seed,samplers", [(1, "direct"), (2, "direct"), (1, "rejection")])
def test_gpu_reproduces_reference_scene_ppm(gpu_lib, seed, samplers):
    """Full reference config (400x225, 100 spp, depth 50) vs the reference's
    own scene.ppm, within SURVEY.md §8c's statistical tolerance: the default
    loop-free samplers (two seeds) and the rejection samplers."""
    from rtclj import raytracing as R
    from test_oracle_pinning import within_tolerance
    rgb = R.main(100, 50, out_path="/tmp/rtclj_scene_gpu.ppm", seed=seed, flags=_flags(samplers))
    ok, info = within_tolerance(rgb)
    assert all(ok.values()), (ok, info)
    assert np.array_equal(R.read_ppm("/tmp/rtclj_scene_gpu.ppm"), rgb)


def test_c1_frame_properties(gpu_lib):
    """BASELINE config C1 at full size (1200x675x100spp, cover scene): finite,
    in-range, deterministic, and its top rows match the mirror bit for bit."""
    from rtclj import raytracing as R
    from rtclj import scenes
    sc = scenes.cover(11)
    cam = scenes.cover_camera(1200, 675)
    st = {}
    a = R.render(sc, cam, 1200, 675, spp=100, max_depth=50, seed=1, stats=st)
    b = R.render(sc, cam, 1200, 675, spp=100, max_depth=50, seed=1)
    assert np.array_equal(a, b)
    assert np.isfinite(a).all() and a.min() >= 0 and a.max() <= 1.0 + 1e-6
    assert 2.5 < st["segments"] / st["samples"] < 2.9
    ref, _, _ = _mirror(sc, cam, 1200, 675, 100, 50, seed=1, rows=(300, 302))
    _assert_parity(a[300:302], ref, "C1 rows 300-301")


@pytest.mark.parametrize("v", [11, 12, 16, 18, 22, 24, 26])
def test_bvh_bit_exact_on_full_c1_and_reference(gpu_lib, v):
    """The BVH traversal returns the scan's hits bit for bit: full C1 frame
    (1200x675, 100 spp) and the reference scene, BVH vs brute-force scan."""
    from rtclj import raytracing as R
    from rtclj import scenes
    from rtclj._lib import lib
    cases = [(scenes.cover(11), scenes.cover_camera(1200, 675), 1200, 675, 100),
             (scenes.cover(16), scenes.cover_camera(640, 360), 640, 360, 16),
             (_ref_scene(), R.camera(400, 225, **R.REFERENCE_CAMERA), 400, 225, 100)]
    for sc, cam, w, h, spp in cases:
        with variant(5) as dll:
            st_a = {}
            a = R.render(sc, cam, w, h, spp=spp, seed=1, stats=st_a, library=dll)
        with variant(v) as dll:
            st_b = {}
            b = R.render(sc, cam, w, h, spp=spp, seed=1, stats=st_b, library=dll)
        assert np.array_equal(a, b), (w, h, int((a != b).any(axis=-1).sum()))
        assert st_a["segments"] == st_b["segments"]


def test_bvh_axis_aligned_rays(gpu_lib):
    """Rays with exactly-zero direction components (axis-aligned camera looking
    down -z at pixel centres on the axes) through the BVH == the scan."""
    from rtclj import raytracing as R
    from rtclj import scenes
    from rtclj._lib import lib
    sc = scenes.cover(11)
    # vfov / position chosen so the centre column and row give u_x = 0 / u_y = 0
    cam = R.camera(65, 37, 60.0, (0.0, 1.0, 12.0), (0.0, 1.0, 0.0), (0.0, 1.0, 0.0), 0.0, 12.0)
    out = {}
    for v in (5, 11, 16):
        with variant(v) as dll:
            out[v] = R.render(sc, cam, 65, 37, spp=64, seed=3, library=dll)
    assert np.array_equal(out[5], out[11])
    assert np.array_equal(out[5], out[16])


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 6, 7, 9, 13, 33])
def test_bvh_small_scenes(gpu_lib, n):
    """Small and ragged body counts (a leaf-only tree, a repeated leaf, pad
    bodies in a 2- or 4-body leaf) through both trees == the scan."""
    from rtclj import raytracing as R
    from rtclj._lib import lib
    rng = np.random.default_rng(n)
    sph = np.zeros((n, 4), np.float32)
    sph[:, 0] = rng.uniform(-3, 3, n)
    sph[:, 1] = rng.uniform(0, 2, n)
    sph[:, 2] = rng.uniform(-6, -1, n)
    sph[:, 3] = rng.uniform(0.2, 0.9, n)
    kind = rng.integers(0, 3, n).astype(np.int32)
    mat = np.column_stack([rng.uniform(0, 1, (n, 3)), np.where(kind == 2, 1.5, 0.3)]).astype(np.float32)
    sc = R.Scene(sph, kind, mat)
    cam = R.camera(48, 27, **R.REFERENCE_CAMERA)
    out = {}
    for v in (5, 11, 16, 18, 22, 24, 26):
        with variant(v) as dll:
            out[v] = R.render(sc, cam, 48, 27, spp=8, max_depth=20, seed=5, library=dll)
    for v in (11, 16, 18, 22, 24, 26):
        assert np.array_equal(out[5], out[v]), v
    ref, _, _ = _mirror(sc, cam, 48, 27, 8, 20, seed=5)
    assert np.array_equal(out[5], ref)


@pytest.mark.parametrize("n_big", [1, 3, 4, 5, 9, 12])
def test_bvh_big_bodies(gpu_lib, n_big):
    """Bodies > 4x the median radius leave the tree (up to 8 of them, largest
    first; bvh.cpp) and are tested as packed leaves of their own before every
    traversal: 1, 2 or 3 such leaves for 2-, 4- and 8-body trees, ties in
    radius, the rest staying in the tree -- all == the scan and the mirror."""
    from rtclj import raytracing as R
    from rtclj._lib import lib
    rng = np.random.default_rng(100 + n_big)
    n = 60 + n_big
    sph = np.zeros((n, 4), np.float32)
    sph[:, 0] = rng.uniform(-4, 4, n)
    sph[:, 1] = rng.uniform(0, 1, n)
    sph[:, 2] = rng.uniform(-8, -1, n)
    sph[:, 3] = 0.2
    big = rng.choice(n, n_big, replace=False)
    sph[big, 3] = rng.choice([1.0, 1.5], n_big)          # ties among the big radii
    sph[big[0]] = (0.0, -100.5, -1.0, 100.0)             # a ground
    kind = rng.integers(0, 3, n).astype(np.int32)
    mat = np.column_stack([rng.uniform(0, 1, (n, 3)), np.where(kind == 2, 1.5, 0.3)]).astype(np.float32)
    sc = R.Scene(sph, kind, mat)
    cam = R.camera(64, 36, **R.REFERENCE_CAMERA)
    out = {}
    for v in (5, 11, 16, 18, 22, 24, 26):
        with variant(v) as dll:
            out[v] = R.render(sc, cam, 64, 36, spp=8, max_depth=20, seed=9, library=dll)
    for v in (11, 16, 18, 22, 24, 26):
        assert np.array_equal(out[5], out[v]), v
    ref, _, _ = _mirror(sc, cam, 64, 36, 8, 20, seed=9)
    assert np.array_equal(out[5], ref)


def test_bvh_cover16_u8_stack_and_u16_indices(gpu_lib):
    """C4's scene (cover grid 16, 1025 bodies): the 8-body-leaf traversal
    (u8 stack, u16 body indices, leaves in two halves; the scene's resolved
    variant), the 4-body one, and the 4-body compact image in 4-, 8- and
    16-wave workgroups (22, 24, 26: the default launch here) == the scan ==
    the mirror."""
    import ctypes as C
    from rtclj import raytracing as R
    from rtclj import scenes
    from rtclj._lib import check, lib
    sc = scenes.cover(16)
    cam = scenes.cover_camera(96, 54)
    ds = C.c_void_p()
    check(lib.rt_scene_upload(0, C.byref(sc.c), C.byref(ds)))
    try:
        assert lib.rt_resolve_variant(ds) == 18
    finally:
        lib.rt_scene_free(ds)
    out = {}
    for v in (0, 5, 16, 18, 22, 24, 26):
        with variant(v) as dll:
            out[v] = R.render(sc, cam, 96, 54, spp=6, max_depth=64, seed=4, library=dll)
    for v in (0, 16, 18, 22, 24, 26):
        assert np.array_equal(out[5], out[v]), v
    ref, _, _ = _mirror(sc, cam, 96, 54, 6, 64, seed=4)
    assert np.array_equal(out[5], ref)


def test_bvh_8body_tree_over_256_nodes_uses_4body(gpu_lib):
    """An 8-body tree with more than 256 nodes cannot use the u8 stack:
    variant 18 resolves to 16 (or to 12 when that tree misses LDS) -- same
    bits as the scan."""
    import ctypes as C
    from rtclj import raytracing as R
    from rtclj._lib import check, lib
    rng = np.random.default_rng(7)
    n = 2600
    sph = np.zeros((n, 4), np.float32)
    sph[:, 0] = rng.uniform(-30, 30, n)
    sph[:, 1] = rng.uniform(0, 1, n)
    sph[:, 2] = rng.uniform(-40, -2, n)
    sph[:, 3] = rng.uniform(0.05, 0.2, n)
    kind = rng.integers(0, 3, n).astype(np.int32)
    mat = np.column_stack([rng.uniform(0, 1, (n, 3)), np.where(kind == 2, 1.5, 0.3)]).astype(np.float32)
    sc = R.Scene(sph, kind, mat)
    cam = R.camera(64, 36, 40.0, (0, 2, 3), (0, 0, -10), (0, 1, 0), 0.0, 10.0)
    ds = C.c_void_p()
    check(lib.rt_scene_upload(0, C.byref(sc.c), C.byref(ds)))
    old = lib.rt_set_variant(18)
    try:
        assert lib.rt_resolve_variant(ds) in (16, 12)
    finally:
        lib.rt_set_variant(old)
        lib.rt_scene_free(ds)
    out = {}
    for v in (5, 18):
        with variant(v) as dll:
            out[v] = R.render(sc, cam, 64, 36, spp=4, max_depth=10, seed=2, library=dll)
    assert np.array_equal(out[5], out[18])


@pytest.mark.parametrize("vsel", [0, 11, 16, 18, 22, 24, 26])
def test_bvh_large_scene_falls_back(gpu_lib, vsel):
    """8192 bodies: the trees exceed the LDS budget, the launch falls back to
    the global-memory traversal of the 2-body tree: same bits as the scan."""
    from rtclj import raytracing as R
    from rtclj._lib import lib, RT_MAX_SPHERES
    rng = np.random.default_rng(1)
    n = RT_MAX_SPHERES
    sph = np.zeros((n, 4), np.float32)
    sph[:, 0] = rng.uniform(-40, 40, n)
    sph[:, 1] = rng.uniform(-1, 3, n)
    sph[:, 2] = rng.uniform(-60, -5, n)
    sph[:, 3] = rng.uniform(0.05, 0.3, n)
    kind = rng.integers(0, 3, n).astype(np.int32)
    mat = np.column_stack([rng.uniform(0, 1, (n, 3)), np.where(kind == 2, 1.5, 0.3)]).astype(np.float32)
    sc = R.Scene(sph, kind, mat)
    cam = R.camera(96, 54, 40.0, (0, 1, 3), (0, 1, -10), (0, 1, 0), 0.0, 10.0)
    out = {}
    for v in (5, vsel):
        with variant(v) as dll:
            out[v] = R.render(sc, cam, 96, 54, spp=4, max_depth=10, seed=2, library=dll)
    assert np.array_equal(out[5], out[vsel])


def _realm_mirror(scene, cam, w, h, spp, depth, seed=1, rows=None, mode=KERNEL_REALM32):
    out, _, segs, smp = oracle.render(mode, scene.sphere.astype(np.float64), scene.kind,
                                      scene.mat.astype(np.float64), cam.as_list(), cam.defocus, w, h, spp, depth,
                                      seed=seed, rows=rows)
    return out, segs, smp


@pytest.mark.parametrize("samplers", SAMPLERS)
@pytest.mark.parametrize("vsel", [0, 5, 11, 16, 18, 22, 24, 26, 28])
def test_realm_flag_matches_mirror(gpu_lib, vsel, samplers):
    """RT_FLAG_REALM (realm.raytracing semantics) through the kernel == the
    oracle's MODE_REALM32 (| DIRECT with the default samplers), bit for bit:
    the realm scene and the cover scene."""
    from rtclj import raytracing as R
    from rtclj import realm, scenes
    from rtclj._lib import lib
    cases = [(R.Scene.from_bodies(realm.hittables), realm.camera(48, 27), 48, 27, 8),
             (scenes.cover(11), scenes.cover_camera(40, 22), 40, 22, 7)]
    with variant(vsel) as dll:
        for sc, cam, w, h, spp in cases:
            st = {}
            g = realm.render(sc, cam, w, h, spp=spp, max_depth=50, seed=3, stats=st, library=dll,
                             flags=_flags(samplers))
            ref, segs, smp = _realm_mirror(sc, cam, w, h, spp, 50, seed=3, mode=_mode(samplers, realm=True))
            assert np.array_equal(g, ref), (vsel, w, h)
            assert st["segments"] == segs and st["samples"] == smp


def test_realm_shards_and_fixture(gpu_lib):
    """realm's own frame (400x224, 100 spp, depth 50) on the GPU: sharded ==
    single, rows bit-exact with the mirror, and the image within the
    scene-realm.ppm tolerances (tests/test_realm.py)."""
    import json
    from pathlib import Path
    from rtclj import raytracing as R
    from rtclj import realm
    from rtclj._lib import RT_FLAG_SHARDS_ON_DEVICE0
    sc = R.Scene.from_bodies(realm.hittables)
    w = 400
    h = realm.image_height(w)
    cam = realm.camera(w, h)
    lin = realm.render(sc, cam, w, h, seed=1)
    shard = realm.render(sc, cam, w, h, seed=1, n_devices=3, flags=RT_FLAG_SHARDS_ON_DEVICE0)
    assert np.array_equal(lin, shard)
    ref, _, _ = _realm_mirror(sc, cam, w, h, 100, 50, seed=1, rows=(100, 104))
    assert np.array_equal(lin[100:104], ref)
    g = Path(__file__).parent / "golden"
    st = json.loads((g / "scene_realm_ppm_stats.json").read_text())
    pix = np.load(g / "scene_realm_ppm.npz")["pixels"]
    rgb = R.write_color(lin).astype(np.float64)
    blocks = np.array([[rgb[y * h // 9:(y + 1) * h // 9, x * w // 16:(x + 1) * w // 16].reshape(-1, 3).mean(0)
                        for x in range(16)] for y in range(9)])
    d = np.abs(blocks - np.array(st["blocks"]))
    assert d.mean() <= 0.25 and d.max() <= 2.5, (d.mean(), d.max())
    assert np.abs(rgb - pix).mean() <= 3.5


def test_compact_variant_limits(gpu_lib):
    """Variant 22 (the 4-body walk in a compact LDS image: u8 node-index
    stack, u32 pixel sums with their wraps counted in a byte per channel,
    seven workgroups per CU), when selected, runs only where those sums
    cannot overflow: spp < 65536 and every albedo within [-1, 1] (a sample
    adds at most 2^24 per channel, so a channel wraps at most spp / 256 <
    256 times). At spp 255 -- the largest sums without a wrap -- it equals
    the mirror bit for bit; at 65536, or with an albedo above 1, the launch
    runs 16 (u64 sums). The default selector runs 22 wherever it applies."""
    import ctypes as C
    from rtclj import raytracing as R
    from rtclj import scenes
    from rtclj._lib import check, lib, rt_params

    def launch_variant(sc, w, h, spp):
        ds = C.c_void_p()
        check(lib.rt_scene_upload(0, C.byref(sc.c), C.byref(ds)))
        try:
            p = rt_params(width=w, height=h, row_begin=0, row_end=h, spp=spp, max_depth=50, seed=1)
            o = (C.c_int * 4)()
            check(lib.rt_launch_occupancy(ds, C.byref(p), o))
            return o[3], o[0]
        finally:
            lib.rt_scene_free(ds)

    sc = scenes.cover(11)
    assert launch_variant(sc, 1200, 675, 100) == (22, 7)   # the default where it applies
    assert launch_variant(sc, 3840, 2160, 500) == (22, 7)   # C2 (its sums count their wraps)
    assert launch_variant(sc, 3840, 2160, 1000) == (22, 7)  # C3
    assert launch_variant(sc, 64, 36, 65536)[0] == 16       # a channel could wrap 256 times
    # a launch of few 8 x 8 tiles stays on 22 (sample splits) by default; with
    # RTCLJ_TH4=2 (fewer tiles than twice the device's workgroup slots) it runs
    # 22's image on whole 8 x 4-pixel pools (28): C1's 8- and 4-GPU shards
    assert launch_variant(sc, 1200, 84, 100) == (22, 7)
    import os
    os.environ["RTCLJ_TH4"] = "2"
    try:
        assert launch_variant(sc, 1200, 84, 100) == (28, 7)
        assert launch_variant(sc, 1200, 168, 100) == (28, 7)
        assert launch_variant(sc, 1200, 340, 100) == (22, 7)   # (2-GPU shard: 6,375 tiles, whole 8 x 8)
        assert launch_variant(sc, 200, 112, 100) == (28, 7)
    finally:
        del os.environ["RTCLJ_TH4"]
    with variant(22):
        assert launch_variant(sc, 1200, 675, 100) == (22, 7)
        assert launch_variant(sc, 1200, 675, 255)[0] == 22
        assert launch_variant(sc, 1200, 675, 65535)[0] == 22
        assert launch_variant(sc, 1200, 675, 65536)[0] == 16
        hot = R.Scene(sc.sphere.copy(), sc.kind.copy(), sc.mat.copy())
        lam = np.nonzero(hot.kind == 0)[0]   # (RT_LAMBERTIAN)
        hot.mat[lam[0], 0] = 1.5                      # one albedo channel above 1
        assert launch_variant(hot, 1200, 675, 100)[0] == 16
        # spp 255 on a small cover frame: the u32 sums at their largest
        cam = scenes.cover_camera(160, 90)
        g = R.render(sc, cam, 160, 90, spp=255, seed=3)
    ref, _, _ = _mirror(sc, cam, 160, 90, 255, 50, seed=3)
    assert np.array_equal(g, ref)


@pytest.mark.parametrize("scene_kind,w,h,spp", [("sky", 24, 16, 1300), ("cover", 48, 27, 600)])
def test_compact_variant_counts_wraps(gpu_lib, scene_kind, w, h, spp):
    """spp > 255 in the compact variant: a pixel's u32 sum wraps past
    2^32 every ~256 bright samples and the wraps are counted per channel
    (trace_kernel.h s_carry). A sky-only frame (colour up to 1: ~4 wraps per
    channel at 1300 spp) and the cover scene at 600 spp equal the mirror bit
    for bit, on 22 (the default) and on 28 (the same image on 8 x 4-pixel
    pools)."""
    import ctypes as C
    from rtclj import raytracing as R
    from rtclj import scenes
    from rtclj._lib import check, lib, rt_params
    if scene_kind == "sky":   # one small body behind the camera: every sample is the sky
        sc = R.Scene(np.array([[0.0, 0.0, 10.0, 0.1]]), np.array([0]), np.array([[0.5, 0.5, 0.5, 0.0]]))
        cam = R.camera(w, h, **R.REFERENCE_CAMERA)
    else:
        sc = scenes.cover(11)
        cam = scenes.cover_camera(w, h)
    ref, segs, _ = _mirror(sc, cam, w, h, spp, 50, seed=4)
    for vsel, want in ((0, 22), (28, 28)):
        with variant(vsel):
            ds = C.c_void_p()
            check(lib.rt_scene_upload(0, C.byref(sc.c), C.byref(ds)))
            try:
                o = (C.c_int * 4)()
                p = rt_params(width=w, height=h, row_begin=0, row_end=h, spp=spp, max_depth=50, seed=1)
                check(lib.rt_launch_occupancy(ds, C.byref(p), o))
                assert o[3] == want, (vsel, o[3])
            finally:
                lib.rt_scene_free(ds)
            st = {}
            g = R.render(sc, cam, w, h, spp=spp, max_depth=50, seed=4, stats=st)
        assert np.array_equal(g, ref), vsel
        assert st["segments"] == segs


def test_compact_variant_wide_frame(gpu_lib):
    """Variant 22's pixel table packs (x | y << 16): a frame wider than 65536
    pixels runs 16 instead, and its columns past 65536 equal the
    mirror bit for bit (a 70000 x 2 frame at 1 spp, those columns checked)."""
    import ctypes as C
    from rtclj import raytracing as R
    from rtclj import scenes
    from rtclj._lib import check, lib, rt_params
    sc = scenes.cover(11)
    w, h = 70000, 2
    ds = C.c_void_p()
    check(lib.rt_scene_upload(0, C.byref(sc.c), C.byref(ds)))
    try:
        o = (C.c_int * 4)()
        p = rt_params(width=w, height=h, row_begin=0, row_end=h, spp=1, max_depth=50, seed=1)
        check(lib.rt_launch_occupancy(ds, C.byref(p), o))
        assert o[3] == 16, o[3]
        p = rt_params(width=65536, height=h, row_begin=0, row_end=h, spp=1, max_depth=50, seed=1)
        check(lib.rt_launch_occupancy(ds, C.byref(p), o))
        assert o[3] == 22, o[3]
    finally:
        lib.rt_scene_free(ds)
    cam = scenes.cover_camera(w, h)
    g = R.render(sc, cam, w, h, spp=1, seed=5)
    cols = (65520, 65600)
    ref, _, _, _ = oracle.render(KERNEL32, sc.sphere.astype(np.float64), sc.kind,
                                 sc.mat.astype(np.float64), cam.as_list(), cam.defocus, w, h, 1, 50, seed=5, cols=cols)
    assert np.array_equal(g[:, cols[0]:cols[1]], ref[:, cols[0]:cols[1]])
