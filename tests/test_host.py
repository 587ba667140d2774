"""Host-side mirror of the reference interface (rtclj): scene data, camera,
write-color!, PPM, scene builders, shard planning.  No GPU needed."""
import numpy as np
import pytest


def test_image_height_uses_exact_ratio():
    from rtclj.raytracing import image_height
    # (int (/ image-width 16/9)) with Clojure's exact ratio (raytracing.clj:105-107)
    assert [image_height(w) for w in (400, 200, 1200, 3840, 7680, 1)] == [225, 112, 675, 2160, 4320, 0]


def test_reference_scene_matches_c_builder():
    from rtclj import raytracing as R
    from rtclj import scenes
    a = R.Scene.from_bodies(R.hittables)
    b = scenes.reference()
    assert np.array_equal(a.sphere, b.sphere) and np.array_equal(a.kind, b.kind) and np.array_equal(a.mat, b.mat)
    assert a.kind.tolist() == [0, 0, 2, 2, 1]
    assert a.mat[3, 3] == np.float32(1.0 / 1.5)   # the bubble (raytracing.clj:74-75)


def test_flatten_and_errors():
    from rtclj import hittable, material
    from rtclj import raytracing as R
    bodies = [{**hittable.sphere((1, 2, 3), 0.5), **material.metal((0.1, 0.2, 0.3), 0.7)},
              hittable.sphere((0, 0, 0), 1.0)]
    sph, kind, mat = R.flatten(bodies)
    assert sph.tolist() == [[1, 2, 3, 0.5], [0, 0, 0, 1]]
    assert kind.tolist() == [1, 3]
    assert mat[0].tolist() == pytest.approx([0.1, 0.2, 0.3, 0.7])
    with pytest.raises(ValueError):
        R.flatten([{"hittable/kind": "box"}])
    with pytest.raises(ValueError):
        R.flatten([{**hittable.sphere((0, 0, 0), 1), "material/type": "plastic"}])
    with pytest.raises(ValueError):
        hittable.sphere((0, 0), 1)
    s64, k64, m64 = R.flatten64(R.hittables)
    assert s64.dtype == np.float64 and m64[1, :3].tolist() == [0.1, 0.2, 0.5]


def test_material_reflectance_mirror():
    from rtclj import material
    import oracle
    for c, ri in [(0.0, 1.5), (0.3, 1 / 1.5), (1.0, 1.5)]:
        assert material.reflectance(c, ri) == pytest.approx(oracle.reflectance(c, ri), rel=1e-15)


def test_cover_scene_deterministic_and_sized():
    from rtclj import scenes
    a, b = scenes.cover(11, 42), scenes.cover(11, 42)
    assert np.array_equal(a.sphere, b.sphere) and np.array_equal(a.mat, b.mat)
    assert 470 <= len(a) <= 490 and len(scenes.cover(16)) > 1000
    assert not np.array_equal(scenes.cover(11, 43).sphere, a.sphere)
    assert a.sphere[0].tolist() == [0, -1000, 0, 1000]
    small = a.sphere[1:-3]
    assert (small[:, 3] == np.float32(0.2)).all() and (small[:, 1] == np.float32(0.2)).all()
    d = np.hypot(small[:, 0] - 4.0, small[:, 2])
    assert (d > 0.9).all()                                     # RTIOW §14 exclusion
    assert set(np.unique(a.kind)) <= {0, 1, 2}
    met = a.mat[a.kind == 1]
    assert (met[:, :3] >= 0.5).all() and (met[:, 3] < 0.5).all()


def test_ppm_round_trip(tmp_path):
    from rtclj import raytracing as R
    img = np.random.default_rng(0).integers(0, 256, (5, 7, 3)).astype(np.uint8)
    p = tmp_path / "x.ppm"
    R.write_ppm(p, img)
    text = p.read_text().splitlines()
    assert text[:3] == ["P3", "7 5", "255"] and len(text) == 3 + 35
    assert text[3] == " ".join(str(v) for v in img[0, 0])   # "r g b" per line (raytracing.clj:24-26)
    assert np.array_equal(R.read_ppm(p), img)


def test_ppm_bytes_equal_per_value_formatting(tmp_path):
    """rt_write_ppm's table of decimal strings writes the bytes a "%d %d %d\\n"
    per pixel would (raytracing.clj:172-175): every value 0..255, and a frame
    of C1's width."""
    from rtclj import raytracing as R
    vals = np.arange(256, dtype=np.uint8)
    rng = np.random.default_rng(1)
    for img in (np.stack([vals, vals[::-1], np.roll(vals, 7)], -1).reshape(16, 16, 3),
                rng.integers(0, 256, (9, 1200, 3)).astype(np.uint8)):
        p = tmp_path / "v.ppm"
        R.write_ppm(p, img)
        h, w = img.shape[:2]
        want = f"P3\n{w} {h}\n255\n" + "".join(f"{r} {g} {b}\n" for r, g, b in img.reshape(-1, 3).tolist())
        assert p.read_bytes() == want.encode()


def test_shard_plans_cover_frame_once():
    from rtclj.shard import gather_rows, shard_params, shard_rows
    h, w = 675, 3
    for world in (1, 2, 3, 4, 8):
        parts = []
        for r in range(world):
            p = shard_params(world, r, w, h, 100, 50, scaling="strong")
            rows = shard_rows(h, p.get("row_tile", 8), p.get("tile_first", 0), p.get("tile_step", 0))
            parts.append((rows, np.full((len(rows), w, 3), r, np.float32)))
        img = gather_rows(h, w, parts)
        assert (img[:, 0, 0] == (np.arange(h) // 8) % world).all()
        wk = [shard_params(world, r, w, h, 100, 50, scaling="weak")["sample_begin"] for r in range(world)]
        assert wk == [100 * r for r in range(world)]
    with pytest.raises(ValueError):
        gather_rows(4, 1, [([0, 1], np.zeros((2, 1, 3))), ([1, 2, 3], np.zeros((3, 1, 3)))])
    with pytest.raises(ValueError):
        shard_params(2, 2, 1, 1, 1, 1)


def test_render_out_buffer_is_checked_before_any_device_call():
    """render(out=...) reuses a caller framebuffer: the wrong shape, dtype or
    layout is refused before the library is called (no GPU needed)."""
    import numpy as np
    import pytest
    from rtclj import raytracing as R, scenes
    sc = scenes.cover(11)
    cam = scenes.cover_camera(64, 36)
    for bad in (np.empty((36, 64, 3), np.float64), np.empty((35, 64, 3), np.float32),
                np.empty((64, 36, 3), np.float32).transpose(1, 0, 2)):
        with pytest.raises(ValueError):
            R.render(sc, cam, 64, 36, 1, 50, out=bad)
