"""realm.raytracing semantics (RT_FLAG_REALM): the oracle's realm modes
against the reference's own realm output, scene-realm.ppm (`clojure -M:realm`,
400x224, 100 spp, depth 50), and the host constants of the realm namespace.

Tolerances as for scene.ppm: 16x9 block means mean |d| <= 0.25
and max |d| <= 2.5, image mean within 0.15, neighbour-difference std within
0.15, per-pixel mean |d| <= 3.5.  Measured: block mean 0.105 / max 0.83,
per-pixel 2.24.  -main's semantics on the same scene and camera must fail
(block max ~97: Schlick reflectance on the glass).
"""
import json
from pathlib import Path

import numpy as np
import pytest

import oracle

G = Path(__file__).parent / "golden"
STATS = json.loads((G / "scene_realm_ppm_stats.json").read_text())
PIX = np.load(G / "scene_realm_ppm.npz")["pixels"]


def _stats(img):
    img = img.astype(np.float64)
    h, w = img.shape[:2]
    blocks = np.array([[img[y * h // 9:(y + 1) * h // 9, x * w // 16:(x + 1) * w // 16].reshape(-1, 3).mean(0)
                        for x in range(16)] for y in range(9)])
    return img.reshape(-1, 3).mean(0), blocks, np.diff(img, axis=1).reshape(-1, 3).std(0)


def _checks(rgb8):
    mean, blocks, nbr = _stats(rgb8)
    d = np.abs(blocks - np.array(STATS["blocks"]))
    return {"block_mean": d.mean() <= 0.25, "block_max": d.max() <= 2.5,
            "image_mean": bool((np.abs(mean - np.array(STATS["mean"])) <= 0.15).all()),
            "nbr_std": bool((np.abs(nbr - np.array(STATS["nbr_std"])) <= 0.15).all()),
            "pixel_mean": np.abs(rgb8.astype(np.float64) - PIX.astype(np.float64)).mean() <= 3.5}


def _quantize(lin):
    """write-color! in numpy (raytracing.clj:19-26; realm/raytracing.clj:353-356)."""
    g = np.where(lin > 0, np.sqrt(np.maximum(lin, 0)), 0.0)
    return (256.0 * np.clip(g, 0.0, 0.999)).astype(np.int64).astype(np.uint8)


def _render(mode, spp=100, seed=1, w=400, h=None, depth=50, bodies=None):
    from rtclj import raytracing as R
    from rtclj import realm
    h = realm.image_height(w) if h is None else h
    sc = R.Scene.from_bodies(realm.hittables if bodies is None else bodies)
    cam = realm.camera(w, h)
    out, out64, segs, smp = oracle.render(mode, sc.sphere.astype(np.float64), sc.kind, sc.mat.astype(np.float64),
                                          cam.as_list(), cam.defocus, w, h, spp, depth, seed=seed,
                                          want64=mode in (oracle.MODE_REF64, oracle.MODE_REALM64))
    return (out64 if out64 is not None else out), segs, smp


def test_realm_host_constants():
    from rtclj import realm
    # (int (/ ^double 400 ^double 16/9)): Ratio.doubleValue rounds 16/9 through a
    # 16-digit decimal, 400 / 1.777777777777778 = 224.99999999999997 -> 224
    assert realm.image_height(400) == 224 == PIX.shape[0] == STATS["height"]
    assert PIX.shape[1] == 400
    assert realm.focal_length() == pytest.approx(12 ** 0.5, abs=1e-15)
    assert [b["hittable/center"] for b in realm.hittables][:2] == [(0.0, 0.0, -1.2), (0.0, -100.5, -1.0)]


@pytest.mark.parametrize("mode", ["REALM64", "REALM32"])
def test_realm_modes_reproduce_scene_realm_ppm(mode):
    lin, segs, smp = _render(getattr(oracle, f"MODE_{mode}"))
    assert smp == 400 * 224 * 100
    checks = _checks(_quantize(lin))
    assert all(checks.values()), checks


def test_main_semantics_fail_the_realm_fixture():
    lin, _, _ = _render(oracle.MODE_REF64)
    checks = _checks(_quantize(lin))
    assert not checks["block_max"] and not checks["block_mean"], checks


@pytest.mark.parametrize("name,direct", [("mirror_small.npz", 0), ("mirror_small_direct.npz", 0x30)])
def test_realm_mirror_matches_committed_fixture(name, direct):
    fx = np.load(G / name)
    lin, segs, _ = _render(oracle.MODE_REALM32 | direct, spp=8, seed=3, w=48, h=27)
    assert np.array_equal(lin, fx["realm_48x27_spp8_seed3"])
    assert segs == int(fx["segments"][2])


def test_realm_flag_only_changes_its_three_rules():
    """Without dielectrics the draws are the same and the near-zero fallback
    never fires; with spp a power of two sum*(1/spp) == sum/spp exactly: the
    realm and main fp32 contracts then agree bit for bit.  With the glass they
    differ (no Schlick draw)."""
    from rtclj import realm
    opaque = [b for b in realm.hittables if b["material/type"] != "dielectric"]
    a, sa, _ = _render(oracle.MODE_REALM32, spp=8, w=40, h=22, bodies=opaque)
    b, sb, _ = _render(oracle.MODE_MIRROR32, spp=8, w=40, h=22, bodies=opaque)
    assert np.array_equal(a, b) and sa == sb
    c, _, _ = _render(oracle.MODE_REALM32, spp=8, w=40, h=22)
    d, _, _ = _render(oracle.MODE_MIRROR32, spp=8, w=40, h=22)
    assert not np.array_equal(c, d)
