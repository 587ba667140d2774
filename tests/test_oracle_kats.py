"""Oracle pinning, part 1: every hot-path function of the oracle's fp64
reference mode against known answers derived independently (pure Python,
tests/golden/make_golden.py) from the cited Clojure formulas; the product's
host helpers (camera, write-color!) against the same answers."""
import ctypes as C
import json
import math
from pathlib import Path

import numpy as np
import pytest

import oracle

K = json.loads((Path(__file__).parent / "golden" / "kats.json").read_text())
RNG = json.loads((Path(__file__).parent / "golden" / "rng_golden.json").read_text())


@pytest.mark.parametrize("case", K["sphere_hit"], ids=lambda c: c["name"])
def test_sphere_hit(case):
    tmax = math.inf if case["tmax"] == "inf" else case["tmax"]
    got = oracle.sphere_hit(case["sphere"], case["o"], case["d"], case["tmin"], tmax)
    exp = case["out"]
    assert got["hit"] == exp["hit"]
    if exp["hit"]:
        assert got["t"] == pytest.approx(exp["t"], rel=1e-15, abs=1e-15)
        assert got["p"] == pytest.approx(exp["p"], rel=1e-14, abs=1e-15)
        assert got["n"] == pytest.approx(exp["n"], rel=1e-14, abs=1e-15)
        assert got["front"] == exp["front"]


def test_sphere_hit_semantics_spotchecks():
    """Hand-derived: unit sphere at z=-1 r=.5 from the origin along -z hits at
    t=.5 front; with d=(0,0,-2) the root is t=.25 (un-normalised direction);
    from inside the far root is taken and the normal flips (back face)."""
    by = {c["name"]: c["out"] for c in K["sphere_hit"]}
    assert by["front hit"]["t"] == 0.5 and by["front hit"]["front"]
    assert by["unnormalised dir"]["t"] == 0.25
    assert not by["behind"]["hit"] and not by["miss"]["hit"]
    inside = by["inside -> far root, back face"]
    assert inside["hit"] and not inside["front"] and inside["t"] == pytest.approx(1.2)
    assert inside["n"] == pytest.approx([0, 0, 1])
    assert by["tmin straddle: near root <= tmin"]["t"] == pytest.approx(0.9995)
    assert not by["t-max cut"]["hit"]
    # near root 0.5 lies in (1e-3, 0.75): taken although the far root 1.5 is past t-max
    assert by["t-max between roots"]["hit"] and by["t-max between roots"]["t"] == 0.5


@pytest.mark.parametrize("case", K["reflect"])
def test_reflect(case):
    assert oracle.reflect(case["v"], case["n"]) == pytest.approx(case["out"], abs=1e-15)


@pytest.mark.parametrize("case", K["refract"])
def test_refract(case):
    assert oracle.refract(case["uv"], case["n"], case["eta"]) == pytest.approx(case["out"], abs=1e-15)


@pytest.mark.parametrize("case", K["reflectance"])
def test_reflectance(case):
    assert oracle.reflectance(case["cos"], case["ri"]) == pytest.approx(case["out"], rel=1e-15)


def test_reflectance_endpoints():
    r0 = ((1 - 1.5) / (1 + 1.5)) ** 2
    assert oracle.reflectance(1.0, 1.5) == pytest.approx(r0)      # normal incidence
    assert oracle.reflectance(0.0, 1.5) == pytest.approx(1.0)     # grazing


@pytest.mark.parametrize("case", K["lambertian_dir"])
def test_lambertian(case):
    assert oracle.lambertian_dir(case["unit"], case["n"]) == pytest.approx(case["out"], abs=1e-15)


def test_lambertian_near_zero_fallback():
    c = K["lambertian_dir"][2]   # unit ~= -n: scatter ~ 0 -> the normal itself (vec3a.clj:88-92)
    assert c["out"] == c["n"]


@pytest.mark.parametrize("case", K["metal_dir"])
def test_metal(case):
    ok, r = oracle.metal_dir(case["d"], case["n"], case["fuzz"], case["unit"])
    assert ok == case["scattered"]
    assert r == pytest.approx(case["out"], abs=1e-15)


def test_metal_absorbs_and_keeps_unnormalised_d():
    by = K["metal_dir"]
    assert by[0]["out"] == [1, 1, 0] and by[0]["scattered"]          # (1,-1,0) mirrored about y
    assert not by[1]["scattered"]                                     # fuzz pushes below the surface
    assert not by[3]["scattered"]


@pytest.mark.parametrize("case", K["dielectric_dir"])
def test_dielectric(case):
    refl, r = oracle.dielectric_dir(case["d"], case["n"], case["front"], case["eta"], case["xi"])
    assert refl == case["reflected"]
    assert r == pytest.approx(case["out"], abs=1e-14)


def test_dielectric_total_internal_reflection():
    c = K["dielectric_dir"][2]   # leaving glass at a grazing angle: ri*sin > 1 -> reflect
    assert c["reflected"]


@pytest.mark.parametrize("case", K["quantize"])
def test_quantize_oracle(case):
    c = float("nan") if case["c"] == "nan" else case["c"]
    assert oracle.quantize(c) == case["out"]


def test_quantize_known_values():
    q = {c["c"]: c["out"] for c in K["quantize"]}
    assert q[0.25] == 128 and q[0.998] == 255 and q[1.0] == 255 and q[0.0] == 0 and q[-1.0] == 0 and q["nan"] == 0


def test_quantize_product_matches(tmp_path):
    from rtclj import raytracing as R
    vals = [float("nan") if c["c"] == "nan" else c["c"] for c in K["quantize"]]
    rng = np.random.default_rng(0)
    vals += list(rng.uniform(-0.1, 1.2, 2000)) + [np.float32(v) for v in (0.0625, 0.25, 0.998001)]
    lin = np.array(vals, np.float32)
    got = R.write_color(lin)
    exp = np.array([oracle.quantize(float(v)) for v in lin], np.uint8)
    assert np.array_equal(got, exp)


@pytest.mark.parametrize("case", K["camera"], ids=lambda c: c["name"])
def test_camera_oracle_and_product(case):
    args = (case["w"], case["h"], case["vfov"], case["look_from"], case["look_at"], case["vup"],
            case["defocus_angle"], case["focus_dist"])
    got = oracle.camera(*args)
    assert got == pytest.approx(case["out"], rel=1e-14, abs=1e-15)
    from rtclj import raytracing as R
    cam = R.camera(*args)
    assert cam.as_list() == pytest.approx(np.float32(case["out"]).tolist(), rel=0, abs=0)
    assert cam.defocus == (1 if case["defocus_angle"] > 0 else 0)


@pytest.mark.parametrize("case", RNG, ids=lambda c: f"{c['seed']}-{c['pixel']}-{c['sample']}")
def test_rng_contract(case):
    got = oracle.rng_stream(case["seed"], case["pixel"], case["sample"], len(case["draws"]))
    assert got.tolist() == case["draws"]
