"""PNG output (rt_write_png, rt_ppm_to_png = src/ppm2png.clj:35-87's job):
host-only, no GPU.  Decoded by tests/pngdec.py, an independent decoder that
tests/golden/make_golden.py checked against the reference's own scene.png
(its pixels equal scene.ppm's; tests/golden/scene_png.json)."""
import hashlib
import json
from pathlib import Path

import numpy as np
import pytest

import pngdec

G = Path(__file__).parent / "golden"


@pytest.fixture(scope="module")
def R():
    from rtclj import raytracing
    return raytracing


@pytest.mark.parametrize("shape", [(1, 1), (3, 7), (9, 64), (31, 17)])
def test_round_trip(R, tmp_path, shape):
    rng = np.random.default_rng(sum(shape))
    img = rng.integers(0, 256, shape + (3,), dtype=np.uint8)
    p = tmp_path / "a.png"
    R.write_png(p, img)
    px, info = pngdec.decode(p.read_bytes())
    assert (info["width"], info["height"], info["color_type"], info["depth"]) == (shape[1], shape[0], 2, 8)
    assert np.array_equal(px, img)


def test_reference_scene_pixels_round_trip_to_the_reference_png_content(R, tmp_path):
    """scene.ppm's pixels -> our PNG -> decode: the same RGB bytes the
    reference's scene.png decodes to (sha256 recorded by make_golden.py)."""
    rec = json.loads((G / "scene_png.json").read_text())
    assert rec["equals_scene_ppm"] and (rec["width"], rec["height"], rec["color_type"]) == (400, 225, 2)
    pix = np.load(G / "scene_ppm.npz")["pixels"]
    p = tmp_path / "scene.png"
    R.write_png(p, pix)
    px, info = pngdec.decode(p.read_bytes())
    assert hashlib.sha256(px.tobytes()).hexdigest() == rec["decoded_rgb_sha256"]
    assert len(set(info["row_filters"])) > 1          # adaptive filtering at work
    assert p.stat().st_size < pix.size                 # and it compresses


def test_ppm_to_png_equals_write_png(R, tmp_path):
    pix = np.load(G / "scene_ppm.npz")["pixels"][:40, :50]
    R.write_ppm(tmp_path / "s.ppm", pix)
    R.ppm_to_png(tmp_path / "s.ppm", tmp_path / "a.png")
    R.write_png(tmp_path / "b.png", pix)
    assert (tmp_path / "a.png").read_bytes() == (tmp_path / "b.png").read_bytes()


def test_ppm_to_png_accepts_any_whitespace_and_a_lower_max_value(R, tmp_path):
    (tmp_path / "w.ppm").write_text("P3 2 1\n7\n1 2 3   4\n5 6\n")
    R.ppm_to_png(tmp_path / "w.ppm", tmp_path / "w.png")
    px, _ = pngdec.decode((tmp_path / "w.png").read_bytes())
    assert px.tolist() == [[[1, 2, 3], [4, 5, 6]]]     # values as they are (ppm2png does not rescale)


@pytest.mark.parametrize("text,code", [
    ("P6\n1 1\n255\n0 0 0\n", -1),        # not P3 (ppm2png: "bad header")
    ("P3\n1 1\n256\n0 0 0\n", -1),        # colour size > 255
    ("P3\n0 1\n255\n", -1),               # bad dimensions
    ("P3\n2 1\n255\n0 0 0\n1 1\n", -1),   # truncated pixel data
    ("P3\n1 1\n9\n10 0 0\n", -1),         # value above the maximum
    ("P3\n1 1\n255\n0 x 0\n", -1),        # not a number
    ("P3\n1 1\n255\n0 0 99999999999999999999999\n", -1),   # a 23-digit token (stops at the tenth digit)
    ("P3\n1234567890 1\n255\n0 0 0\n", -1),                # a 10-digit dimension
])
def test_ppm_to_png_rejects_malformed_input(R, tmp_path, text, code):
    from rtclj import RTError
    (tmp_path / "bad.ppm").write_text(text)
    with pytest.raises(RTError) as e:
        R.ppm_to_png(tmp_path / "bad.ppm", tmp_path / "bad.png")
    assert e.value.code == code
    assert not (tmp_path / "bad.png").exists()


def test_io_errors(R, tmp_path):
    from rtclj import RTError
    with pytest.raises(RTError) as e:
        R.ppm_to_png(tmp_path / "missing.ppm", tmp_path / "x.png")
    assert e.value.code == -6
    with pytest.raises(RTError) as e:
        R.write_png(tmp_path / "no" / "dir.png", np.zeros((2, 2, 3), np.uint8))
    assert e.value.code == -6


def test_ppm_to_png_parses_a_large_frame_in_spans(R, tmp_path):
    """A frame whose text spans several parse spans (~1 MB each): the PNG
    equals rt_write_png's of the same pixels, and text after the last pixel
    is ignored (as a sequential parse ignores it)."""
    rng = np.random.default_rng(7)
    pix = rng.integers(0, 256, (450, 800, 3), dtype=np.uint8)
    R.write_ppm(tmp_path / "s.ppm", pix)
    assert (tmp_path / "s.ppm").stat().st_size > 3 << 20
    R.ppm_to_png(tmp_path / "s.ppm", tmp_path / "a.png")
    R.write_png(tmp_path / "b.png", pix)
    assert (tmp_path / "a.png").read_bytes() == (tmp_path / "b.png").read_bytes()
    with open(tmp_path / "s.ppm", "a") as f:
        f.write("trailing x 999 words\n")
    R.ppm_to_png(tmp_path / "s.ppm", tmp_path / "c.png")
    assert (tmp_path / "c.png").read_bytes() == (tmp_path / "b.png").read_bytes()


@pytest.mark.parametrize("bad_pixel,token", [(3, "x"), (200_000, "256"), (359_999, "1234567890")])
def test_ppm_to_png_reports_the_first_bad_pixel_in_any_span(R, tmp_path, bad_pixel, token):
    """A bad token early, in a middle span and at the last pixel: the error
    names the pixel a sequential parse stops at."""
    from rtclj import RTError
    rng = np.random.default_rng(bad_pixel)
    pix = rng.integers(0, 256, (450, 800, 3), dtype=np.uint8)
    lines = ["P3", "800 450", "255"] + [" ".join(map(str, p)) for p in pix.reshape(-1, 3)]
    lines[3 + bad_pixel] = f"1 {token} 2"
    later = min(bad_pixel + 70_000, 359_999)
    if later > bad_pixel:
        lines[3 + later] = "0 -1 0"                     # a later bad token, in a later span: not the one named
    (tmp_path / "bad.ppm").write_text("\n".join(lines) + "\n0 0 q\n")
    with pytest.raises(RTError) as e:
        R.ppm_to_png(tmp_path / "bad.ppm", tmp_path / "bad.png")
    assert e.value.code == -1
    assert f"bad pixel value at {bad_pixel}" in str(e.value)
    assert not (tmp_path / "bad.png").exists()
