"""The non-Python host of the C ABI on the GPU: lib/rt_main, the C++ driver
that mirrors `clojure -M:main [spp] [depth]` (src/raytracing.clj:95-177) and
`clojure -M:realm` (src/realm/raytracing.clj:279-359), run as a fresh child
process.  Unlike the pytest process (torch's bundled HIP runtime, loaded first
by conftest.gpu_lib), the child loads /opt/rocm's libamdhip64 through
librtclj.so's own dependency -- the runtime a JVM or C++ host gets.

Its scene.ppm must equal write-color! (rt_quantize) of the oracle's fp32
kernel mirror at the same seed, byte for byte; the PNG it writes decodes to
the same pixels.
"""
from __future__ import annotations

import json
import os
import subprocess
from pathlib import Path

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parent.parent
RT_MAIN = ROOT / "raytracing-clj_amd" / "lib" / "rt_main"


def _child_env():
    env = dict(os.environ)
    env.pop("RTCLJ_LIBRARY", None)
    return env


def _run(args, tmp_path):
    assert RT_MAIN.exists(), "lib/rt_main is not built (make -C raytracing-clj_amd)"
    r = subprocess.run([str(RT_MAIN), *args], cwd=tmp_path, capture_output=True, text=True, timeout=120,
                       env=_child_env())
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    return r.stdout


def _mirror_q8(mode, scene, cam, w, h, spp, depth, seed):
    from rtclj import raytracing as R
    out, _, segs, smp = oracle.render(mode, scene.sphere.astype(np.float64), scene.kind,
                                      scene.mat.astype(np.float64), cam.as_list(), cam.defocus, w, h, spp, depth,
                                      seed=seed, nthreads=min(16, os.cpu_count() or 1))
    return R.write_color(out), segs / smp


def _segs_per_sample(stdout):
    line = [ln for ln in stdout.splitlines() if "segments/sample" in ln][-1]
    return float(line.split(",")[-1].split()[0])


def test_rt_main_reference_scene_equals_mirror(gpu_lib, tmp_path):
    from pngdec import decode
    from rtclj import raytracing as R
    out = _run(["16", "50", "--out", "scene.ppm", "--png", "scene.png", "--gpus", "1"], tmp_path)
    assert out.startswith("config: {:samples-per-px 16, :max-depth 50}")
    img = R.read_ppm(tmp_path / "scene.ppm")
    assert img.shape == (225, 400, 3)
    sc = R.Scene.from_bodies(R.hittables)
    cam = R.camera(400, 225, **R.REFERENCE_CAMERA)
    ref, sps = _mirror_q8(oracle.MODE_MIRROR32 | oracle.DIRECT, sc, cam, 400, 225, 16, 50, seed=1)
    assert np.array_equal(img, ref)
    assert abs(_segs_per_sample(out) - sps) < 1e-3
    assert np.array_equal(decode((tmp_path / "scene.png").read_bytes())[0], img)
    # the frame is quantised on the device (rt_render_u8); rt_render's floats
    # through rt_quantize on the host write the same file
    _run(["16", "50", "--out", "host.ppm", "--gpus", "1", "--host-quantize"], tmp_path)
    assert (tmp_path / "host.ppm").read_bytes() == (tmp_path / "scene.ppm").read_bytes()


def test_rt_main_realm_equals_mirror(gpu_lib, tmp_path):
    from rtclj import raytracing as R
    from rtclj import realm
    _run(["8", "50", "--realm", "--out", "realm.ppm"], tmp_path)
    img = R.read_ppm(tmp_path / "realm.ppm")
    w, h = 400, realm.image_height(400)
    assert img.shape == (h, w, 3) == (224, 400, 3)
    sc = R.Scene.from_bodies(realm.hittables)
    ref, _ = _mirror_q8(oracle.MODE_REALM32 | oracle.DIRECT, sc, realm.camera(w, h), w, h, 8, 50, seed=1)
    assert np.array_equal(img, ref)


def test_rt_main_cover_scene(gpu_lib, tmp_path):
    """The benchmark scene (cover, 484 bodies: the BVH traversal) through the
    C++ host at another width and seed."""
    from rtclj import raytracing as R
    from rtclj import scenes
    from pngdec import decode
    out = _run(["4", "50", "--scene", "cover", "--width", "160", "--seed", "9", "--out", "c.ppm", "--json"], tmp_path)
    img = R.read_ppm(tmp_path / "c.ppm")
    h = R.image_height(160)
    ref, _ = _mirror_q8(oracle.MODE_MIRROR32 | oracle.DIRECT, scenes.cover(11), scenes.cover_camera(160, h), 160, h, 4, 50, seed=9)
    assert np.array_equal(img, ref)
    # like -main's (ppm->png "scene.ppm" "scene.png") (raytracing.clj:176): the
    # PPM is converted beside it by default, inside the timed part
    assert np.array_equal(decode((tmp_path / "c.png").read_bytes())[0], img)
    rec = json.loads(out.strip().splitlines()[-1])
    assert rec["png_ms"] > 0 and rec["process_ms"] >= rec["png_ms"]
    _run(["1", "5", "--scene", "cover", "--width", "64", "--out", "n.ppm", "--no-png"], tmp_path)
    assert (tmp_path / "n.ppm").exists() and not (tmp_path / "n.png").exists()


def test_prepare_and_first_context_streams(gpu_lib):
    """rt_prepare (a device's start-up ahead of the first render) reports its
    four parts and refuses a device that is not there; after rt_cache_clear
    the first rt_render runs on the device's NULL stream and the next call
    moves that context to a stream of its own with the tile order it
    recorded (rt_host.cpp take_ctx): every call renders the same bits, with
    a new scene uploaded between them."""
    import ctypes as C
    import numpy as np
    from rtclj import raytracing as R, scenes
    from rtclj._lib import lib
    ms = (C.c_double * 4)()
    assert lib.rt_prepare(0, ms) == 0 and all(x >= 0.0 for x in ms)
    assert lib.rt_prepare(0, None) == 0
    assert lib.rt_prepare(lib.rt_device_count(), ms) == -5   # RT_E_NODEV
    lib.rt_cache_clear()
    sc = scenes.cover(11)
    w, h = 120, 68
    cam = scenes.cover_camera(w, h)
    frames = [R.render(sc, cam, w, h, spp=6, seed=3) for _ in range(2)]
    other = R.render(R.Scene.from_bodies(R.hittables), R.camera(64, 36, **R.REFERENCE_CAMERA), 64, 36, spp=2)
    frames += [R.render(sc, cam, w, h, spp=6, seed=3) for _ in range(2)]
    assert other.shape == (36, 64, 3)
    assert all(np.array_equal(f, frames[0]) for f in frames[1:])
    lib.rt_cache_clear()
