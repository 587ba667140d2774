"""The C ABI library (no GPU needed): it loads, exports every function
include/rt.h declares, and its host-side paths and error behaviour hold."""
import ctypes as C
import re
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
HEADER = (ROOT / "include" / "rt.h").read_text()


def declared_functions():
    body = re.sub(r"/\*.*?\*/", "", HEADER, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(rt_[a-z_0-9]+)\s*\(", body, flags=re.M)))


def test_header_declares_the_expected_boundary():
    fns = declared_functions()
    for name in ("rt_render", "rt_quantize", "rt_last_error", "rt_device_count", "rt_camera_setup",
                 "rt_write_ppm", "rt_scene_upload", "rt_scene_free", "rt_launch", "rt_rows_out"):
        assert name in fns


@pytest.mark.parametrize("which", ["product", "diag"])
def test_library_exports_every_declared_symbol(which):
    import rtclj
    from rtclj._lib import SIGNATURES, diag_library_path
    dll = C.CDLL(str(rtclj.library_path if which == "product" else diag_library_path))
    for name in declared_functions():
        assert hasattr(dll, name), f"{name} declared in rt.h but not exported"
        assert name in SIGNATURES, f"{name} has no ctypes signature in rtclj._lib"
    assert set(SIGNATURES) == set(declared_functions())


def test_exports_are_unmangled_c():
    import subprocess
    import rtclj
    out = subprocess.run(["nm", "-D", "--defined-only", str(rtclj.library_path)], capture_output=True, text=True)
    if out.returncode != 0:
        pytest.skip("nm unavailable")
    syms = set(re.findall(r"\b(rt_[a-z_0-9]+)\b", out.stdout))
    assert set(declared_functions()) <= syms
    # -fvisibility=hidden: no C++ functions leak (kernel handles aside)
    funcs = [ln.split()[-1] for ln in out.stdout.splitlines() if " T " in ln]
    assert all(f.startswith("rt_") for f in funcs), [f for f in funcs if not f.startswith("rt_")]


def test_struct_layouts_match_header():
    from rtclj._lib import rt_camera, rt_params, rt_scene, rt_stats
    assert C.sizeof(rt_camera) == 18 * 4 + 4
    assert C.sizeof(rt_scene) == 32
    assert rt_params.seed.offset == 24 and C.sizeof(rt_params) == 56
    assert C.sizeof(rt_stats) == 112 and rt_stats.upload_ms.offset == 40 and rt_stats.d2h_ms.offset == 104


def test_abi_revision_matches_header():
    """rt.h's RT_ABI_VERSION == the binding's == the loaded library's
    (rt_stats grew without a revision the caller could check)."""
    import rtclj
    from rtclj._lib import RT_ABI_VERSION
    hdr = (ROOT / "include" / "rt.h").read_text()
    m = re.search(r"#define RT_ABI_VERSION (\d+)", hdr)
    assert m and int(m.group(1)) == RT_ABI_VERSION == rtclj.lib.rt_abi_version()
    assert f"abi {RT_ABI_VERSION}" in rtclj.lib.rt_version().decode()


def test_flag_values_match_header():
    """rt.h's RT_FLAG_* == the Python binding's == the JNI side's Native.FLAG_*
    (the Clojure ns passes Native's constants)."""
    from rtclj import _lib
    hdr = (ROOT / "include" / "rt.h").read_text()
    flags = {k: int(v) for k, v in re.findall(r"#define RT_FLAG_(\w+) (\d+)", hdr)}
    assert set(flags) == {"SHARDS_ON_DEVICE0", "REALM", "STREAMED", "REJECTION_SAMPLERS"}
    for k, v in flags.items():
        assert getattr(_lib, "RT_FLAG_" + k) == v, k
    java = (ROOT / "raytracing-clj_amd" / "jni" / "src" / "rtclj" / "Native.java").read_text()
    jflags = {k: int(v) for k, v in re.findall(r"static final int FLAG_(\w+) = (\d+);", java)}
    assert jflags == {"REALM": flags["REALM"], "REJECTION_SAMPLERS": flags["REJECTION_SAMPLERS"]}


def test_no_gpu_here_fails_loudly():
    from rtclj import RTError
    from rtclj import raytracing as R
    import rtclj
    if rtclj.lib.rt_device_count() > 0:
        pytest.skip("a GPU is visible")
    cam = R.camera(16, 9, **R.REFERENCE_CAMERA)
    with pytest.raises(RTError) as ei:
        R.render(R.hittables, cam, 16, 9, spp=1)
    assert ei.value.code == -5 and "no GPU" in str(ei.value)
    ds = C.c_void_p()
    sc = R.Scene.from_bodies(R.hittables)
    assert rtclj.lib.rt_scene_upload(0, C.byref(sc.c), C.byref(ds)) < 0


def test_argument_errors():
    import rtclj
    from rtclj._lib import rt_camera, rt_params, rt_scene
    from rtclj import raytracing as R
    lib = rtclj.lib
    cam = R.camera(16, 9, **R.REFERENCE_CAMERA)
    sc = R.Scene.from_bodies(R.hittables)
    out = np.zeros(16 * 9 * 3, np.float32)
    fp = out.ctypes.data_as(C.POINTER(C.c_float))
    p = rt_params(width=16, height=9, row_begin=0, row_end=9, spp=1, max_depth=5)
    assert lib.rt_render(None, C.byref(cam), C.byref(p), fp, out.size, None) == -1
    assert b"NULL" in lib.rt_last_error()
    p_bad = rt_params(width=16, height=9, row_begin=5, row_end=3, spp=1, max_depth=5)
    assert lib.rt_render(C.byref(sc.c), C.byref(cam), C.byref(p_bad), fp, out.size, None) == -1
    p_short = rt_params(width=16, height=9, row_begin=0, row_end=9, spp=1, max_depth=5)
    assert lib.rt_render(C.byref(sc.c), C.byref(cam), C.byref(p_short), fp, 10, None) == -1
    assert b"out_len" in lib.rt_last_error()
    p_flag = rt_params(width=16, height=9, row_begin=0, row_end=9, spp=1, max_depth=5, flags=16)   # (an unknown bit)
    assert lib.rt_render(C.byref(sc.c), C.byref(cam), C.byref(p_flag), fp, out.size, None) == -1
    p_spp = rt_params(width=16, height=9, row_begin=0, row_end=9, spp=(1 << 24) + 1, max_depth=5)
    assert lib.rt_render(C.byref(sc.c), C.byref(cam), C.byref(p_spp), fp, out.size, None) == -1
    p_tiles = rt_params(width=16, height=9, row_begin=0, row_end=9, spp=1, max_depth=5, tile_step=2)
    assert lib.rt_render(C.byref(sc.c), C.byref(cam), C.byref(p_tiles), fp, out.size, None) == -1
    assert lib.rt_camera_setup(0, 9, 20.0, None, None, None, 0.0, 1.0, C.byref(rt_camera())) == -1
    assert lib.rt_quantize(None, None, 4) == -1
    assert lib.rt_quantize(None, None, 0) == 0
    assert lib.rt_quantize_device(None, None, 4, None) == -1
    assert lib.rt_quantize_device(None, None, 0, None) == 0
    b8 = (C.c_uint8 * (16 * 9 * 3))()
    assert lib.rt_render_u8(None, C.byref(cam), C.byref(p), b8, 16 * 9 * 3, None) == -1
    assert lib.rt_render_u8(C.byref(sc.c), C.byref(cam), C.byref(p_short), b8, 10, None) == -1
    assert b"out_len" in lib.rt_last_error()
    assert lib.rt_write_ppm(b"/nonexistent-dir/x.ppm", (C.c_uint8 * 3)(), 1, 1) == -6
    bad = rt_scene(-1, None, None, None)
    assert lib.rt_scene_upload(0, C.byref(bad), C.byref(C.c_void_p())) == -1
    assert lib.rt_last_error() != b""
    assert lib.rt_cache_clear() == 0              # nothing cached without a GPU


def test_rows_out():
    import rtclj
    from rtclj._lib import rt_params
    from rtclj.shard import shard_rows
    lib = rtclj.lib
    for h, tile, step in [(675, 8, 1), (675, 8, 8), (45, 16, 3), (7, 8, 2), (2160, 8, 7)]:
        total = 0
        for first in range(max(step, 1)):
            p = rt_params(width=4, height=h, row_begin=0, row_end=h, row_tile=tile,
                          tile_first=first if step > 1 else 0, tile_step=step if step > 1 else 0)
            n = lib.rt_rows_out(C.byref(p))
            assert n == len(shard_rows(h, tile, p.tile_first, p.tile_step))
            total += n
        assert total == h
    assert lib.rt_rows_out(C.byref(rt_params(width=4, height=10, row_begin=3, row_end=8))) == 5
    assert lib.rt_rows_out(C.byref(rt_params(width=4, height=10, row_begin=3, row_end=11))) == 0
    assert lib.rt_rows_out(None) == 0


def test_version_and_variant():
    import rtclj
    from rtclj._lib import diag_lib
    assert b"gfx950" in rtclj.lib.rt_version()
    # the product build holds the default traversal and its fallbacks only
    for v in (5, 12, 16, 18, 22, 24, 26):
        old = rtclj.lib.rt_set_variant(v)
        assert rtclj.lib.rt_set_variant(old) == v
    for v in (2, 3, 11, 17, 99, -1):
        assert rtclj.lib.rt_set_variant(v) == -1 and b"not in this build" in rtclj.lib.rt_last_error()
    assert rtclj.lib.rt_set_variant(0) == 0
    # the diagnostic build (trace_diag.hip) holds every variant but the
    # dropped while-while traversal (14, 15)
    d = diag_lib()
    for v in [v for v in range(1, 27) if v not in (14, 15, 23, 25)]:
        assert d.rt_set_variant(v) >= 0, v
    for v in (14, 15, 23, 25):
        assert d.rt_set_variant(v) == -1 and b"not in this build" in d.rt_last_error()
    assert d.rt_set_variant(0) == 26
    assert rtclj.lib.rt_resolve_variant(None) == -1
    out4 = (C.c_int * 4)()
    assert rtclj.lib.rt_launch_occupancy(None, None, out4) < 0   # NULL scene: error, no device call


def test_schedule_switch():
    import rtclj
    assert rtclj.lib.rt_set_schedule(1) == 0      # adaptive is the default
    assert rtclj.lib.rt_set_schedule(7) == -1     # rejected
    assert rtclj.lib.rt_set_schedule(0) == 1
