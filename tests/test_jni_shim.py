"""The JNI shim (raytracing-clj_amd/jni/rtclj_jni.c), compiled unchanged
against tests/jni_mock/: a recording stand-in for the JNI function table (no
JDK in this image).  A logic test of the shim, not JVM verification:

  * argument checks: Java nulls, spheres/mats not 4 x kinds, camera not 18
    floats, an output array shorter than width x height x 3 -> RT_E_ARG and
    a pending RuntimeException("rt error -1: ..."), before any array is copied;
  * every Get<Type>ArrayElements / GetStringUTFChars released exactly once
    with JNI_ABORT (inputs are never written back), on success and on every
    error path;
  * a failed array copy (the JVM's OutOfMemoryError) stays the pending
    exception: no further JNI call but the releases, no RuntimeException over it;
  * the rt error -> exception mapping (rt_render's code and rt_last_error());
  * on the GPU box: the shim's render equals rt_render's pixels bit for bit
    (both flags), and only the frame is copied back (a longer Java array keeps
    its tail: ADVICE r02); renderBytes equals rt_render_u8's bytes;
  * cameraSetup equals rt_camera_setup (-main's camera let block,
    raytracing.clj:105-139); writePpm writes what rt_write_ppm writes.

Replaces compute-pixel + the executor (src/raytracing.clj:141-171) and
ppm->png (src/ppm2png.clj:35-87) for a Clojure host.
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
MOCK_DIR = ROOT / "tests" / "jni_mock"
MOCK_LIB = MOCK_DIR / "_build" / "libjni_mock.so"

RT_E_ARG, RT_E_NODEV, RT_E_IO = -1, -5, -6
VP = C.c_void_p


def _load():
    if not MOCK_LIB.exists():   # built by __graft_entry__.build(); a CPU-side gcc build
        subprocess.run(["make", "-C", str(MOCK_DIR)], check=True, capture_output=True)
    d = C.CDLL(str(MOCK_LIB))
    d.mock_env.restype = VP
    for f in ("mock_float_array", "mock_int_array", "mock_byte_array"):
        getattr(d, f).restype = VP
        getattr(d, f).argtypes = [VP, C.c_int32]
    d.mock_double_array.restype = VP
    d.mock_double_array.argtypes = [VP, C.c_int32]
    d.mock_string.restype = VP
    d.mock_string.argtypes = [C.c_char_p]
    d.mock_data.restype = VP
    d.mock_data.argtypes = [VP]
    d.mock_stats.argtypes = [C.POINTER(C.c_int)]
    d.mock_exception_class.restype = C.c_char_p
    d.mock_exception_message.restype = C.c_char_p
    d.mock_fail_get.argtypes = [C.c_int]
    i32, i64 = C.c_int32, C.c_int64
    d.Java_rtclj_Native_render.restype = i32
    d.Java_rtclj_Native_render.argtypes = [VP, VP, VP, VP, VP, VP, i32, i32, i32, i32, i32, i64, i32, VP]
    d.Java_rtclj_Native_renderWithFlags.restype = i32
    d.Java_rtclj_Native_renderWithFlags.argtypes = [VP, VP, VP, VP, VP, VP, i32, i32, i32, i32, i32, i64, i32, i32,
                                                     VP]
    d.Java_rtclj_Native_renderBytes.restype = i32
    d.Java_rtclj_Native_renderBytes.argtypes = [VP, VP, VP, VP, VP, VP, i32, i32, i32, i32, i32, i64, i32, i32, VP]
    d.Java_rtclj_Native_submitBytes.restype = i64
    d.Java_rtclj_Native_submitBytes.argtypes = [VP, VP, VP, VP, VP, VP, i32, i32, i32, i32, i32, i64, i32, i32]
    d.Java_rtclj_Native_waitBytes.restype = i32
    d.Java_rtclj_Native_waitBytes.argtypes = [VP, VP, i64, VP]
    d.Java_rtclj_Native_cameraSetup.restype = i32
    d.Java_rtclj_Native_cameraSetup.argtypes = [VP, VP, i32, i32, C.c_double, VP, VP, VP, C.c_double, C.c_double, VP]
    d.Java_rtclj_Native_writePpm.restype = i32
    d.Java_rtclj_Native_writePpm.argtypes = [VP, VP, VP, VP, i32, i32]
    d.Java_rtclj_Native_deviceCount.restype = i32
    d.Java_rtclj_Native_deviceCount.argtypes = [VP, VP]
    d.Java_rtclj_Native_writePng.restype = i32
    d.Java_rtclj_Native_writePng.argtypes = [VP, VP, VP, VP, i32, i32]
    d.Java_rtclj_Native_ppmToPng.restype = i32
    d.Java_rtclj_Native_ppmToPng.argtypes = [VP, VP, VP, VP]
    return d


@pytest.fixture()
def jni():
    d = _load()
    d.mock_reset()
    yield d
    d.mock_reset()


def stats(d):
    s = (C.c_int * 8)()
    d.mock_stats(s)
    keys = ("outstanding_pins", "bad_releases", "calls_while_pending", "throws", "region_oob", "set_regions",
            "pending", "gets")
    return dict(zip(keys, list(s)))


def clean(st):
    """The JNI rules held: nothing left pinned, no bad release, nothing called
    with an exception pending, no out-of-bounds region."""
    return st["outstanding_pins"] == 0 and st["bad_releases"] == 0 and st["calls_while_pending"] == 0 \
        and st["region_oob"] == 0


def farr(d, a):
    a = np.ascontiguousarray(a, np.float32)
    return d.mock_float_array(a.ctypes.data, a.size)


def iarr(d, a):
    a = np.ascontiguousarray(a, np.int32)
    return d.mock_int_array(a.ctypes.data, a.size)


def read_f(d, obj, n):
    return np.ctypeslib.as_array(C.cast(d.mock_data(obj), C.POINTER(C.c_float)), (n,)).copy()


def read_b(d, obj, n):
    return np.ctypeslib.as_array(C.cast(d.mock_data(obj), C.POINTER(C.c_uint8)), (n,)).copy()


def barr(d, a):
    a = np.ascontiguousarray(a, np.uint8).view(np.int8)
    return d.mock_byte_array(a.ctypes.data, a.size)


def darr(d, a):
    a = np.ascontiguousarray(a, np.float64)
    return d.mock_double_array(a.ctypes.data, a.size)


def _scene_args(d):
    from rtclj import raytracing as R
    sc = R.Scene.from_bodies(R.hittables)
    w, h = 32, 18
    cam = R.camera(w, h, **R.REFERENCE_CAMERA)
    return sc, cam, w, h, (farr(d, sc.sphere.reshape(-1)), iarr(d, sc.kind), farr(d, sc.mat.reshape(-1)),
                           farr(d, cam.as_list()))


def _render(d, arrays, cam, w, h, out, spp=4, depth=50, seed=1, ngpu=1, flags=None):
    env = d.mock_env()
    sph, knd, mat, c18 = arrays
    if flags is None:
        return d.Java_rtclj_Native_render(env, None, sph, knd, mat, c18, cam.defocus, w, h, spp, depth, seed, ngpu,
                                          out)
    return d.Java_rtclj_Native_renderWithFlags(env, None, sph, knd, mat, c18, cam.defocus, w, h, spp, depth, seed,
                                               ngpu, flags, out)


def test_length_checks_throw_before_any_copy(jni):
    d = jni
    sc, cam, w, h, (sph, knd, mat, c18) = _scene_args(d)
    out = farr(d, np.full(w * h * 3, 7.0))
    env = d.mock_env()
    bad = [
        (farr(d, sc.sphere.reshape(-1)[:-1]), knd, mat, c18),          # spheres not 4 x n
        (sph, knd, farr(d, sc.mat.reshape(-1)[:-4]), c18),             # mats not 4 x n
        (sph, iarr(d, sc.kind[:-1]), mat, c18),                        # kinds shorter
        (sph, knd, mat, farr(d, np.zeros(17))),                        # camera not 18 floats
        (None, knd, mat, c18),                                         # Java null
    ]
    for args in bad:
        d.mock_clear_exception()
        rc = d.Java_rtclj_Native_render(env, None, *args, cam.defocus, w, h, 4, 50, 1, 1, out)
        st = stats(d)
        assert rc == RT_E_ARG and st["pending"] and clean(st) and st["gets"] == 0, st
        assert d.mock_exception_class() == b"java/lang/RuntimeException"
        assert d.mock_exception_message().startswith(b"rt error -1: ")
    # output shorter than the frame; zero / negative sizes
    for ww, hh, n in ((w, h, w * h * 3 - 1), (0, h, 10), (w, -1, 10)):
        d.mock_clear_exception()
        short = farr(d, np.zeros(n))
        rc = d.Java_rtclj_Native_render(env, None, sph, knd, mat, c18, cam.defocus, ww, hh, 4, 50, 1, 1, short)
        st = stats(d)
        assert rc == RT_E_ARG and st["pending"] and clean(st) and st["gets"] == 0, (ww, hh, st)
    assert stats(d)["set_regions"] == 0
    assert np.all(read_f(d, out, w * h * 3) == 7.0)


@pytest.mark.parametrize("k", [1, 2, 3])
def test_failed_copy_keeps_the_out_of_memory_error(jni, k):
    """The k-th array copy fails: the JVM's OutOfMemoryError stays pending, the
    copies made before it are released, no other JNI call follows it."""
    d = jni
    sc, cam, w, h, arrays = _scene_args(d)
    out = farr(d, np.full(w * h * 3, 7.0))
    d.mock_fail_get(k)
    rc = _render(d, arrays, cam, w, h, out)
    st = stats(d)
    assert rc == RT_E_ARG and clean(st) and st["throws"] == 0 and st["gets"] == k - 1, st
    assert d.mock_exception_class() == b"java/lang/OutOfMemoryError"
    assert np.all(read_f(d, out, w * h * 3) == 7.0)


def test_rt_error_maps_to_runtime_exception(jni):
    """A well-formed call: on this machine without a GPU rt_render's RT_E_NODEV
    becomes RuntimeException("rt error -5: <rt_last_error>"), every copy is
    released and the Java output array is untouched; with a GPU it renders."""
    import rtclj
    d = jni
    sc, cam, w, h, arrays = _scene_args(d)
    out = farr(d, np.full(w * h * 3, 7.0))
    rc = _render(d, arrays, cam, w, h, out)
    st = stats(d)
    assert clean(st) and st["gets"] == 3, st
    if rtclj.lib.rt_device_count() > 0:
        assert rc == 0 and not st["pending"] and st["set_regions"] == 1
        return
    assert rc == RT_E_NODEV and st["pending"] and st["throws"] == 1 and st["set_regions"] == 0
    assert d.mock_exception_message().startswith(b"rt error -5: ")
    assert np.all(read_f(d, out, w * h * 3) == 7.0)


def test_render_bytes_checks_and_errors(jni):
    """renderBytes: a byte[] shorter than the frame is an argument error
    before any copy; a well-formed call maps rt_render_u8's status (no GPU
    here: RT_E_NODEV) and leaves the Java array untouched."""
    import rtclj
    d = jni
    env = d.mock_env()
    sc, cam, w, h, (sph, knd, mat, c18) = _scene_args(d)
    short = barr(d, np.full(w * h * 3 - 1, 9))
    rc = d.Java_rtclj_Native_renderBytes(env, None, sph, knd, mat, c18, cam.defocus, w, h, 4, 50, 1, 1, 0, short)
    st = stats(d)
    assert rc == RT_E_ARG and st["pending"] and clean(st) and st["gets"] == 0, st
    d.mock_clear_exception()
    out = barr(d, np.full(w * h * 3, 9))
    rc = d.Java_rtclj_Native_renderBytes(env, None, sph, knd, mat, c18, cam.defocus, w, h, 4, 50, 1, 1, 0, out)
    st = stats(d)
    assert clean(st) and st["gets"] == 3, st
    if rtclj.lib.rt_device_count() > 0:
        assert rc == 0 and st["set_regions"] == 1
        return
    assert rc == RT_E_NODEV and st["pending"] and st["set_regions"] == 0
    assert np.all(read_b(d, out, w * h * 3) == 9)


def test_submit_wait_checks_and_errors(jni):
    """submitBytes / waitBytes (frames in flight): a null input is an
    argument error before any copy; a well-formed submit maps
    rt_render_submit_u8's status (no GPU here: RT_E_NODEV, handle 0) with
    every copy released; waitBytes(0) is an argument error."""
    import rtclj
    d = jni
    env = d.mock_env()
    sc, cam, w, h, (sph, knd, mat, c18) = _scene_args(d)
    hd = d.Java_rtclj_Native_submitBytes(env, None, None, knd, mat, c18, cam.defocus, w, h, 4, 50, 1, 1, 0)
    st = stats(d)
    assert hd == 0 and st["pending"] and clean(st) and st["gets"] == 0, st
    d.mock_clear_exception()
    rc = d.Java_rtclj_Native_waitBytes(env, None, 0, barr(d, np.zeros(w * h * 3)))
    assert rc == RT_E_ARG and stats(d)["pending"]
    d.mock_clear_exception()
    # a handle the shim never gave out (handles are ids of live frames, not
    # pointers: ADVICE r5): an argument error, nothing dereferenced
    for bogus in (1 << 40, -7, 0x7f00deadbeef):
        rc = d.Java_rtclj_Native_waitBytes(env, None, bogus, barr(d, np.zeros(w * h * 3)))
        assert rc == RT_E_ARG and stats(d)["pending"], bogus
        assert b"not a frame in flight" in d.mock_exception_message()
        d.mock_clear_exception()
    hd = d.Java_rtclj_Native_submitBytes(env, None, sph, knd, mat, c18, cam.defocus, w, h, 4, 50, 1, 1, 0)
    st = stats(d)
    assert clean(st) and st["gets"] == 3, st
    if rtclj.lib.rt_device_count() > 0:
        assert hd != 0 and not st["pending"]
        assert d.Java_rtclj_Native_waitBytes(env, None, hd, barr(d, np.zeros(w * h * 3))) == 0
        return
    assert hd == 0 and st["pending"] and d.mock_exception_message().startswith(b"rt error -5: ")


def test_camera_setup_equals_rt_camera_setup(jni):
    from rtclj import raytracing as R
    d = jni
    env = d.mock_env()
    rc_cam = R.REFERENCE_CAMERA
    out = farr(d, np.zeros(18))
    rc = d.Java_rtclj_Native_cameraSetup(env, None, 400, 225, float(rc_cam["vfov"]), darr(d, rc_cam["look_from"]),
                                         darr(d, rc_cam["look_at"]), darr(d, rc_cam["vup"]),
                                         float(rc_cam["defocus_angle"]), float(rc_cam["focus_dist"]), out)
    st = stats(d)
    ref = R.camera(400, 225, **rc_cam)
    assert rc == ref.defocus == 1 and clean(st) and not st["pending"] and st["set_regions"] == 1, st
    assert np.array_equal(read_f(d, out, 18), np.asarray(ref.as_list(), np.float32))
    # wrong lengths, a null, a bad image size (rt_camera_setup's own check)
    for args in ((darr(d, [0, 0]), darr(d, [0, 0, 0]), darr(d, [0, 1, 0]), out),
                 (darr(d, [0, 0, 1]), None, darr(d, [0, 1, 0]), out),
                 (darr(d, [0, 0, 1]), darr(d, [0, 0, 0]), darr(d, [0, 1, 0]), farr(d, np.zeros(17)))):
        d.mock_clear_exception()
        rc = d.Java_rtclj_Native_cameraSetup(env, None, 400, 225, 20.0, *args[:3], 0.0, 1.0, args[3])
        assert rc == RT_E_ARG and d.mock_exception_class() == b"java/lang/RuntimeException"
    d.mock_clear_exception()
    rc = d.Java_rtclj_Native_cameraSetup(env, None, 0, 225, 20.0, darr(d, [0, 0, 1]), darr(d, [0, 0, 0]),
                                         darr(d, [0, 1, 0]), 0.0, 1.0, out)
    assert rc == RT_E_ARG and clean(stats(d))


def test_write_ppm_equals_rt_write_ppm(jni, tmp_path):
    from rtclj import raytracing as R
    d = jni
    env = d.mock_env()
    px = np.random.default_rng(5).integers(0, 256, size=(6, 9, 3), dtype=np.uint8)
    rgb = barr(d, px.reshape(-1))
    rc = d.Java_rtclj_Native_writePpm(env, None, d.mock_string(str(tmp_path / "a.ppm").encode()), rgb, 9, 6)
    st = stats(d)
    assert rc == 0 and clean(st) and not st["pending"], st
    R.write_ppm(tmp_path / "b.ppm", px)
    assert (tmp_path / "a.ppm").read_bytes() == (tmp_path / "b.ppm").read_bytes()
    rc = d.Java_rtclj_Native_writePpm(env, None, d.mock_string(str(tmp_path / "a.ppm").encode()), rgb, 9, 7)
    assert rc == RT_E_ARG and d.mock_exception_message().startswith(b"rt error -1: ")
    d.mock_clear_exception()
    rc = d.Java_rtclj_Native_writePpm(env, None, d.mock_string(str(tmp_path / "no" / "a.ppm").encode()), rgb, 9, 6)
    assert rc == RT_E_IO and clean(stats(d))


def test_device_count_matches_the_library(jni):
    import rtclj
    assert jni.Java_rtclj_Native_deviceCount(jni.mock_env(), None) == rtclj.lib.rt_device_count()


def test_write_png_and_ppm_to_png(jni, tmp_path):
    from pngdec import decode
    d = jni
    env = d.mock_env()
    rng = np.random.default_rng(3)
    w, h = 7, 5
    px = rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8)
    b = px.astype(np.int8).reshape(-1)
    rgb = d.mock_byte_array(b.ctypes.data, b.size)
    path = tmp_path / "a.png"
    rc = d.Java_rtclj_Native_writePng(env, None, d.mock_string(str(path).encode()), rgb, w, h)
    st = stats(d)
    assert rc == 0 and clean(st) and not st["pending"] and st["gets"] == 2, st
    assert np.array_equal(decode(path.read_bytes())[0], px)
    # too short for w x h x 3, then a directory that does not exist
    rc = d.Java_rtclj_Native_writePng(env, None, d.mock_string(str(path).encode()), rgb, w, h + 1)
    assert rc == RT_E_ARG and d.mock_exception_message().startswith(b"rt error -1: ")
    d.mock_clear_exception()
    rc = d.Java_rtclj_Native_writePng(env, None, d.mock_string(str(tmp_path / "no" / "a.png").encode()), rgb, w, h)
    st = stats(d)
    assert rc == RT_E_IO and clean(st) and d.mock_exception_message().startswith(b"rt error -6: "), st
    d.mock_clear_exception()
    # ppm->png: a P3 file round trip, a missing file, a failed string copy
    ppm = tmp_path / "s.ppm"
    ppm.write_text(f"P3\n{w} {h}\n255\n" + "".join(f"{r} {g} {bb}\n" for r, g, bb in px.reshape(-1, 3)))
    dst = tmp_path / "s.png"
    rc = d.Java_rtclj_Native_ppmToPng(env, None, d.mock_string(str(ppm).encode()), d.mock_string(str(dst).encode()))
    assert rc == 0 and np.array_equal(decode(dst.read_bytes())[0], px)
    rc = d.Java_rtclj_Native_ppmToPng(env, None, d.mock_string(str(tmp_path / "none.ppm").encode()),
                                      d.mock_string(str(dst).encode()))
    st = stats(d)
    assert rc == RT_E_IO and st["pending"] and clean(st), st
    d.mock_clear_exception()
    d.mock_fail_get(2)
    rc = d.Java_rtclj_Native_ppmToPng(env, None, d.mock_string(str(ppm).encode()), d.mock_string(str(dst).encode()))
    st = stats(d)
    assert rc == RT_E_ARG and clean(st) and d.mock_exception_class() == b"java/lang/OutOfMemoryError", st


@pytest.mark.gpu
def test_shim_render_equals_rt_render(gpu_lib, jni):
    """Through the shim on the MI355X: the same bits as rt_render for -M:main
    and -M:realm semantics, and a longer Java array keeps its tail."""
    from rtclj import raytracing as R
    from rtclj._lib import RT_FLAG_REALM
    d = jni
    sc, cam, w, h, arrays = _scene_args(d)
    for flags in (None, RT_FLAG_REALM):
        d.mock_reset()
        sc, cam, w, h, arrays = _scene_args(d)
        n = w * h * 3
        out = farr(d, np.full(n + 5, 7.0))
        rc = _render(d, arrays, cam, w, h, out, spp=8, seed=3, flags=flags)
        st = stats(d)
        assert rc == 0 and clean(st) and not st["pending"] and st["set_regions"] == 1, st
        got = read_f(d, out, n + 5)
        ref = R.render(sc, cam, w, h, spp=8, max_depth=50, seed=3, flags=flags or 0)
        assert np.array_equal(got[:n].reshape(h, w, 3), ref)
        assert np.all(got[n:] == 7.0)
        # renderBytes: rt_render_u8's bytes == write-color! of those pixels
        ob = barr(d, np.full(n + 3, 9))
        sph, knd, mat, c18 = arrays
        rc = d.Java_rtclj_Native_renderBytes(d.mock_env(), None, sph, knd, mat, c18, cam.defocus, w, h, 8, 50, 3, 1,
                                             flags or 0, ob)
        st = stats(d)
        assert rc == 0 and clean(st) and not st["pending"], st
        gb = read_b(d, ob, n + 3)
        assert np.array_equal(gb[:n].reshape(h, w, 3), R.write_color(ref))
        assert np.all(gb[n:] == 9)
        # submitBytes / waitBytes: two frames in flight, waited on in reverse;
        # each equals renderBytes' bytes; a short array at the wait throws
        env = d.mock_env()
        h1 = d.Java_rtclj_Native_submitBytes(env, None, sph, knd, mat, c18, cam.defocus, w, h, 8, 50, 3, 1,
                                             flags or 0)
        h2 = d.Java_rtclj_Native_submitBytes(env, None, sph, knd, mat, c18, cam.defocus, w, h, 8, 50, 4, 1,
                                             flags or 0)
        assert h1 and h2 and not stats(d)["pending"]
        o2 = barr(d, np.full(n, 9))
        assert d.Java_rtclj_Native_waitBytes(env, None, h2, o2) == 0
        ref4 = R.render(sc, cam, w, h, spp=8, max_depth=50, seed=4, flags=flags or 0)
        assert np.array_equal(read_b(d, o2, n).reshape(h, w, 3), R.write_color(ref4))
        o1 = barr(d, np.full(n + 3, 9))
        assert d.Java_rtclj_Native_waitBytes(env, None, h1, o1) == 0
        g1 = read_b(d, o1, n + 3)
        assert np.array_equal(g1[:n].reshape(h, w, 3), R.write_color(ref)) and np.all(g1[n:] == 9)
        # waiting on a handle twice: an argument error, not a double free
        assert not stats(d)["pending"]
        assert d.Java_rtclj_Native_waitBytes(env, None, h1, o1) == RT_E_ARG and stats(d)["pending"]
        d.mock_clear_exception()
        h3 = d.Java_rtclj_Native_submitBytes(env, None, sph, knd, mat, c18, cam.defocus, w, h, 8, 50, 3, 1,
                                             flags or 0)
        assert d.Java_rtclj_Native_waitBytes(env, None, h3, barr(d, np.zeros(n - 1))) == RT_E_ARG
        assert stats(d)["pending"] and clean(stats(d))
        d.mock_clear_exception()
