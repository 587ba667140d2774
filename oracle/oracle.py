"""ctypes wrapper of oracle/_build/liboracle.so — TEST INFRASTRUCTURE ONLY.

Parity status: pinned statistically against the reference's own render
(/root/reference/scene.ppm -> tests/golden/scene_ppm.npz, scene_ppm_stats.json)
and by hand-derived known answers (tests/golden/kats.json).  The reference's
RNG is unseeded java.util.Random, so no bitwise reference image can exist.
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "_build" / "liboracle.so"
MODE_REF64, MODE_MIRROR32, MODE_BOOK64, MODE_REALM64, MODE_REALM32 = 0, 1, 2, 3, 4
# ored into MODE_MIRROR32 / MODE_REALM32: the kernel's loop-free samplers
# (RT_FLAG_DIRECT_SAMPLERS): the unit-sphere draw, the defocus disk, both
DIRECT_SPHERE, DIRECT_DISK = 0x10, 0x20
DIRECT = DIRECT_SPHERE | DIRECT_DISK

_dll = None


def build(force: bool = False) -> Path:
    if force or not LIB.exists() or LIB.stat().st_mtime < (HERE / "rt_oracle.cpp").stat().st_mtime:
        subprocess.run(["make", "-C", str(HERE)], check=True, capture_output=True)
    return LIB


def _lib():
    global _dll
    if _dll is None:
        build()
        d = C.CDLL(str(LIB))
        dp, ip, fp, u64p = C.POINTER(C.c_double), C.POINTER(C.c_int), C.POINTER(C.c_float), C.POINTER(C.c_uint64)
        d.oracle_render.restype = C.c_int
        d.oracle_render.argtypes = [C.c_int, C.c_int, dp, ip, dp, dp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                    C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_int, fp, dp, u64p]
        d.oracle_render_cols.restype = C.c_int
        d.oracle_render_cols.argtypes = [C.c_int, C.c_int, dp, ip, dp, dp, C.c_int, C.c_int, C.c_int, C.c_int,
                                         C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint64,
                                         C.c_int, fp, dp, u64p]
        d.oracle_sphere_hit.restype = C.c_int
        d.oracle_sphere_hit.argtypes = [dp, dp, dp, C.c_double, C.c_double, dp]
        d.oracle_reflect.argtypes = [dp, dp, dp]
        d.oracle_refract.argtypes = [dp, dp, C.c_double, dp]
        d.oracle_reflectance.restype = C.c_double
        d.oracle_reflectance.argtypes = [C.c_double, C.c_double]
        d.oracle_quantize.restype = C.c_int
        d.oracle_quantize.argtypes = [C.c_double]
        d.oracle_camera.argtypes = [C.c_int, C.c_int, C.c_double, dp, dp, dp, C.c_double, C.c_double, dp]
        d.oracle_lambertian_dir.argtypes = [dp, dp, dp]
        d.oracle_metal_dir.restype = C.c_int
        d.oracle_metal_dir.argtypes = [dp, dp, C.c_double, dp, dp]
        d.oracle_dielectric_dir.restype = C.c_int
        d.oracle_dielectric_dir.argtypes = [dp, dp, C.c_int, C.c_double, C.c_double, dp]
        d.oracle_rng_stream.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_int, fp]
        d.oracle_sampler_draws.restype = C.c_int
        d.oracle_sampler_draws.argtypes = [C.c_int, C.c_uint64, C.c_int, fp]
        d.oracle_turn24.argtypes = [C.c_int, C.POINTER(C.c_uint32), C.c_float, fp]
        _dll = d
    return _dll


def _d(a):
    a = np.ascontiguousarray(a, np.float64)
    return a, a.ctypes.data_as(C.POINTER(C.c_double))


def render(mode, sphere, kind, mat, cam, defocus, width, height, spp, max_depth, seed=1, rows=None,
           sample_begin=0, nthreads=0, want64=False, row_step=1, cols=None):
    """Render rows r0, r0+row_step, ... < r1 (default all) -> (float32 (rows,W,3),
    float64 or None, segments, samples).  cols=(c0, c1): only those columns
    of the rows (the others NaN; samples counts the rendered pixels')."""
    r0, r1 = (0, height) if rows is None else rows
    nrows = (r1 - r0 + row_step - 1) // row_step
    sph, sp = _d(np.asarray(sphere, np.float64).reshape(-1, 4))
    mt, mp = _d(np.asarray(mat, np.float64).reshape(-1, 4))
    kd = np.ascontiguousarray(kind, np.int32).reshape(-1)
    cm, cp = _d(np.asarray(cam, np.float64).reshape(18))
    c0, c1 = (0, width) if cols is None else cols
    out = np.full((nrows, width, 3), np.nan, np.float32)
    out64 = np.full((nrows, width, 3), np.nan, np.float64) if want64 else None
    cnt = np.zeros(2, np.uint64)
    rc = _lib().oracle_render_cols(mode, len(kd), sp, kd.ctypes.data_as(C.POINTER(C.c_int)), mp, cp, int(defocus),
                                   width, height, r0, r1, row_step, c0, c1, spp, sample_begin, max_depth, seed,
                                   nthreads, out.ctypes.data_as(C.POINTER(C.c_float)),
                                   out64.ctypes.data_as(C.POINTER(C.c_double)) if want64 else None,
                                   cnt.ctypes.data_as(C.POINTER(C.c_uint64)))
    if rc != 0:
        raise ValueError(f"oracle_render rejected its arguments (rc={rc})")
    return out, out64, int(cnt[0]), int(cnt[1])


def sphere_hit(sphere4, o, d, tmin, tmax):
    s, sp = _d(sphere4)
    oo, op = _d(o)
    dd, dp = _d(d)
    out, outp = _d(np.zeros(9))
    _lib().oracle_sphere_hit(sp, op, dp, tmin, tmax, outp)
    return dict(hit=bool(out[0]), t=out[1], p=out[2:5].tolist(), n=out[5:8].tolist(), front=bool(out[8]))


def reflect(v, n):
    a, ap = _d(v)
    b, bp = _d(n)
    o, op = _d(np.zeros(3))
    _lib().oracle_reflect(ap, bp, op)
    return o.tolist()


def refract(uv, n, eta):
    a, ap = _d(uv)
    b, bp = _d(n)
    o, op = _d(np.zeros(3))
    _lib().oracle_refract(ap, bp, eta, op)
    return o.tolist()


def reflectance(cosine, ri):
    return _lib().oracle_reflectance(cosine, ri)


def quantize(c):
    return _lib().oracle_quantize(c)


def camera(w, h, vfov, look_from, look_at, vup, defocus_angle, focus_dist):
    lf, lp = _d(look_from)
    la, ap = _d(look_at)
    up, upp = _d(vup)
    o, op = _d(np.zeros(18))
    _lib().oracle_camera(w, h, vfov, lp, ap, upp, defocus_angle, focus_dist, op)
    return o


def rng_stream(seed, pixel, sample, n):
    out = np.zeros(n, np.float32)
    _lib().oracle_rng_stream(seed, pixel, sample, n, out.ctypes.data_as(C.POINTER(C.c_float)))
    return out


def lambertian_dir(unit, n):
    a, ap = _d(unit)
    b, bp = _d(n)
    o, op = _d(np.zeros(3))
    _lib().oracle_lambertian_dir(ap, bp, op)
    return o.tolist()


def metal_dir(d, n, fuzz, unit):
    a, ap = _d(d)
    b, bp = _d(n)
    u, up = _d(unit)
    o, op = _d(np.zeros(3))
    ok = _lib().oracle_metal_dir(ap, bp, fuzz, up, op)
    return bool(ok), o.tolist()


def dielectric_dir(d, n, front, eta, xi):
    a, ap = _d(d)
    b, bp = _d(n)
    o, op = _d(np.zeros(3))
    refl = _lib().oracle_dielectric_dir(ap, bp, int(front), eta, xi, op)
    return bool(refl), o.tolist()


SAMPLERS = {"sphere_rejection": 0, "sphere_direct": 1, "disk_rejection": 2, "disk_direct": 3}


def sampler_draws(which, seed, n):
    """n consecutive draws of one sampler from the keyed stream (seed, 0, 0):
    (n, 3) float32 (the disk's z = 0).  which: a SAMPLERS key."""
    out = np.zeros((n, 3), np.float32)
    if _lib().oracle_sampler_draws(SAMPLERS[which], seed, n, out.ctypes.data_as(C.POINTER(C.c_float))) != 0:
        raise ValueError(which)
    return out


def turn24(u, r=1.0):
    """The kernel's (r cos, r sin) of 2 pi u / 2^24 for 24-bit integers u: (n, 2) float32."""
    u = np.ascontiguousarray(u, np.uint32).reshape(-1)
    out = np.zeros((len(u), 2), np.float32)
    _lib().oracle_turn24(len(u), u.ctypes.data_as(C.POINTER(C.c_uint32)), r, out.ctypes.data_as(C.POINTER(C.c_float)))
    return out
