"""ctypes binding of include/rt.h (librtclj.so).

This is the same binding a maintainer would add to the reference's host
(a JNI shim for Clojure); Python uses it for the tests,
bench.py and the Python host API.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

_PKG_ROOT = Path(__file__).resolve().parent.parent          # raytracing-clj_amd/
# RTCLJ_LIBRARY: load another build of the same ABI (A/B of kernel builds)
library_path = Path(os.environ["RTCLJ_LIBRARY"]) if os.environ.get("RTCLJ_LIBRARY") else _PKG_ROOT / "lib" / "librtclj.so"
# the diagnostic build (A/B and statistics kernel variants; same ABI)
diag_library_path = _PKG_ROOT / "lib" / "librtclj_diag.so"

RT_OK, RT_E_ARG, RT_E_MATERIAL, RT_E_TOO_MANY, RT_E_HIP, RT_E_NODEV, RT_E_IO = 0, -1, -2, -3, -4, -5, -6
RT_LAMBERTIAN, RT_METAL, RT_DIELECTRIC, RT_NONE = 0, 1, 2, 3
RT_MAX_SPHERES = 8192
RT_MAX_SPP = 1 << 24
RT_FLAG_SHARDS_ON_DEVICE0 = 1
RT_FLAG_REALM = 2
RT_FLAG_STREAMED = 4
RT_FLAG_REJECTION_SAMPLERS = 8   # vec3a.clj:74-86's rejection loops instead of the loop-free samplers


class RTError(RuntimeError):
    """A negative rt_status from the C ABI, with rt_last_error()'s message."""

    def __init__(self, code: int, message: str):
        super().__init__(f"rt error {code}: {message}")
        self.code = code


class rt_scene(C.Structure):
    _fields_ = [("n", C.c_int), ("sphere", C.POINTER(C.c_float)),
                ("mat_kind", C.POINTER(C.c_int)), ("mat", C.POINTER(C.c_float))]


class rt_camera(C.Structure):
    _fields_ = [("center", C.c_float * 3), ("p00", C.c_float * 3), ("du", C.c_float * 3),
                ("dv", C.c_float * 3), ("disk_u", C.c_float * 3), ("disk_v", C.c_float * 3),
                ("defocus", C.c_int)]

    def as_list(self):
        """18 floats: center, p00, du, dv, disk_u, disk_v (the oracle's camera layout)."""
        out = []
        for f in ("center", "p00", "du", "dv", "disk_u", "disk_v"):
            out.extend(getattr(self, f))
        return out


class rt_params(C.Structure):
    _fields_ = [("width", C.c_int), ("height", C.c_int), ("row_begin", C.c_int), ("row_end", C.c_int),
                ("spp", C.c_int), ("max_depth", C.c_int), ("seed", C.c_uint64), ("sample_begin", C.c_int),
                ("n_devices", C.c_int), ("row_tile", C.c_int), ("tile_first", C.c_int),
                ("tile_step", C.c_int), ("flags", C.c_int)]


class rt_stats(C.Structure):
    _fields_ = [("segments", C.c_uint64), ("samples", C.c_uint64), ("kernel_ms", C.c_double),
                ("total_ms", C.c_double), ("n_devices", C.c_int), ("scene_cached", C.c_int),
                ("upload_ms", C.c_double), ("gather_ms", C.c_double), ("kernel_ms_mean", C.c_double),
                ("setup_ms", C.c_double), ("enqueue_ms", C.c_double), ("wait_ms", C.c_double),
                ("scatter_ms", C.c_double), ("other_ms", C.c_double), ("d2h_ms", C.c_double)]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


# symbol -> (restype, argtypes); every function include/rt.h declares
SIGNATURES = {
    "rt_camera_setup": (C.c_int, [C.c_int, C.c_int, C.c_double, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                  C.POINTER(C.c_double), C.c_double, C.c_double, C.POINTER(rt_camera)]),
    "rt_quantize": (C.c_int, [C.POINTER(C.c_float), C.POINTER(C.c_uint8), C.c_size_t]),
    "rt_write_ppm": (C.c_int, [C.c_char_p, C.POINTER(C.c_uint8), C.c_int, C.c_int]),
    "rt_write_png": (C.c_int, [C.c_char_p, C.POINTER(C.c_uint8), C.c_int, C.c_int]),
    "rt_ppm_to_png": (C.c_int, [C.c_char_p, C.c_char_p]),
    "rt_rows_out": (C.c_int, [C.POINTER(rt_params)]),
    "rt_prepare": (C.c_int, [C.c_int, C.POINTER(C.c_double)]),
    "rt_scene_reference": (C.c_int, [C.POINTER(C.c_float), C.POINTER(C.c_int), C.POINTER(C.c_float), C.c_int]),
    "rt_scene_cover": (C.c_int, [C.c_int, C.c_uint64, C.POINTER(C.c_float), C.POINTER(C.c_int),
                                 C.POINTER(C.c_float), C.c_int]),
    "rt_render": (C.c_int, [C.POINTER(rt_scene), C.POINTER(rt_camera), C.POINTER(rt_params),
                            C.POINTER(C.c_float), C.c_size_t, C.POINTER(rt_stats)]),
    "rt_render_u8": (C.c_int, [C.POINTER(rt_scene), C.POINTER(rt_camera), C.POINTER(rt_params),
                               C.POINTER(C.c_uint8), C.c_size_t, C.POINTER(rt_stats)]),
    "rt_render_submit": (C.c_int, [C.POINTER(rt_scene), C.POINTER(rt_camera), C.POINTER(rt_params),
                                   C.POINTER(C.c_float), C.c_size_t, C.POINTER(C.c_void_p)]),
    "rt_render_submit_u8": (C.c_int, [C.POINTER(rt_scene), C.POINTER(rt_camera), C.POINTER(rt_params),
                                      C.POINTER(C.c_uint8), C.c_size_t, C.POINTER(C.c_void_p)]),
    "rt_render_wait": (C.c_int, [C.c_void_p, C.POINTER(rt_stats)]),
    "rt_cache_clear": (C.c_int, []),
    "rt_scene_upload": (C.c_int, [C.c_int, C.POINTER(rt_scene), C.POINTER(C.c_void_p)]),
    "rt_scene_free": (C.c_int, [C.c_void_p]),
    "rt_launch": (C.c_int, [C.c_void_p, C.POINTER(rt_camera), C.POINTER(rt_params), C.c_void_p,
                            C.c_void_p, C.c_void_p]),
    "rt_quantize_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]),
    "rt_set_variant": (C.c_int, [C.c_int]),
    "rt_resolve_variant": (C.c_int, [C.c_void_p]),
    "rt_launch_occupancy": (C.c_int, [C.c_void_p, C.POINTER(rt_params), C.POINTER(C.c_int)]),
    "rt_set_schedule": (C.c_int, [C.c_int]),
    "rt_debug_stats": (C.c_int, [C.POINTER(C.c_uint64)]),
    "rt_debug_waves": (C.c_int, [C.c_int, C.POINTER(C.c_uint64), C.c_size_t]),
    "rt_steal_stats": (C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64)]),
    "rt_export_stats": (C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64)]),
    "rt_device_count": (C.c_int, []),
    "rt_last_error": (C.c_char_p, []),
    "rt_version": (C.c_char_p, []),
    "rt_abi_version": (C.c_int, []),
}

RT_ABI_VERSION = 3   # include/rt.h; the structures above are this revision's
# functions added within the revision (a build from before them still loads)
ADDITIVE = {"rt_prepare", "rt_render_u8", "rt_quantize_device", "rt_render_submit", "rt_render_submit_u8",
            "rt_render_wait", "rt_export_stats"}


def load(path: Path) -> C.CDLL:
    """Load a build of include/rt.h's ABI with every signature bound.  Local
    binding (RTLD_LOCAL; the library exports only rt_* symbols): the product
    and the diagnostic build can be loaded side by side."""
    if not Path(path).exists():
        raise ImportError(f"{path} is missing: build it with `make -C {_PKG_ROOT}` "
                          "(or __graft_entry__.build()); there is no CPU fallback")
    dll = C.CDLL(str(path), mode=os.RTLD_NOW | os.RTLD_LOCAL)
    for name, (res, args) in SIGNATURES.items():
        if name in ADDITIVE and not hasattr(dll, name):
            continue   # (an older build of the same revision: A/B of library builds)
        fn = getattr(dll, name)
        fn.restype = res
        fn.argtypes = args
    if dll.rt_abi_version() != RT_ABI_VERSION:
        raise ImportError(f"{path}: ABI revision {dll.rt_abi_version()}, this binding is {RT_ABI_VERSION} "
                          "(rebuild the library: make -C raytracing-clj_amd)")
    return dll


lib = load(library_path)
_diag = None


def diag_lib() -> C.CDLL:
    """The diagnostic build (lib/librtclj_diag.so: the A/B and statistics
    kernel variants, rt_set_variant 1-19), loaded on first use."""
    global _diag
    if _diag is None:
        _diag = load(diag_library_path)
    return _diag


def check(code: int) -> int:
    """Raise RTError for a negative status, else return it."""
    if code < 0:
        raise RTError(code, lib.rt_last_error().decode(errors="replace"))
    return code


def fptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def iptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_int))


def u8ptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_uint8))


def dptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))
