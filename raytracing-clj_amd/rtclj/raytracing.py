"""Mirror of src/raytracing.clj — the reference's host entry points.

    hittables       raytracing.clj:63-78   the five-body scene, as data
    camera          raytracing.clj:105-139 basis/viewport (rt_camera_setup)
    render          raytracing.clj:141-171 compute-pixel over every pixel,
                                           on the GPU(s) via rt_render
    write_color     raytracing.clj:19-26   gamma-2, clamp 0.999, x256
    write_ppm       raytracing.clj:172-175 P3, one pixel per line
    write_png,      ppm2png.clj:35-87      8-bit RGB PNG of the same pixels
      ppm_to_png
    main            raytracing.clj:95-177  `clojure -M:main [spp] [depth]`

The per-pixel loop (compute-pixel -> ray-color -> hit-anything -> hit-fn /
scatter-fn) is the hand-written gfx950 kernel behind include/rt.h.  There is
no CPU path here: without the library or a GPU, render raises RTError.
"""
from __future__ import annotations

import ctypes as C
import sys
import time
from fractions import Fraction

import numpy as np

from . import hittable, material
from ._lib import (RT_DIELECTRIC, RT_LAMBERTIAN, RT_METAL, RT_NONE, RTError, check, dptr, fptr, iptr, lib,
                   rt_camera, rt_params, rt_scene, rt_stats, u8ptr)

# ---- scene (raytracing.clj:63-78) --------------------------------------------
hittables = [
    {**hittable.sphere((0.0, -100.5, -1.0), 100.0), **material.lambertian((0.8, 0.8, 0.0))},   # ground
    {**hittable.sphere((0.0, 0.0, -1.2), 0.5), **material.lambertian((0.1, 0.2, 0.5))},       # center
    {**hittable.sphere((-1.0, 0.0, -1.0), 0.5), **material.dielectric(1.5)},                  # left
    {**hittable.sphere((-1.0, 0.0, -1.0), 0.4), **material.dielectric(1.00 / 1.5)},          # bubble
    {**hittable.sphere((1.0, 0.0, -1.0), 0.5), **material.metal((0.8, 0.6, 0.2), 1.0)},       # right
]

# camera constants of -main (raytracing.clj:105-115)
ASPECT = Fraction(16, 9)
REFERENCE_CAMERA = dict(vfov=20.0, look_from=(-2.0, 2.0, 1.0), look_at=(0.0, 0.0, -1.0), vup=(0.0, 1.0, 0.0),
                        defocus_angle=10.0, focus_dist=3.4)


def image_height(image_width: int, aspect=ASPECT) -> int:
    """(int (/ image-width aspect-ratio)) with Clojure's exact ratio (:105-107)."""
    return int(Fraction(image_width) / Fraction(aspect))


def flatten(bodies):
    """Bodies (merged hittable+material maps) -> the rt_scene arrays.

    Returns (sphere float32[n,4], kind int32[n], mat float32[n,4]).  A body
    with no material is kept (it renders black, as ray-color does when the hit
    body has no ::scatter-fn, raytracing.clj:49-54)."""
    n = len(bodies)
    sph = np.zeros((n, 4), np.float32)
    kind = np.zeros(n, np.int32)
    mat = np.zeros((n, 4), np.float32)
    for i, b in enumerate(bodies):
        if b.get("hittable/kind") != "sphere":
            raise ValueError(f"body {i}: only spheres are supported (hittable.clj:7)")
        sph[i, :3] = b["hittable/center"]
        sph[i, 3] = b["hittable/radius"]
        t = b.get("material/type")
        if t == "lambertian":
            kind[i] = RT_LAMBERTIAN
            mat[i, :3] = b["material/albedo"]
        elif t == "metal":
            kind[i] = RT_METAL
            mat[i, :3] = b["material/albedo"]
            mat[i, 3] = b["material/fuzz"]
        elif t == "dielectric":
            kind[i] = RT_DIELECTRIC
            mat[i, 3] = b["material/refraction-index"]
        elif t is None:
            kind[i] = RT_NONE
        else:
            raise ValueError(f"body {i}: unsupported material {t!r}")
    return sph, kind, mat


def flatten64(bodies):
    """As flatten, in float64 (the oracle's reference-semantics input)."""
    sph, kind, mat = flatten(bodies)
    sph64 = np.array([[*b["hittable/center"], b["hittable/radius"]] for b in bodies], np.float64).reshape(-1, 4)
    mat64 = np.zeros((len(bodies), 4), np.float64)
    for i, b in enumerate(bodies):
        if "material/albedo" in b:
            mat64[i, :3] = b["material/albedo"]
        mat64[i, 3] = b.get("material/fuzz", b.get("material/refraction-index", 0.0))
    return sph64, kind, mat64


class Scene:
    """Flattened scene arrays plus the rt_scene struct pointing at them."""

    def __init__(self, sphere, kind, mat):
        self.sphere = np.ascontiguousarray(sphere, np.float32).reshape(-1, 4)
        self.kind = np.ascontiguousarray(kind, np.int32).reshape(-1)
        self.mat = np.ascontiguousarray(mat, np.float32).reshape(-1, 4)
        if not (len(self.sphere) == len(self.kind) == len(self.mat)):
            raise ValueError("scene arrays disagree in length")
        self.c = rt_scene(len(self.kind), fptr(self.sphere), iptr(self.kind), fptr(self.mat))

    @classmethod
    def from_bodies(cls, bodies):
        return cls(*flatten(bodies))

    def __len__(self):
        return len(self.kind)


def camera(image_width, image_h, vfov, look_from, look_at, vup, defocus_angle, focus_dist) -> rt_camera:
    """Camera values of -main (raytracing.clj:117-139), computed in double."""
    cam = rt_camera()
    d3 = C.c_double * 3
    check(lib.rt_camera_setup(int(image_width), int(image_h), float(vfov), d3(*look_from), d3(*look_at),
                              d3(*vup), float(defocus_angle), float(focus_dist), C.byref(cam)))
    return cam


def _frame_args(scene, width, height, spp, max_depth, seed, n_devices, rows, sample_begin, row_tile, flags, out, u8):
    if not isinstance(scene, Scene):
        scene = Scene.from_bodies(scene)
    r0, r1 = (0, height) if rows is None else rows
    p = rt_params(width=width, height=height, row_begin=r0, row_end=r1, spp=spp, max_depth=max_depth,
                  seed=seed, sample_begin=sample_begin, n_devices=n_devices, row_tile=row_tile, flags=flags)
    shape = (max(r1 - r0, 0), width, 3)
    dt = np.uint8 if u8 else np.float32
    if out is None:
        out = np.empty(shape, dt)
    elif out.shape != shape or out.dtype != dt or not out.flags.c_contiguous:
        raise ValueError(f"render: out must be C-contiguous {np.dtype(dt).name} {shape}")
    return scene, p, out


def render(scene, cam: rt_camera, width: int, height: int, spp: int = 100, max_depth: int = 50, seed: int = 1,
           n_devices: int = 0, rows=None, sample_begin: int = 0, row_tile: int = 8, stats: dict | None = None,
           flags: int = 0, library=None, out=None, u8: bool = False):
    """compute-pixel for every pixel of rows [r0, r1) (default: all), on the GPU.

    Returns float32 (rows, width, 3) linear RGB, each pixel the mean of its spp
    samples (raytracing.clj:155).  `scene` is a Scene or a list of bodies.
    `library`: another loaded build of the ABI (rtclj._lib.diag_lib()).
    `out`: a C-contiguous float32 (rows, width, 3) array to render into (a
    renderer drawing frames reuses its framebuffer; a fresh 10 MB array's
    pages are first touched by the copy into it).
    `u8`: return write-color!'s bytes instead (rt_render_u8: the frame is
    quantised on the device; bit-identical to write_color(render(...)))."""
    dll = library if library is not None else lib
    scene, p, out = _frame_args(scene, width, height, spp, max_depth, seed, n_devices, rows, sample_begin,
                                row_tile, flags, out, u8)
    st = rt_stats()
    if u8:
        code = dll.rt_render_u8(C.byref(scene.c), C.byref(cam), C.byref(p), u8ptr(out), out.size, C.byref(st))
    else:
        code = dll.rt_render(C.byref(scene.c), C.byref(cam), C.byref(p), fptr(out), out.size, C.byref(st))
    if code < 0:
        raise RTError(code, dll.rt_last_error().decode(errors="replace"))
    if stats is not None:
        stats.update(st.as_dict())
    return out


class Frame:
    """A frame in flight (rt_render_submit): wait() blocks until its rows are
    in the array and returns it.  Holds the scene, parameters and array until
    then; a frame dropped unwaited is waited on by its finaliser."""

    def __init__(self, dll, handle, keep, out):
        self._dll, self._h, self._keep, self.out = dll, handle, keep, out

    def wait(self, stats: dict | None = None):
        if self._h is None:
            raise RuntimeError("Frame.wait: already waited on")
        st = rt_stats()
        h, self._h = self._h, None
        code = self._dll.rt_render_wait(h, C.byref(st))
        self._keep = None
        if code < 0:
            raise RTError(code, self._dll.rt_last_error().decode(errors="replace"))
        if stats is not None:
            stats.update(st.as_dict())
        return self.out

    def __del__(self):
        if getattr(self, "_h", None) is not None:
            self._dll.rt_render_wait(self._h, None)


def render_async(scene, cam: rt_camera, width: int, height: int, spp: int = 100, max_depth: int = 50,
                 seed: int = 1, n_devices: int = 0, rows=None, sample_begin: int = 0, row_tile: int = 8,
                 flags: int = 0, library=None, out=None, u8: bool = False) -> Frame:
    """render(...) without waiting (rt_render_submit): the devices start on
    the frame and the call returns a Frame; several frames submitted before
    the first is waited on run concurrently.  The bits are render's."""
    dll = library if library is not None else lib
    scene, p, out = _frame_args(scene, width, height, spp, max_depth, seed, n_devices, rows, sample_begin,
                                row_tile, flags, out, u8)
    h = C.c_void_p()
    if u8:
        code = dll.rt_render_submit_u8(C.byref(scene.c), C.byref(cam), C.byref(p), u8ptr(out), out.size,
                                       C.byref(h))
    else:
        code = dll.rt_render_submit(C.byref(scene.c), C.byref(cam), C.byref(p), fptr(out), out.size, C.byref(h))
    if code < 0:
        raise RTError(code, dll.rt_last_error().decode(errors="replace"))
    return Frame(dll, h, (scene, cam, p), out)


def write_color(lin) -> np.ndarray:
    """write-color!'s channel mapping (raytracing.clj:19-26) -> uint8 array."""
    lin = np.ascontiguousarray(lin, np.float32)
    out = np.empty(lin.shape, np.uint8)
    check(lib.rt_quantize(fptr(lin), u8ptr(out), lin.size))
    return out


def write_ppm(path, rgb8) -> None:
    """PPM P3 as -main writes it (raytracing.clj:172-175)."""
    rgb8 = np.ascontiguousarray(rgb8, np.uint8)
    h, w = rgb8.shape[:2]
    check(lib.rt_write_ppm(str(path).encode(), u8ptr(rgb8), w, h))


def write_png(path, rgb8) -> None:
    """The same pixels as write_ppm, as an 8-bit RGB PNG (rt_write_png; the
    format src/ppm2png.clj produces)."""
    rgb8 = np.ascontiguousarray(rgb8, np.uint8)
    h, w = rgb8.shape[:2]
    check(lib.rt_write_png(str(path).encode(), u8ptr(rgb8), w, h))


def ppm_to_png(src, dst) -> None:
    """ppm2png/ppm->png (src/ppm2png.clj:35-87) via rt_ppm_to_png."""
    check(lib.rt_ppm_to_png(str(src).encode(), str(dst).encode()))


def read_ppm(path) -> np.ndarray:
    """Parse a P3 file (as written by write_ppm or the reference) -> uint8 (H, W, 3)."""
    tok = open(path).read().split()
    if tok[0] != "P3":
        raise ValueError(f"{path}: not a P3 PPM")
    w, h, mx = int(tok[1]), int(tok[2]), int(tok[3])
    if mx != 255:
        raise ValueError(f"{path}: max value {mx} != 255")
    return np.array(tok[4:4 + w * h * 3], np.int64).astype(np.uint8).reshape(h, w, 3)


def main(*args, out_path="scene.ppm", seed: int = 1, n_devices: int = 0, flags: int = 0) -> np.ndarray:
    """-main [spp] [depth] (raytracing.clj:95-177): render the five-body scene
    at 400 x 225 and write `out_path` (PPM P3).  Returns the uint8 image.
    flags: rt_params.flags (e.g. RT_FLAG_REJECTION_SAMPLERS)."""
    spp = int(args[0]) if len(args) > 0 and args[0] is not None else 100
    max_depth = int(args[1]) if len(args) > 1 and args[1] is not None else 50
    print("config:", {"samples-per-px": spp, "max-depth": max_depth})
    t0 = time.perf_counter()
    width = 400
    height = image_height(width)
    cam = camera(width, height, **REFERENCE_CAMERA)
    lin = render(hittables, cam, width, height, spp, max_depth, seed=seed, n_devices=n_devices, flags=flags)
    rgb = write_color(lin)
    write_ppm(out_path, rgb)
    print(f'"Elapsed time: {(time.perf_counter() - t0) * 1e3:.3f} msecs"')
    return rgb


if __name__ == "__main__":  # python -m rtclj.raytracing [spp] [depth]
    try:
        main(*sys.argv[1:3])
    except RTError as e:
        sys.exit(str(e))


__all__ = ["hittables", "REFERENCE_CAMERA", "image_height", "flatten", "flatten64", "Scene", "camera", "render",
           "write_color", "write_ppm", "write_png", "ppm_to_png", "read_ppm", "main", "dptr"]
