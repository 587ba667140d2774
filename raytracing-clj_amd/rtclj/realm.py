"""Mirror of src/realm/raytracing.clj — the reference's second namespace
(`clojure -M:realm`), the same path under slightly different semantics.

    hittables   realm/raytracing.clj:307-317   the five bodies, in realm's order
                                               (centre first: it wins ties)
    camera      realm/raytracing.clj:285-300   no defocus, focal length
                                               |look-from - look-at|
    render      realm/raytracing.clj:320-357   rt_render with RT_FLAG_REALM:
                lambertian without the near-zero fallback (:137-143), dielectric
                without Schlick reflectance (:158-177), pixel = sum * (1/spp)
    main        realm/raytracing.clj:279-359   400 x 224, 100 spp, depth 50 ->
                scene-realm.ppm

The per-pixel loop is the same gfx950 kernel as rtclj.raytracing's, with the
realm flag; there is no CPU path.
"""
from __future__ import annotations

import math
import sys
import time
from decimal import Context, Decimal

import numpy as np

from . import hittable, material
from . import raytracing as R
from ._lib import RT_FLAG_REALM, RTError

# realm/raytracing.clj:307-317 (the commented-out R spheres are not rendered)
hittables = [
    {**hittable.sphere((0.0, 0.0, -1.2), 0.5), **material.lambertian((0.1, 0.2, 0.5))},       # centre
    {**hittable.sphere((0.0, -100.5, -1.0), 100.0), **material.lambertian((0.8, 0.8, 0.0))},  # ground
    {**hittable.sphere((-1.0, 0.0, -1.0), 0.5), **material.dielectric(1.50)},                 # left
    {**hittable.sphere((-1.0, 0.0, -1.0), 0.4), **material.dielectric(1.0 / 1.50)},           # bubble
    {**hittable.sphere((1.0, 0.0, -1.0), 0.5), **material.metal((0.8, 0.6, 0.2), 1.0)},       # right
]

LOOK_FROM = (-2.0, 2.0, 1.0)
LOOK_AT = (0.0, 0.0, -1.0)
VUP = (0.0, 1.0, 0.0)
VFOV = 20.0
IMAGE_WIDTH = 400
SAMPLES_PER_PX = 100
MAX_DEPTH = 50


# ^double on the var holding the Ratio 16/9 casts it with Ratio.doubleValue,
# which rounds through a 16-digit decimal: 1.777777777777778, slightly above
# 16/9 (realm/raytracing.clj:20-22)
ASPECT_DOUBLE = float(Context(prec=16).divide(Decimal(16), Decimal(9)))


def image_height(image_width: int) -> int:
    """(int (/ ^double image-width ^double aspect-ratio)) -- a double division
    by 1.777777777777778 (realm/raytracing.clj:20-22): 400 -> 224, as
    scene-realm.ppm is, where -main's exact ratio gives 225."""
    return int(float(image_width) / ASPECT_DOUBLE)


def focal_length() -> float:
    """(.length (look-from - look-at)) (realm/raytracing.clj:291-292)."""
    return math.sqrt(sum((a - b) ** 2 for a, b in zip(LOOK_FROM, LOOK_AT)))


def camera(image_width: int, image_h: int):
    """realm's camera: -main's basis/viewport with the focal length as the
    focus distance and no defocus disk (realm/raytracing.clj:285-300, 320-337)."""
    return R.camera(image_width, image_h, VFOV, LOOK_FROM, LOOK_AT, VUP, 0.0, focal_length())


def render(scene, cam, width: int, height: int, spp: int = SAMPLES_PER_PX, max_depth: int = MAX_DEPTH,
           seed: int = 1, n_devices: int = 0, rows=None, stats: dict | None = None, flags: int = 0, library=None):
    """The realm loop (realm/raytracing.clj:339-357) for every pixel, on the GPU."""
    return R.render(scene, cam, width, height, spp, max_depth, seed=seed, n_devices=n_devices, rows=rows,
                    stats=stats, flags=flags | RT_FLAG_REALM, library=library)


def main(out_path="scene-realm.ppm", seed: int = 1, n_devices: int = 0, png_path=None) -> np.ndarray:
    """realm.raytracing/-main: 400 x 224, 100 spp, depth 50 -> scene-realm.ppm
    (P3, one pixel per line).  png_path: also write a PNG (rt_write_png)."""
    t0 = time.perf_counter()
    width = IMAGE_WIDTH
    height = image_height(width)
    lin = render(hittables, camera(width, height), width, height, seed=seed, n_devices=n_devices)
    rgb = R.write_color(lin)
    R.write_ppm(out_path, rgb)
    if png_path:
        R.write_png(png_path, rgb)
    print(f'"Elapsed time: {(time.perf_counter() - t0) * 1e3:.3f} msecs"')
    return rgb


if __name__ == "__main__":  # python -m rtclj.realm
    try:
        main()
    except RTError as e:
        sys.exit(str(e))


__all__ = ["hittables", "image_height", "focal_length", "camera", "render", "main"]
