"""Scene builders beyond the reference's five bodies.

The RTIOW cover scene is the workload BASELINE.json's configs name; the
reference has no such scene, so it is defined here (book §14)
and generated deterministically by rt_scene_cover in the C library.
"""
from __future__ import annotations

import numpy as np

from ._lib import RT_MAX_SPHERES, fptr, iptr, lib
from .raytracing import Scene, camera

COVER_CAMERA = dict(vfov=20.0, look_from=(13.0, 2.0, 3.0), look_at=(0.0, 0.0, 0.0), vup=(0.0, 1.0, 0.0),
                    defocus_angle=0.6, focus_dist=10.0)


def cover(grid: int = 11, seed: int = 42) -> Scene:
    """RTIOW §14 cover scene: grid 11 -> ~485 bodies, grid 16 -> ~1000."""
    n = lib.rt_scene_cover(grid, seed, None, None, None, 0)
    if n > RT_MAX_SPHERES:
        raise ValueError(f"cover grid {grid}: {n} bodies > RT_MAX_SPHERES")
    sph = np.zeros((n, 4), np.float32)
    kind = np.zeros(n, np.int32)
    mat = np.zeros((n, 4), np.float32)
    got = lib.rt_scene_cover(grid, seed, fptr(sph), iptr(kind), fptr(mat), n)
    assert got == n
    return Scene(sph, kind, mat)


def reference() -> Scene:
    """The reference's five bodies via the C builder (same as raytracing.hittables)."""
    n = lib.rt_scene_reference(None, None, None, 0)
    sph = np.zeros((n, 4), np.float32)
    kind = np.zeros(n, np.int32)
    mat = np.zeros((n, 4), np.float32)
    lib.rt_scene_reference(fptr(sph), iptr(kind), fptr(mat), n)
    return Scene(sph, kind, mat)


def cover_camera(width: int, height: int):
    return camera(width, height, **COVER_CAMERA)
