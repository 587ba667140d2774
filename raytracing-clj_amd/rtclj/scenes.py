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


def cover(grid: int = 11, seed: int = 42, max_bodies: int | None = None) -> Scene:
    """RTIOW §14 cover scene: grid 11 -> 484 bodies (C1, C2), grid 16 -> 1025.

    max_bodies truncates the random field: the ground, the field's first
    max_bodies - 4 bodies in generation order, and the three r = 1 bodies.
    C4's "1000-sphere scene" (BASELINE.json configs[4]) is cover(16,
    max_bodies=1000), SURVEY.md §8d's "or truncate to exactly 1000"."""
    n = lib.rt_scene_cover(grid, seed, None, None, None, 0)
    if max_bodies is None and n > RT_MAX_SPHERES:
        raise ValueError(f"cover grid {grid}: {n} bodies > RT_MAX_SPHERES")
    sph = np.zeros((n, 4), np.float32)
    kind = np.zeros(n, np.int32)
    mat = np.zeros((n, 4), np.float32)
    got = lib.rt_scene_cover(grid, seed, fptr(sph), iptr(kind), fptr(mat), n)
    assert got == n
    if max_bodies is not None and max_bodies < n:
        if max_bodies < 4:
            raise ValueError("max_bodies < 4: the ground and the three r = 1 bodies are kept")
        keep = np.r_[0:max_bodies - 3, n - 3:n]
        sph, kind, mat = sph[keep], kind[keep], mat[keep]
    return Scene(sph, kind, mat)


C4_BODIES = 1000


def cover_c4() -> Scene:
    """BASELINE.json configs[4]'s 1000-sphere scene: cover(16) truncated."""
    return cover(16, 42, max_bodies=C4_BODIES)


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
