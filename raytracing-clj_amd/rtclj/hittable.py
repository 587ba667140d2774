"""Mirror of src/hittable.clj.

The reference's `sphere` (hittable.clj:7-31) returns a map holding a closure
`::hit-fn` with centre and radius captured, so they cannot be inspected.  The
host API carries them as data instead, so a scene can be flattened into the
sphere table the kernel stages in LDS; the hit test itself (hittable.clj:9-31)
runs on the GPU (raytracing-clj_amd/csrc/trace.hip).
"""
from __future__ import annotations


def sphere(center, radius) -> dict:
    """(hittable/sphere center radius) -> a body without material."""
    c = tuple(float(v) for v in center)
    if len(c) != 3:
        raise ValueError("sphere center must have 3 components")
    return {"hittable/kind": "sphere", "hittable/center": c, "hittable/radius": float(radius)}
