"""Mirror of src/material.clj: material constructors as data.

Each returns a map to `merge` with a hittable, as the reference does
(raytracing.clj:65-78).  The scatter functions (material.clj:13-46) run on
the GPU; `reflectance` is mirrored here for the host's own use.
"""
from __future__ import annotations


def lambertian(albedo) -> dict:
    """material.clj:13-19"""
    return {"material/type": "lambertian", "material/albedo": tuple(float(v) for v in albedo)}


def metal(albedo, fuzz) -> dict:
    """material.clj:21-28 (reflects the un-normalised direction, then adds fuzz)."""
    return {"material/type": "metal", "material/albedo": tuple(float(v) for v in albedo),
            "material/fuzz": float(fuzz)}


def dielectric(refraction_index) -> dict:
    """material.clj:34-46"""
    return {"material/type": "dielectric", "material/refraction-index": float(refraction_index)}


def reflectance(cosine: float, refraction_index: float) -> float:
    """Schlick's approximation, material.clj:30-32."""
    r0 = ((1.0 - refraction_index) / (1.0 + refraction_index)) ** 2
    return r0 + (1.0 - r0) * (1.0 - cosine) ** 5
