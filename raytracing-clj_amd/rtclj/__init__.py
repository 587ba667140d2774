"""rtclj — host-side mirror of keychera/raytracing-clj's render entry points.

The Clojure namespaces of the reference's hot path map onto modules here:

    hittable   (src/hittable.clj)    sphere constructor, as data
    material   (src/material.clj)    lambertian / metal / dielectric, as data
    raytracing (src/raytracing.clj)  hittables, camera, render, write-color!, -main
    scenes                           RTIOW cover scene (benchmark workload)
    shard      (raytracing.clj:157-171) multi-GPU row-tile / sample-stripe split

Everything below `render` runs on the MI355X through the C ABI in
include/rt.h (librtclj.so, built by raytracing-clj_amd/Makefile).  There is
no CPU fallback: if the library or a GPU is missing, calls raise.
"""
from ._lib import RTError, lib, library_path  # noqa: F401
from . import hittable, material, raytracing, scenes, shard  # noqa: F401

__all__ = ["RTError", "lib", "library_path", "hittable", "material", "raytracing", "scenes", "shard"]
