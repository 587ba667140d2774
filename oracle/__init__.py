"""TEST INFRASTRUCTURE ONLY — the parity oracle (see rt_oracle.cpp header).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this.  The product (raytracing-clj_amd/) never does.
"""
from .oracle import MODE_BOOK64, MODE_MIRROR32, MODE_REF64, MODE_REALM64, MODE_REALM32, DIRECT, DIRECT_SPHERE, \
    DIRECT_DISK, build, render, sphere_hit, reflect, refract, \
    reflectance, quantize, camera, rng_stream, lambertian_dir, metal_dir, dielectric_dir, sampler_draws, turn24  # noqa: F401
