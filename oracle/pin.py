"""Statistics of the fp64 reference-semantics pin -- TEST INFRASTRUCTURE ONLY
(tests/, __graft_entry__.smoke(), bench.py's cpu_baseline leg).

An image rendered with the reference's semantics in double (oracle
MODE_REF64, the Clojure path restated) against one rendered under the
kernel's fp32 contract (the GPU, or MODE_MIRROR32) from the same keyed RNG
stream: the paths agree except where an fp32 decision flips, so the images
agree far inside the reference fixture's statistical noise.  The bounds
(`within`) are written in tests/test_oracle_cover_pin.py's docstring with
the values they were measured at.
"""
from __future__ import annotations

import numpy as np


def q8(lin):
    """write-color! (raytracing.clj:19-26) as int64, vectorised."""
    g = np.where(lin > 0, np.sqrt(np.maximum(np.asarray(lin, np.float64), 0)), 0.0)
    return (256 * np.clip(g, 0.0, 0.999)).astype(np.int64)


def blocks(img, by, bx=16):
    """by x bx grid of block means (SURVEY.md §8c's grid definition)."""
    h, w = img.shape[:2]
    return np.array([[img[y * h // by:(y + 1) * h // by, x * w // bx:(x + 1) * w // bx].reshape(-1, 3).mean(0)
                      for x in range(bx)] for y in range(by)])


def compare(a64, seg_per_sample64, a32, seg_per_sample32, by):
    """fp64-semantics image vs fp32-contract image (same rows, same seed)."""
    d = np.abs(np.asarray(a64, np.float64) - np.asarray(a32, np.float64))
    A, B = q8(a64), q8(a32)
    bd = np.abs(blocks(A.astype(np.float64), by) - blocks(B.astype(np.float64), by))
    return {"seg_rel": abs(seg_per_sample32 - seg_per_sample64) / seg_per_sample64,
            "lin_mean": float(d.mean()), "lin_max": float(d.max()),
            "px8_mean": float(np.abs(A - B).mean()), "px8_max": int(np.abs(A - B).max()),
            "px8_off_gt1": float((np.abs(A - B) > 1).mean()),
            "block_mean": float(bd.mean()), "block_max": float(bd.max())}


# same draws (the fp32 contract with the reference's rejection samplers,
# RT_FLAG_REJECTION_SAMPLERS / MODE_MIRROR32): the paths agree except where an
# fp32 decision flips, so per-pixel bounds hold
BOUNDS = {"seg_rel": 2e-3, "lin_mean": 5e-4, "px8_mean": 0.25, "px8_off_gt1": 0.02, "block_mean": 0.25,
          "block_max": 2.5}
# independent draws (the kernel's default loop-free samplers draw the same
# distributions from a different number of uniforms, so every path after the
# first scatter differs): the bounds SURVEY.md §8c sets for a render against
# the reference's own unseeded one -- block means (8-bit) mean |d| <= 0.25,
# max <= 2.5, per-pixel mean |d| <= 3.5 -- and segments/sample within 2e-3
BOUNDS_INDEPENDENT = {"seg_rel": 2e-3, "px8_mean": 3.5, "block_mean": 0.25, "block_max": 2.5}


def within(st, bounds=None):
    return {k: st[k] <= v for k, v in (BOUNDS if bounds is None else bounds).items()}
