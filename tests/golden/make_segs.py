#!/usr/bin/env python3
"""Regenerate tests/golden/segs_ref64.json: segments per sample of each
BASELINE.json config's scene under the reference's semantics in double
(oracle MODE_REF64, the Clojure path restated: raytracing.clj:45-58 counts one
hit-anything call per segment), at the config's own resolution, camera and
depth.

Segments per sample is a property of the workload (scene, camera, depth),
not of spp, seed or tiling: the GPU's full-frame count (one counter per
hit-anything call) must land on it within the cover pin's 2e-3 relative bound
(oracle/pin.py), which catches a systematic shift of the shading or the
traversal that the image statistics would blur (tests/test_gpu_configs.py).

Each estimate covers every row (row_step 1, or 2 for C4's 4320 rows) at a
few spp, split into 4 batches of disjoint sample indices (sample_begin), so
the file also carries the estimate's standard error (std of the batch means
/ 2).  The render seed (7) differs from the tests' (1): the estimate is
independent of the frames it checks.

Usage: python tests/golden/make_segs.py   (~3 min on 8 threads)
"""
from __future__ import annotations

import json
import os
import sys
import time
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "raytracing-clj_amd"))

import oracle  # noqa: E402
from rtclj import raytracing as R  # noqa: E402
from rtclj import scenes  # noqa: E402

# config -> (scene, width, depth, spp per batch, row_step)
CONFIGS = {
    "c1": ("cover11", 1200, 50, 4, 1),
    "c2": ("cover11", 3840, 50, 1, 1),     # C3 renders the same scene and camera
    "c4": ("c4", 7680, 64, 1, 2),
}
BATCHES = 4
SEED = 7


def main():
    nt = os.cpu_count() or 1
    res = {"generator": "tests/golden/make_segs.py", "mode": "oracle MODE_REF64", "seed": SEED, "configs": {}}
    for name, (scene, w, depth, spp, step) in CONFIGS.items():
        sc = scenes.cover_c4() if scene == "c4" else scenes.cover(11)
        h = R.image_height(w)
        cam = scenes.cover_camera(w, h)
        args = (sc.sphere.astype(np.float64), sc.kind, sc.mat.astype(np.float64), cam.as_list(), cam.defocus,
                w, h, spp, depth)
        t0 = time.perf_counter()
        per = []
        for b in range(BATCHES):
            _, _, segs, smp = oracle.render(oracle.MODE_REF64, *args, seed=SEED, sample_begin=b * spp,
                                            row_step=step, nthreads=nt)
            per.append((segs, smp))
        segs = sum(s for s, _ in per)
        smp = sum(n for _, n in per)
        means = np.array([s / n for s, n in per])
        se = float(means.std(ddof=1) / np.sqrt(BATCHES))
        res["configs"][name] = {"scene": scene, "bodies": len(sc), "width": w, "height": h, "max_depth": depth,
                                "rows": f"every {step}" if step > 1 else "all", "spp": spp * BATCHES,
                                "segments": segs, "samples": smp, "segments_per_sample": segs / smp,
                                "std_error": se, "rel_std_error": se / (segs / smp)}
        print(name, res["configs"][name], f"{time.perf_counter() - t0:.1f} s", flush=True)
    (HERE / "segs_ref64.json").write_text(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
