#!/usr/bin/env python3
"""rt_render call by call (design tool): C1 through the Python mirror, first
call after rt_cache_clear(), then N calls into fresh arrays and N into one
reused array; prints each call's rt_stats (total, kernel, D2H ms)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "raytracing-clj_amd"))

import numpy as np  # noqa: E402

from rtclj import raytracing as R, scenes  # noqa: E402
from rtclj._lib import lib  # noqa: E402


def main(n=8):
    W, H, spp = 1200, 675, 100
    sc = scenes.cover(11, 42)
    cam = scenes.cover_camera(W, H)
    lib.rt_cache_clear()
    for label, reuse in (("first", None), ("fresh", None), ("reused", np.empty((H, W, 3), np.float32))):
        for k in range(1 if label == "first" else n):
            st = {}
            R.render(sc, cam, W, H, spp, 50, seed=1, stats=st, out=reuse)
            print(f"{label:6s} {k}: total {st['total_ms']:.3f} kernel {st['kernel_ms']:.3f} d2h {st['d2h_ms']:.3f} "
                  f"enqueue {st['enqueue_ms']:.3f}", flush=True)


if __name__ == "__main__":
    main()
