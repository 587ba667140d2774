#!/usr/bin/env python3
"""C1's scene at the same sample count spread over more or fewer tiles
(round 6): width 2400 / 1200 / 600 / 300 with spp 25 / 100 / 400 / 1600
(81 M samples each, the cover camera at each size), 10 launches back to back
after 3 warm-ups, ms per launch.  A per-frame cost that follows the tile
count is per workgroup (set-up, drain); one that stays is the launch's.

  python tools/tiles_vs_samples.py
"""
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "raytracing-clj_amd"))

import torch  # noqa: E402

from rtclj import raytracing as R, scenes  # noqa: E402
from rtclj._lib import check, lib, rt_params  # noqa: E402


def main():
    sc = scenes.cover(11, 42)
    ds = C.c_void_p()
    check(lib.rt_scene_upload(0, C.byref(sc.c), C.byref(ds)))
    s = torch.cuda.current_stream()
    for w, spp in ((2400, 25), (1200, 100), (600, 400), (300, 1600), (1200, 100)):
        h = R.image_height(w)
        cam = scenes.cover_camera(w, h)
        p = rt_params(width=w, height=h, row_begin=0, row_end=h, spp=spp, max_depth=50, seed=1)
        out = torch.empty(h * w * 3, dtype=torch.float32, device="cuda")
        for _ in range(3):
            check(lib.rt_launch(ds, C.byref(cam), C.byref(p), C.c_void_p(out.data_ptr()), None, C.c_void_p(s.cuda_stream)))
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(10):
            check(lib.rt_launch(ds, C.byref(cam), C.byref(p), C.c_void_p(out.data_ptr()), None, C.c_void_p(s.cuda_stream)))
        e1.record(s)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        tiles = ((w + 7) // 8) * ((h + 7) // 8)
        print(f"{w}x{h} spp {spp}: {tiles} tiles, {w * h * spp / 1e6:.1f} M samples, {ms:.3f} ms per launch, "
              f"{w * h * spp / ms / 1e3:.0f} Mray-samples/s", flush=True)
    lib.rt_scene_free(ds)


if __name__ == "__main__":
    main()
