#!/usr/bin/env python3
"""Kernel time of one library build on a cover scene of a chosen grid (one
process; RTCLJ_LIBRARY selects the build), for A/Bs of builds whose
occupancy differs (e.g. a seven-waves-per-SIMD build on a scene whose LDS
image lets seven workgroups share a CU).  Prints one JSON line: median
kernel ms over the timed frames (rt_launch on one uploaded scene, the
adaptive tile order active after the warm-ups), the launch's occupancy, and
a checksum of the frame's bits (equal across builds: bit-identical frames).

  RTCLJ_LIBRARY=raytracing-clj_amd/lib/ab_w7.so python tools/scene_time.py --grid 9
"""
import argparse
import ctypes as C
import hashlib
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "raytracing-clj_amd"))

import torch  # noqa: E402,F401  (before the library: torch's HIP runtime serves the process)

from rtclj import scenes  # noqa: E402
from rtclj._lib import check, lib, library_path, rt_params  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=11)
    ap.add_argument("--width", type=int, default=1200)
    ap.add_argument("--height", type=int, default=675)
    ap.add_argument("--spp", type=int, default=100)
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args()
    w, h = a.width, a.height
    sc, cam = scenes.cover(a.grid), scenes.cover_camera(w, h)
    ds = C.c_void_p()
    check(lib.rt_scene_upload(0, C.byref(sc.c), C.byref(ds)))
    p = rt_params(width=w, height=h, row_begin=0, row_end=h, spp=a.spp, max_depth=a.depth, seed=1)
    o = (C.c_int * 4)()
    check(lib.rt_launch_occupancy(ds, C.byref(p), o))
    out = torch.empty(h * w * 3, dtype=torch.float32, device="cuda")
    stream = torch.cuda.current_stream()
    ts = []
    for i in range(a.warmup + a.frames):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        check(lib.rt_launch(ds, C.byref(cam), C.byref(p), C.c_void_p(out.data_ptr()), None,
                            C.c_void_p(stream.cuda_stream)))
        e1.record(stream)
        torch.cuda.synchronize()
        if i >= a.warmup:
            ts.append(e0.elapsed_time(e1))
    digest = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16]
    lib.rt_scene_free(ds)
    print(json.dumps({"library": Path(library_path).name, "grid": a.grid, "bodies": len(sc),
                      "frame": f"{w}x{h} spp{a.spp} depth{a.depth}", "kernel_ms": statistics.median(ts),
                      "kernel_ms_min": min(ts), "workgroups_per_cu": o[0], "vgprs": o[1],
                      "lds_bytes_per_wg": o[2], "variant": o[3], "frame_sha256_16": digest}))


if __name__ == "__main__":
    main()
