#!/usr/bin/env python3
"""Launch N frames of a workload through rt_launch on one stream, one after
the other (the first in plain order, the rest in the recorded tile order):
a short program for rocprofv3 PMC passes, whose per-dispatch counters are
then read for the last launch (tools/pmc_frames.py).

  python tools/launch_frames.py [--workload c1] [--frames 3]
"""
import argparse
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "raytracing-clj_amd"))
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

from rtclj import raytracing as R, scenes  # noqa: E402
from rtclj._lib import check, lib, rt_params  # noqa: E402
from bench import WORKLOADS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c1", choices=sorted(WORKLOADS))
    ap.add_argument("--frames", type=int, default=3)
    ap.add_argument("--variant", type=int, default=0)
    a = ap.parse_args()
    check(lib.rt_set_variant(a.variant))
    wl = WORKLOADS[a.workload]
    w = wl["width"]
    h = R.image_height(w)
    sc = scenes.cover_c4() if wl["scene"] == "c4" else scenes.cover(11, 42)
    cam = scenes.cover_camera(w, h)
    ds = C.c_void_p()
    check(lib.rt_scene_upload(0, C.byref(sc.c), C.byref(ds)))
    p = rt_params(width=w, height=h, row_begin=0, row_end=h, spp=wl["spp"], max_depth=wl["depth"], seed=1)
    out = torch.empty(h * w * 3, dtype=torch.float32, device="cuda")
    s = torch.cuda.current_stream()
    for k in range(a.frames):
        check(lib.rt_launch(ds, C.byref(cam), C.byref(p), C.c_void_p(out.data_ptr()), None, C.c_void_p(s.cuda_stream)))
        torch.cuda.synchronize()
        print(f"frame {k} done", flush=True)
    lib.rt_scene_free(ds)


if __name__ == "__main__":
    main()
