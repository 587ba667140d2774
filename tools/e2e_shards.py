#!/usr/bin/env python3
"""rt_render end to end with N shards (design tool).

On one GPU, RT_FLAG_SHARDS_ON_DEVICE0 runs the N shards of an N-GPU call on
device 0 (one host thread each, their kernels sharing the GPU), so the wall
time is not the N-GPU one.  Modelled per rank instead: kernel_ms (the
slowest shard alone... measured with the shards side by side, an upper
bound) plus that shard's D2H of its row tiles into the caller's buffer.

  python tools/e2e_shards.py [--workload c1] [--shards 1 8] [--reps 5]
"""
import argparse
import ctypes as C
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "raytracing-clj_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (before librtclj.so: tests/conftest.py)

from bench import WORKLOADS  # noqa: E402
from rtclj import raytracing as R, scenes  # noqa: E402
from rtclj._lib import RT_FLAG_SHARDS_ON_DEVICE0, check, lib, rt_params, rt_stats  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c1", choices=sorted(WORKLOADS))
    ap.add_argument("--shards", type=int, nargs="+", default=[1, 8])
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    wl = WORKLOADS[a.workload]
    W = wl["width"]
    H = R.image_height(W)
    sc = scenes.cover_c4() if wl["scene"] == "c4" else scenes.cover(11, 42)
    cam = scenes.cover_camera(W, H)
    out = np.empty((H, W, 3), np.float32)
    ref = None
    res = {}
    for n in a.shards:
        p = rt_params(width=W, height=H, row_begin=0, row_end=H, spp=wl["spp"], max_depth=wl["depth"], seed=1,
                      n_devices=n, flags=RT_FLAG_SHARDS_ON_DEVICE0 if n > 1 else 0)
        runs = []
        for r in range(a.reps + 1):
            out.fill(np.nan)
            st = rt_stats()
            check(lib.rt_render(C.byref(sc.c), C.byref(cam), C.byref(p), out.ctypes.data_as(C.POINTER(C.c_float)),
                                out.size, C.byref(st)))
            if ref is None:
                ref = out.copy()
            assert np.array_equal(out, ref), n   # every shard count: the same bits
            if r:
                runs.append(st.as_dict())
        med = {k: statistics.median(x[k] for x in runs) for k in ("total_ms", "kernel_ms", "kernel_ms_mean", "d2h_ms",
                                                                   "gather_ms", "enqueue_ms", "wait_ms")}
        med["modelled_rank_ms"] = med["kernel_ms"] + med["d2h_ms"]
        res[n] = med
        print(f"shards={n}: total {med['total_ms']:.3f} ms (all shards on device 0), kernel max {med['kernel_ms']:.3f} "
              f"mean {med['kernel_ms_mean']:.3f}, d2h max {med['d2h_ms']:.3f}, modelled per-rank "
              f"{med['modelled_rank_ms']:.3f} ms", flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
