#!/usr/bin/env python3
"""rt_render's fan-out overhead (design tool): the median wall time of N-shard
calls on device 0 (RT_FLAG_SHARDS_ON_DEVICE0) of a tiny frame, where the
host side -- per-device threads, context hand-out, copies -- is most of the
call.  RTCLJ_LIBRARY selects the build (A/B).

  python tools/fanout_overhead.py [--shards 1 2 8] [--calls 50]
"""
import argparse
import json
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "raytracing-clj_amd")]

import torch  # noqa: E402,F401

from rtclj import raytracing as R, scenes  # noqa: E402
from rtclj._lib import RT_FLAG_SHARDS_ON_DEVICE0, library_path  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shards", type=int, nargs="+", default=[1, 2, 8])
    ap.add_argument("--calls", type=int, default=50)
    a = ap.parse_args()
    sc = scenes.cover(11)
    w, h = 128, 72
    cam = scenes.cover_camera(w, h)
    res = {"library": str(library_path)}
    for n in a.shards:
        out = R.render(sc, cam, w, h, spp=1, seed=1, n_devices=n, flags=RT_FLAG_SHARDS_ON_DEVICE0)
        for _ in range(5):
            R.render(sc, cam, w, h, spp=1, seed=1, n_devices=n, flags=RT_FLAG_SHARDS_ON_DEVICE0, out=out)
        ts = []
        for _ in range(a.calls):
            t0 = time.perf_counter()
            R.render(sc, cam, w, h, spp=1, seed=1, n_devices=n, flags=RT_FLAG_SHARDS_ON_DEVICE0, out=out)
            ts.append((time.perf_counter() - t0) * 1e3)
        res[n] = {"median_ms": statistics.median(ts), "min_ms": min(ts)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
