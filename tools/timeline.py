#!/usr/bin/env python3
"""Wave timeline of one launch (design tool, diagnostic build): where a
launch's time goes between ramp-up, steady state and drain.

Runs the default traversal (variant 16) with a per-wave {start, end, HW_ID,
XCC_ID} record (RTCLJ_TIMELINE=1), or its statistics variant 17 (counters as
well, about 16x slower), on a workload's shard, after one
warm-up launch for the adaptive tile order, and prints: span, resident-wave
occupancy over time (20 bins), workgroup durations, the time from the last
workgroup start to the end (tail), and the per-wave-iteration lane
efficiency of the outer loop.

  python tools/timeline.py [--workload c1] [--world 8] [--rank 0] [--variant 17]
"""
import argparse
import ctypes as C
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "raytracing-clj_amd"))
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from rtclj import raytracing as R, scenes  # noqa: E402
from rtclj._lib import check, diag_lib, rt_params  # noqa: E402
from rtclj.shard import shard_params  # noqa: E402
from bench import WORKLOADS  # noqa: E402

os.environ.setdefault("RTCLJ_TIMELINE", "1")   # read when the diagnostic build loads
lib = diag_lib()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c1", choices=sorted(WORKLOADS))
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--variant", type=int, default=16, help="16: the default traversal (timeline only); 17: with counters (~16x slower)")
    ap.add_argument("--bins", type=int, default=20)
    ap.add_argument("--warm", type=int, default=1, help="untimed launches before the recorded one (the adaptive order's history)")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    wl = WORKLOADS[a.workload]
    W = wl["width"]
    H = R.image_height(W)
    sc = scenes.cover_c4() if wl["scene"] == "c4" else scenes.cover(11, 42)
    cam = scenes.cover_camera(W, H)
    stream = torch.cuda.current_stream()
    sh = C.c_void_p(stream.cuda_stream)
    check(lib.rt_set_variant(a.variant))
    ds = C.c_void_p()
    check(lib.rt_scene_upload(0, C.byref(sc.c), C.byref(ds)))
    p = rt_params(**shard_params(a.world, a.rank, W, H, wl["spp"], wl["depth"], 1, "strong"))
    rows = check(lib.rt_rows_out(C.byref(p)))
    out = torch.empty(rows * W * 3, dtype=torch.float32, device="cuda")
    cnt = torch.zeros(2, dtype=torch.int64, device="cuda")
    occ = (C.c_int * 4)()
    check(lib.rt_launch_occupancy(ds, C.byref(p), occ))

    def launch():
        check(lib.rt_launch(ds, C.byref(cam), C.byref(p), C.c_void_p(out.data_ptr()), C.c_void_p(cnt.data_ptr()), sh))

    for _ in range(a.warm):   # warm-up: the adaptive order's record for the next launch
        launch()
    torch.cuda.synchronize()
    st = (C.c_uint64 * 32)()
    check(lib.rt_debug_stats(st))
    wv = np.zeros(4 * 131072, np.uint64)
    check(lib.rt_debug_waves(0, wv.ctypes.data_as(C.POINTER(C.c_uint64)), 131072))
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(stream)
    launch()
    e.record(stream)
    torch.cuda.synchronize()
    ms = s.elapsed_time(e)
    check(lib.rt_debug_stats(st))
    n = check(lib.rt_debug_waves(0, wv.ctypes.data_as(C.POINTER(C.c_uint64)), 131072))
    w = wv[: 4 * n].reshape(n, 4).astype(np.int64)
    w = w[w[:, 1] > 0]
    t0 = w[:, 0].min()
    start = (w[:, 0] - t0) / 100.0   # us (100 MHz)
    end = (w[:, 1] - t0) / 100.0
    span = end.max()
    dur = end - start
    wg_start = start.reshape(-1, 4).min(1) if len(start) % 4 == 0 else start
    slots = occ[0] * 4 * 256 if occ[0] else None   # workgroups per CU x 4 waves x 256 CUs
    bins = np.linspace(0, span, a.bins + 1)
    resident = [float(((start < hi) & (end > lo)).sum()) for lo, hi in zip(bins[:-1], bins[1:])]
    # time-weighted resident waves per bin
    busy = []
    for lo, hi in zip(bins[:-1], bins[1:]):
        ov = np.clip(np.minimum(end, hi) - np.maximum(start, lo), 0, None)
        busy.append(float(ov.sum() / (hi - lo)))
    res = {
        "workload": a.workload, "world": a.world, "rank": a.rank, "variant": a.variant, "warm": a.warm,
        "kernel_ms_event": ms, "span_us": float(span), "waves": int(len(w)),
        "occupancy_api": list(occ),
        "wave_us": {"mean": float(dur.mean()), "p50": float(np.median(dur)), "p95": float(np.percentile(dur, 95)),
                    "max": float(dur.max())},
        "last_wave_start_us": float(start.max()),
        "tail_us": float(span - start.max()),
        "mean_resident_waves": float(dur.sum() / span),
        "resident_slots": slots,
        "busy_waves_per_bin": [round(b, 1) for b in busy],
        "outer_lanes_active": float(st[1]) / max(1, st[0]) / 64.0,
        "wave_iters": int(st[0]),
        # the 12 waves that end last: (dispatch slot, start us, end us)
        "last_enders": [(int(i) // 4, round(float(start[i]), 1), round(float(end[i]), 1))
                        for i in np.argsort(end)[-12:]],
        # end-time quantiles of the waves (us)
        "end_q": {q: round(float(np.percentile(end, q)), 1) for q in (50, 90, 95, 99, 99.9, 100)},
        "start_q": {q: round(float(np.percentile(start, q)), 1) for q in (50, 90, 99, 100)},
    }
    print(json.dumps(res))
    if a.json:
        with open(a.json, "a") as f:
            f.write(json.dumps(res) + "\n")
    lib.rt_scene_free(ds)


if __name__ == "__main__":
    main()
