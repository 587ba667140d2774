#!/usr/bin/env python3
"""Per-shard kernel time of the strong row-tile split on ONE GPU (design tool).

For each world size N, every rank's shard of the frame (shard_params) is
launched on device 0 in turn (warm-up launch for the adaptive tile order,
then --reps timed launches): the max over ranks predicts the N-GPU step time
that bench.py --gpus N measures, without an N-GPU node.

  python tools/shard_time.py [--workload c1] [--worlds 1 2 4 8] [--reps 5]
"""
import argparse
import ctypes as C
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "raytracing-clj_amd"))
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

from rtclj import raytracing as R, scenes  # noqa: E402
from rtclj._lib import check, lib, rt_params  # noqa: E402
from rtclj.shard import shard_params  # noqa: E402
from bench import WORKLOADS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c1", choices=sorted(WORKLOADS))
    ap.add_argument("--worlds", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--row-tile", type=int, default=8, help="rows per interleaved shard tile")
    ap.add_argument("--configs", nargs="*", default=[""],
                    help="environment settings per measurement, e.g. RTCLJ_SPLIT=4,RTCLJ_RING=2 ('' = defaults)")
    a = ap.parse_args()
    wl = WORKLOADS[a.workload]
    W = wl["width"]
    H = R.image_height(W)
    spp = a.spp or wl["spp"]
    sc = scenes.cover_c4() if wl["scene"] == "c4" else scenes.cover(11, 42)
    cam = scenes.cover_camera(W, H)
    stream = torch.cuda.current_stream()
    sh = C.c_void_p(stream.cuda_stream)
    import os
    allres = []
    for cfg in a.configs:
        for k in [k for k in os.environ if k.startswith("RTCLJ_") and k != "RTCLJ_SPLIT_ROUNDS"]:
            del os.environ[k]
        for kv in filter(None, cfg.split(",")):
            k, v = kv.split("=")
            os.environ[k] = v
        print(f"config {cfg!r}", flush=True)
        res = run(a, wl, W, H, spp, sc, cam, sh, stream)
        res["config"] = cfg
        allres.append(res)
    print(json.dumps(allres))


def run(a, wl, W, H, spp, sc, cam, sh, stream):
    res = {"workload": a.workload, "spp": spp, "worlds": {}}
    t1 = None
    for n in a.worlds:
        per = []
        for r in range(n):
            ds = C.c_void_p()
            check(lib.rt_scene_upload(0, C.byref(sc.c), C.byref(ds)))
            p = rt_params(**shard_params(n, r, W, H, spp, wl["depth"], 1, "strong", row_tile=a.row_tile))
            rows = check(lib.rt_rows_out(C.byref(p)))
            out = torch.empty(rows * W * 3, dtype=torch.float32, device="cuda")
            cnt = torch.zeros(2, dtype=torch.int64, device="cuda")

            def launch():
                check(lib.rt_launch(ds, C.byref(cam), C.byref(p), C.c_void_p(out.data_ptr()),
                                    C.c_void_p(cnt.data_ptr()), sh))
            launch()
            torch.cuda.synchronize()
            ts = []
            for _ in range(a.reps):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record(stream)
                launch()
                e.record(stream)
                torch.cuda.synchronize()
                ts.append(s.elapsed_time(e))
            per.append(statistics.median(ts))
            lib.rt_scene_free(ds)
        mx = max(per)
        if n == 1:
            t1 = mx
        res["worlds"][n] = {"max_ms": mx, "mean_ms": sum(per) / n, "per_rank_ms": per,
                            "speedup": (t1 / mx) if t1 else None}
        print(f"N={n}: max {mx:.3f} ms mean {sum(per) / n:.3f} ms speedup {t1 / mx if t1 else 0:.2f}", flush=True)
    return res


if __name__ == "__main__":
    main()
