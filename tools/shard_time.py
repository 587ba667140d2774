#!/usr/bin/env python3
"""Per-shard kernel time of the strong row-tile split on ONE GPU (design tool).

For each world size N, every rank's shard of the frame (shard_params) is
launched on device 0 in turn (warm-up launch for the adaptive tile order,
then --reps timed launches): the max over ranks predicts the N-GPU step time
that bench.py --gpus N measures, without an N-GPU node.

  python tools/shard_time.py [--workload c1] [--worlds 1 2 4 8] [--reps 5]
                             [--inflight S --frames F]

--inflight S: also time F back-to-back frames of each rank's shard issued
round-robin over S streams (frames in flight: frame k+1's workgroups fill the
slots frame k's tail frees), per-frame time = total / F.
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
from rtclj._lib import RT_FLAG_STREAMED, check, lib, rt_params  # noqa: E402
from rtclj.shard import shard_params  # noqa: E402
from bench import WORKLOADS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c1", choices=sorted(WORKLOADS))
    ap.add_argument("--worlds", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--depth", type=int, default=None, help="override the workload's max depth (not a bench line)")
    ap.add_argument("--row-tile", type=int, default=8, help="rows per interleaved shard tile")
    ap.add_argument("--inflight", type=int, nargs="+", default=[0],
                    help="stream counts for the pipelined measurement (0: off)")
    ap.add_argument("--frames", type=int, default=40)
    ap.add_argument("--b2b", type=int, default=0,
                    help="also time this many launches back to back on the one stream (bench.py's timed steps: "
                         "the host's enqueue overlaps the device), per frame")
    ap.add_argument("--no-streamed-flag", action="store_true",
                    help="pipelined launches without RT_FLAG_STREAMED (the single-frame split policy)")
    ap.add_argument("--configs", nargs="*", default=[""],
                    help="environment settings per measurement, e.g. RTCLJ_SPLIT=4,RTCLJ_RING=2 ('' = defaults)")
    a = ap.parse_args()
    wl = WORKLOADS[a.workload]
    W = wl["width"]
    H = R.image_height(W)
    spp = a.spp or wl["spp"]
    if a.depth:
        wl = dict(wl, depth=a.depth)
    sc = scenes.cover_c4() if wl["scene"] == "c4" else scenes.cover(11, 42)
    cam = scenes.cover_camera(W, H)
    stream = torch.cuda.current_stream()
    sh = C.c_void_p(stream.cuda_stream)
    import os
    allres = []
    base = {k: v for k, v in os.environ.items() if k.startswith("RTCLJ_")}   # the caller's settings
    for cfg in a.configs:
        for k in [k for k in os.environ if k.startswith("RTCLJ_")]:
            del os.environ[k]
        os.environ.update(base)
        for kv in filter(None, cfg.split(",")):
            k, v = kv.split("=")
            os.environ[k] = v
        print(f"config {cfg!r}", flush=True)
        res = run(a, wl, W, H, spp, sc, cam, sh, stream)
        res["config"] = cfg
        allres.append(res)
    print(json.dumps(allres))


def run(a, wl, W, H, spp, sc, cam, sh, stream):
    res = {"workload": a.workload, "spp": spp, "depth": wl["depth"], "worlds": {}}
    t1 = None
    t1p = {}
    for n in a.worlds:
        per, per_pipe, per_b2b = [], {}, []
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
            if a.b2b > 0:
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record(stream)
                for _ in range(a.b2b):
                    launch()
                e.record(stream)
                torch.cuda.synchronize()
                per_b2b.append(s.elapsed_time(e) / a.b2b)
            for nin in a.inflight:
                if nin <= 0:
                    continue
                streams = [torch.cuda.Stream() for _ in range(nin)]
                outs = [torch.empty_like(out) for _ in streams]
                shs = [C.c_void_p(x.cuda_stream) for x in streams]
                pp = rt_params(**shard_params(n, r, W, H, spp, wl["depth"], 1, "strong", row_tile=a.row_tile))
                if not a.no_streamed_flag:
                    pp.flags |= RT_FLAG_STREAMED

                def launch_on(i):
                    check(lib.rt_launch(ds, C.byref(cam), C.byref(pp), C.c_void_p(outs[i].data_ptr()),
                                        C.c_void_p(cnt.data_ptr()), shs[i]))
                for _ in range(2):   # each stream's own schedule record
                    for i in range(nin):
                        launch_on(i)
                torch.cuda.synchronize()
                import time
                t0 = time.perf_counter()
                for f in range(a.frames):
                    launch_on(f % nin)
                torch.cuda.synchronize()
                per_pipe.setdefault(nin, []).append((time.perf_counter() - t0) * 1e3 / a.frames)
            lib.rt_scene_free(ds)
        mx = max(per)
        if n == 1:
            t1 = mx
        res["worlds"][n] = {"max_ms": mx, "mean_ms": sum(per) / n, "per_rank_ms": per,
                            "speedup": (t1 / mx) if t1 else None}
        msg = f"N={n}: max {mx:.3f} ms mean {sum(per) / n:.3f} ms speedup {t1 / mx if t1 else 0:.2f}"
        if per_b2b:
            mb = max(per_b2b)
            if n == 1:
                t1b = mb
                res["t1_b2b"] = mb
            t1b = res["t1_b2b"]
            res["worlds"][n]["b2b"] = {"max_ms": mb, "per_rank_ms": per_b2b, "speedup": t1b / mb}
            msg += f" | back to back: {mb:.3f} ms/frame x{t1b / mb:.2f}"
        for nin, pp in per_pipe.items():
            pm = max(pp)
            if n == 1:
                t1p[nin] = pm
            res["worlds"][n][f"pipelined_{nin}"] = {"max_ms": pm, "per_rank_ms": pp,
                                                     "speedup_vs_1gpu_pipelined": t1p[nin] / pm,
                                                     "speedup_vs_1gpu_single": t1 / pm}
            msg += (f" | {nin} streams: {pm:.3f} ms/frame x{t1p[nin] / pm:.2f} (vs 1-GPU single x{t1 / pm:.2f})")
        print(msg, flush=True)
    return res


if __name__ == "__main__":
    main()
