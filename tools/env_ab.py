#!/usr/bin/env python3
"""A/B of rt_launch's environment knobs (read at every launch) in one process
on one GPU: per setting and round, a shape change (so the frame's next
launch has no tile-cost record: plain order, as a process's first frame),
the first launch timed, then `--warm` launches and `--reps` timed launches in
the recorded order.  Settings alternate within each round, in an order that
rotates from round to round; every frame must be bit-identical.

  python tools/env_ab.py --set RTCLJ_SHARE_ROUNDS=2 --set RTCLJ_SHARE_ROUNDS=1000000 \
      [--workload c1] [--rounds 3] [--reps 10] [--json out.jsonl]
A setting is KEY=VALUE[,KEY=VALUE...]; "-" is the default environment.
"""
import argparse
import ctypes as C
import json
import os
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "raytracing-clj_amd"))
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

from rtclj import raytracing as R, scenes  # noqa: E402
from rtclj._lib import check, lib, rt_params  # noqa: E402
from bench import WORKLOADS  # noqa: E402


def parse_setting(s):
    if s == "-":
        return {}
    return dict(kv.split("=", 1) for kv in s.split(","))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--set", action="append", required=True, dest="sets")
    ap.add_argument("--workload", default="c1", choices=sorted(WORKLOADS))
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--warm", type=int, default=3)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    wl = WORKLOADS[a.workload]
    w = wl["width"]
    h = R.image_height(w)
    sc = scenes.cover_c4() if wl["scene"] == "c4" else scenes.cover(11, 42)
    cam = scenes.cover_camera(w, h)
    ds = C.c_void_p()
    check(lib.rt_scene_upload(0, C.byref(sc.c), C.byref(ds)))
    p = rt_params(width=w, height=h, row_begin=0, row_end=h, spp=wl["spp"], max_depth=wl["depth"], seed=1)
    other = rt_params(width=w, height=h, row_begin=0, row_end=h - 8, spp=1, max_depth=wl["depth"], seed=1)
    out = torch.empty(h * w * 3, dtype=torch.float32, device="cuda")
    ref = None
    s = torch.cuda.Stream()
    sh = C.c_void_p(s.cuda_stream)
    base_env = dict(os.environ)
    res = {k: {"first": [], "steady": []} for k in a.sets}

    def launch(q):
        check(lib.rt_launch(ds, C.byref(cam), C.byref(q), C.c_void_p(out.data_ptr()), None, sh))

    def timed(q):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        launch(q)
        e1.record(s)
        e1.synchronize()
        return e0.elapsed_time(e1)

    for rnd in range(a.rounds):
        # the settings rotate: each round starts with the next one (the first
        # launch after another setting's steady launches measured slower)
        for k in a.sets[rnd % len(a.sets):] + a.sets[:rnd % len(a.sets)]:
            os.environ.clear()
            os.environ.update(base_env)
            os.environ.update(parse_setting(k))
            launch(other)                      # a new shape: the next launch runs in plain order
            res[k]["first"].append(timed(p))
            for _ in range(a.warm):
                launch(p)
            res[k]["steady"].extend(timed(p) for _ in range(a.reps))
            torch.cuda.synchronize()
            img = out.cpu()
            if ref is None:
                ref = img
            assert torch.equal(img, ref), f"setting {k}: frame differs from the first one run"
            print(json.dumps({"round": rnd, "set": k, "first_ms": res[k]["first"][-1],
                              "steady_med_ms": statistics.median(res[k]["steady"][-a.reps:])}), flush=True)
    os.environ.clear()
    os.environ.update(base_env)
    summary = {k: {"first_ms_med": statistics.median(v["first"]), "steady_ms_med": statistics.median(v["steady"]),
                   "steady_ms_min": min(v["steady"]), "first": v["first"]} for k, v in res.items()}
    line = {"workload": a.workload, "rounds": a.rounds, "reps": a.reps, "summary": summary}
    print(json.dumps(line), flush=True)
    if a.json:
        with open(a.json, "a") as f:
            f.write(json.dumps(line) + "\n")
    lib.rt_scene_free(ds)


if __name__ == "__main__":
    main()
