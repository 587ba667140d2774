#!/usr/bin/env python3
"""Frames in flight through rt_render_submit .. rt_render_wait against the
streams the process made before (round 6): a fresh child process per case
makes K torch streams, then runs bench.py's frame loop (two frames in flight,
C1) and prints ms per frame beside one rt_render's total.  Cases cross K with
the render contexts' stream kind (RTCLJ_CTX_STREAM: 0 normal priority, 1 full
CU mask, 2 high priority, the default).  (profiles/r06/inflight/'s run also
crossed a pinned-staging copy for submitted frames, a build since reverted.)

  python tools/inflight_queues.py [--frames 28] [--json out.json]
"""
import argparse
import json
import os
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "raytracing-clj_amd"))
sys.path.insert(0, str(ROOT))


def child(k_streams, frames):
    import numpy as np
    import torch
    from rtclj import raytracing as R, scenes
    from bench import WORKLOADS
    wl = WORKLOADS["c1"]
    W = wl["width"]
    H = R.image_height(W)
    sc = scenes.cover(11, 42)
    cam = scenes.cover_camera(W, H)
    kw = dict(seed=1, n_devices=1)
    keep = [torch.cuda.Stream() for _ in range(k_streams)]
    torch.cuda.synchronize()
    out = R.render(sc, cam, W, H, wl["spp"], wl["depth"], **kw)
    for _ in range(3):
        R.render(sc, cam, W, H, wl["spp"], wl["depth"], out=out, **kw)
    st = {}
    R.render(sc, cam, W, H, wl["spp"], wl["depth"], out=out, stats=st, **kw)
    bufs = [np.empty_like(out) for _ in range(2)]
    for i in range(3):
        R.render_async(sc, cam, W, H, wl["spp"], wl["depth"], out=bufs[i % 2], **kw).wait()
    pending = []
    t0 = time.perf_counter()
    for i in range(frames):
        if len(pending) == 2:
            pending.pop(0).wait()
        pending.append(R.render_async(sc, cam, W, H, wl["spp"], wl["depth"], out=bufs[i % 2], **kw))
    last = {}
    pending[0].wait()
    pending[1].wait(stats=last)
    dt = (time.perf_counter() - t0) / frames * 1e3
    ok = all(bool(np.array_equal(b, out)) for b in bufs)
    del keep
    return {"inflight_ms_per_frame": dt, "rt_render_total_ms": st["total_ms"], "kernel_ms": last["kernel_ms"],
            "d2h_ms": last["d2h_ms"], "equal": ok}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=28)
    ap.add_argument("--json", default=None)
    ap.add_argument("--child", type=int, default=None, help=argparse.SUPPRESS)
    a = ap.parse_args()
    if a.child is not None:
        print(json.dumps(child(a.child, a.frames)))
        return
    res = []
    for kind in ("0", "1", "2"):
        for k in (0, 1, 2, 3):
            env = dict(os.environ, RTCLJ_CTX_STREAM=kind)
            r = subprocess.run(["timeout", "-k", "10", "120", sys.executable, __file__, "--child", str(k),
                                "--frames", str(a.frames)], capture_output=True, text=True, env=env)
            if r.returncode != 0:
                print(r.stdout[-1000:], r.stderr[-2000:])
                sys.exit(r.returncode)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            d.update(ctx_stream=int(kind), torch_streams=k)
            res.append(d)
            print(f"ctx_stream {kind} torch streams {k}: in flight "
                  f"{d['inflight_ms_per_frame']:.3f} ms/frame, rt_render {d['rt_render_total_ms']:.3f}, "
                  f"kernel {d['kernel_ms']:.3f}, d2h {d['d2h_ms']:.3f}, equal {d['equal']}", flush=True)
    if a.json:
        Path(a.json).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
