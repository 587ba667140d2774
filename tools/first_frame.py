#!/usr/bin/env python3
"""The first frame of a launch shape, default schedule against the schedule
switched off, alternated (round 6).

Per round and setting: rt_set_schedule(s), a launch of another shape (8 rows
fewer: this shape becomes new again, so its launch runs in plain tile order
with no record, as a process's first frame does), then the timed launch of
the frame, events on its stream around the whole rt_launch (every kernel it
enqueues: the zero-fills of a new shape's cost record and sharing words, the
trace kernel, the order kernel).  Both settings see a new shape each time
(bench.py's dispatch_order leg times schedule-off on a repeated shape).
Then --cold: in a fresh child process per setting, the process's first three
launches of the frame, each timed (the cold kernel: clocks, caches, code
object), after an optional --spin-ms busy kernel.

  python tools/first_frame.py [--workload c1] [--rounds 9] [--json out.json]
"""
import argparse
import ctypes as C
import json
import os
import statistics
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "raytracing-clj_amd"))
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

from rtclj import raytracing as R, scenes  # noqa: E402
from rtclj._lib import check, lib, rt_params  # noqa: E402
from bench import WORKLOADS  # noqa: E402


def setup(workload):
    wl = WORKLOADS[workload]
    w = wl["width"]
    h = R.image_height(w)
    sc = scenes.cover_c4() if wl["scene"] == "c4" else scenes.cover(11, 42)
    cam = scenes.cover_camera(w, h)
    ds = C.c_void_p()
    check(lib.rt_scene_upload(0, C.byref(sc.c), C.byref(ds)))
    p = rt_params(width=w, height=h, row_begin=0, row_end=h, spp=wl["spp"], max_depth=wl["depth"], seed=1)
    other = rt_params(width=w, height=h, row_begin=0, row_end=h - 8, spp=wl["spp"], max_depth=wl["depth"], seed=1)
    out = torch.empty(h * w * 3, dtype=torch.float32, device="cuda")
    s = torch.cuda.Stream()
    return ds, cam, p, other, out, s


def launch(ds, cam, p, out, s):
    check(lib.rt_launch(ds, C.byref(cam), C.byref(p), C.c_void_p(out.data_ptr()), None, C.c_void_p(s.cuda_stream)))


HOST_MS = []   # per timed launch: the host's rt_launch call (enqueue, set-up, allocations)


def timed(ds, cam, p, out, s):
    import time
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    t0 = time.perf_counter()
    launch(ds, cam, p, out, s)
    HOST_MS.append((time.perf_counter() - t0) * 1e3)
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


def cold(workload, schedule, spin_ms):
    """Child process: the first three launches of the frame, each timed."""
    check(lib.rt_set_schedule(schedule))
    ds, cam, p, other, out, s = setup(workload)
    if spin_ms > 0:
        # a busy GPU for spin_ms before the first frame (clock ramp test):
        # back-to-back small matmuls on the same stream
        a = torch.randn(2048, 2048, device="cuda")
        torch.cuda.synchronize()
        import time
        t0 = time.perf_counter()
        with torch.cuda.stream(s):
            while (time.perf_counter() - t0) * 1e3 < spin_ms:
                a = (a @ a).clamp_(-1, 1)
                torch.cuda.synchronize()
    HOST_MS.clear()
    ev = [timed(ds, cam, p, out, s) for _ in range(3)]
    return {"event_ms": ev, "host_call_ms": list(HOST_MS)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c1", choices=sorted(WORKLOADS))
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--json", default=None)
    ap.add_argument("--cold", action="store_true")
    ap.add_argument("--child", nargs=2, type=int, default=None, help=argparse.SUPPRESS)   # schedule, spin_ms
    a = ap.parse_args()
    if a.child:
        print(json.dumps(cold(a.workload, *a.child)))
        return
    ds, cam, p, other, out, s = setup(a.workload)
    res = {0: [], 1: []}
    for r in range(a.rounds):
        for sched in ((0, 1) if r % 2 == 0 else (1, 0)):
            check(lib.rt_set_schedule(sched))
            launch(ds, cam, other, out, s)
            torch.cuda.synchronize()
            res[sched].append(timed(ds, cam, p, out, s))
    check(lib.rt_set_schedule(0))
    summary = {"workload": a.workload, "rounds": a.rounds,
               "first_frame_schedule_on_ms": res[0], "first_frame_schedule_off_ms": res[1],
               "median_on": statistics.median(res[0]), "median_off": statistics.median(res[1])}
    print(f"first frame of a new shape: schedule on median {summary['median_on']:.3f} ms "
          f"(min {min(res[0]):.3f}), off {summary['median_off']:.3f} ms (min {min(res[1]):.3f})", flush=True)
    if a.cold:
        cc = {}
        for sched, spin in ((0, 0), (1, 0), (0, 200)):
            r = subprocess.run(["timeout", "-k", "10", "120", sys.executable, __file__, "--workload", a.workload,
                                "--child", str(sched), str(spin)], capture_output=True, text=True)
            if r.returncode != 0:
                print(r.stderr[-2000:])
                sys.exit(r.returncode)
            cc[f"schedule{sched}_spin{spin}"] = json.loads(r.stdout.strip().splitlines()[-1])
            d = cc[f"schedule{sched}_spin{spin}"]
            print(f"fresh process, schedule {sched}, spin {spin} ms: launches 1-3 "
                  f"{', '.join(f'{x:.3f}' for x in d['event_ms'])} ms (events on the stream); host rt_launch calls "
                  f"{', '.join(f'{x:.3f}' for x in d['host_call_ms'])} ms", flush=True)
        summary["cold"] = cc
    if a.json:
        Path(a.json).write_text(json.dumps(summary, indent=1))
    lib.rt_scene_free(ds)


if __name__ == "__main__":
    main()
