#!/usr/bin/env python3
"""bench.py — Mray-samples/s of the MI355X trace kernel on BASELINE.json's configs.

Workload (default: C1, BASELINE.json configs[1], the metric's own config):
the RTIOW cover scene (grid 11 -> 484 bodies, generator seed 42) at
1200x675, 100 spp, depth 50, fp32, render seed 1.  --workload c2 / c3 / c4
runs the other configs (C4: cover grid 16 truncated to 1000 bodies, depth 64).
A "step" renders one frame:

  * --scaling strong (default): the frame is split into interleaved 8-row
    tiles, tile t on rank t % N -- the north_star row-tile shard of the
    reference's row-chunk executor (raytracing.clj:157-171), one rank per
    GPU, no collective on the data path (the RNG is keyed by (seed, pixel,
    sample), so each rank computes exactly its rows of the 1-GPU frame).
  * --scaling weak: every rank renders the whole frame with its own sample
    stripe [spp*rank, spp*(rank+1)), so per-GPU work is fixed.

Inputs (scene tables, BVH, camera) are resident in HBM before timing; the
frame stays on the device (host gather is not in `value`).  Timing: W untimed
warm-up steps, then K steps bracketed by barrier + synchronize, max over
ranks; kernel durations from HIP events on the launch stream.  After the
timed region rank 0 also times the product's own entry point, rt_render
(scene cache, N-device fan-out over per-device host threads, D2H into pinned
memory and the host gather) as `end_to_end`.

Run:  python bench.py [--gpus N --steps K --warmup W] [--workload c1|c2|c3|c4]
      python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...   (N > 1)
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import csv
import ctypes as C
import json
import os
import platform
import re
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "raytracing-clj_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import rtclj  # noqa: E402
from rtclj import raytracing as R  # noqa: E402
from rtclj import scenes  # noqa: E402
from rtclj._lib import RT_FLAG_REJECTION_SAMPLERS, RT_FLAG_SHARDS_ON_DEVICE0, RT_FLAG_STREAMED, check, diag_lib, lib, \
    rt_params  # noqa: E402
from rtclj.shard import shard_params, shard_rows  # noqa: E402

# BASELINE.json's metric is quoted on C1; the other workloads report the same
# quantity at their own frame (metric_for)
METRIC = "Mray-samples/sec at 1200×675×100spp depth50; achieved HBM GB/s vs peak"


def metric_for(width, height, spp, depth):
    return f"Mray-samples/sec at {width}×{height}×{spp}spp depth{depth}; achieved HBM GB/s vs peak"

# committed rocprofv3 PMC passes of the current build (profiles/pmc.sh), per workload
PMC_DIRS = {"c1": ROOT / "profiles" / "r06" / "pmc_c1", "c4": ROOT / "profiles" / "r06" / "pmc_c4"}
PEAK_FP32_TFLOPS = 157.3   # MI355X_MICROARCH.md: peak FP32 vector rate (packed v_pk_fma_f32)
PEAK_HBM_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E peak
FLOPS_PER_SPHERE = 17      # per-body test, a and r^2 hoisted, fma = 2
FLOPS_PER_SEGMENT_NOMINAL = 100   # SURVEY.md §8d's nominal per-segment term

WORKLOADS = {
    "c1": dict(width=1200, spp=100, depth=50, scene="cover11", name="C1 RTIOW cover 1200x675 100spp depth50"),
    "c2": dict(width=3840, spp=500, depth=50, scene="cover11", name="C2 cover(484) 3840x2160 500spp depth50"),
    "c3": dict(width=3840, spp=1000, depth=50, scene="cover11", name="C3 cover(484) 3840x2160 1000spp depth50"),
    "c4": dict(width=7680, spp=2000, depth=64, scene="c4", name="C4 cover(1000) 7680x4320 2000spp depth64"),
}


def parse():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed frames (default: 100 for c1, a ~0.6 s GPU region; 5 for the larger workloads)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed frames (default: 5 for c1, 1 otherwise)")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="strong")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c1")
    ap.add_argument("--spp", type=int, default=None, help="override the workload's spp (not a bench line)")
    ap.add_argument("--variant", type=int, default=0, help="kernel variant (rt_set_variant; 0 = default)")
    ap.add_argument("--schedule", type=int, default=0,
                    help="tile schedule (rt_set_schedule): 0 adaptive longest-first, 1 plain dispatch order")
    ap.add_argument("--inflight", type=int, default=1,
                    help="frames in flight of the timed steps that make `value`: consecutive frames go "
                         "round-robin to this many streams (rt_launch RT_FLAG_STREAMED when > 1); 1 (default, "
                         "at every N) = one stream, one frame at a time, so `value` is single-frame throughput "
                         "at every N and the rocprof kernel durations are the frame times")
    ap.add_argument("--pipelined", choices=["auto", "off"], default="auto",
                    help="also time the same K frames with the other basis (2 frames in flight if --inflight "
                         "is 1, else 1), reported beside `value` at every N (single_frame / pipelined); "
                         "off for rocprof runs, whose kernel averages must be the single frame's")
    ap.add_argument("--sustained", type=float, default=None,
                    help="seconds of back-to-back single-stream frames after the timed steps, reported as "
                         "`sustained` (clocks and power under a long load; default 5 for c1, 0 otherwise)")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--samplers", choices=["direct", "rejection"], default="direct",
                    help="direct (the product default): the loop-free samplers; rejection: vec3a.clj:74-86's "
                         "rejection loops (RT_FLAG_REJECTION_SAMPLERS) on every launch of the run")
    ap.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    ap.add_argument("--cpu-row-step", type=int, default=2, help="CPU baseline samples rows 0, s, 2s, ...")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every CPU this process may run on")
    ap.add_argument("--e2e", choices=["auto", "off"], default="auto", help="time rt_render end to end on rank 0")
    ap.add_argument("--stats", choices=["auto", "off"], default="auto", help="one untimed stats-build launch")
    ap.add_argument("--first-launch", choices=["auto", "off"], default="auto",
                    help="time a new shape's first launch against the schedule switched off (dispatch_order); "
                         "off for rocprof / PMC runs, whose kernel averages must be the timed frames'")
    a = ap.parse_args()
    global SAMPLER_FLAGS
    SAMPLER_FLAGS = RT_FLAG_REJECTION_SAMPLERS if a.samplers == "rejection" else 0
    if a.steps is None:
        a.steps = 100 if a.workload == "c1" else 5
    if a.warmup is None:
        a.warmup = 5 if a.workload == "c1" else 1
    if a.sustained is None:
        a.sustained = 5.0 if a.workload == "c1" else 0.0
    return a


def host_cpus():
    """CPUs this process can actually use: its affinity set, capped by the
    cgroup CPU quota (the GPU box's share: its affinity lists every CPU of
    the machine, its quota 16; 256 threads on a 16-CPU quota run 2.5x
    slower than 16 -- measured).  Without a readable quota, OMP_NUM_THREADS
    (which the box sets to its share) caps it."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    if quota is None and os.environ.get("OMP_NUM_THREADS", "").isdigit():
        quota = float(os.environ["OMP_NUM_THREADS"])   # the box exports its CPU share here
    n = aff if quota is None else max(1, min(aff, int(quota + 0.5)))
    return n, aff, quota


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


# rt_params.flags bits every launch of the run carries (--samplers)
SAMPLER_FLAGS = 0


def cpu_baseline(scene, cam, w, h, spp, depth, seed, row_step, threads, gpu_rows, gpu_rows_segs):
    """The oracle's fp64 reference-semantics mode (the C++ restatement of the
    Clojure path) on a bounded row sample of the same frame, on host cores;
    and the parity of the GPU frame's same rows: statistically against that
    fp64 render (oracle.pin), and bit for bit against the oracle's fp32 mirror
    of the kernel's contract on four of those rows."""
    sys.path.insert(0, str(ROOT))
    import numpy as np
    import oracle
    from oracle.pin import BOUNDS, BOUNDS_INDEPENDENT, compare, within
    usable, affinity, quota = host_cpus()
    nthreads = threads if threads > 0 else usable
    args = (scene.sphere.astype(np.float64), scene.kind, scene.mat.astype(np.float64), cam.as_list(), cam.defocus,
            w, h, spp, depth)
    t0 = time.perf_counter()
    ref, _, segs, samples = oracle.render(oracle.MODE_REF64, *args, seed=seed, row_step=row_step, nthreads=nthreads)
    dt = time.perf_counter() - t0
    rows = ref.shape[0]
    # the reference's own setting: a pool of 2 threads (raytracing.clj:157),
    # on a 16x sparser row sample (about the same CPU time)
    step2 = row_step * 16
    t1 = time.perf_counter()
    _, _, _, samples2 = oracle.render(oracle.MODE_REF64, *args, seed=seed, row_step=step2, nthreads=min(2, nthreads))
    dt2 = time.perf_counter() - t1
    res = {"value": samples / dt / 1e6, "unit": "Mray-samples/s", "cores": nthreads, "kind": "port",
           "sample": f"rows 0,{row_step},{2 * row_step},... ({rows} rows x {w} px x {spp} spp = {samples} samples) "
                     f"of the same frame, fp64 reference semantics (oracle MODE_REF64), {dt:.1f} s on "
                     f"{nthreads} threads",
           "seconds": dt, "segments_per_sample": segs / max(samples, 1), "cpu_model": cpu_model(),
           "host": platform.node(), "affinity_cpus": affinity, "cgroup_quota_cpus": quota,
           "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
           "two_threads": {"value": samples2 / dt2 / 1e6, "cores": min(2, nthreads),
                           "sample": f"every {step2}th row ({samples2} samples), {dt2:.1f} s: the reference's "
                                     f"pool-size 2 (raytracing.clj:157)"}}
    parity = None
    if gpu_rows is not None:
        direct = not (SAMPLER_FLAGS & RT_FLAG_REJECTION_SAMPLERS)
        # the default loop-free samplers draw other uniforms than the fp64
        # restatement's rejection loops: independent paths, statistical bounds
        bounds = BOUNDS_INDEPENDENT if direct else BOUNDS
        st = compare(ref, segs / samples, gpu_rows, gpu_rows_segs / samples, by=max(1, min(9, rows // 8)))
        ok = within(st, bounds)
        # four of the rows against the fp32 mirror of the same contract and samplers: bit for bit
        mode = oracle.MODE_MIRROR32 | (oracle.DIRECT if direct else 0)
        pick = sorted({0, rows // 4, rows // 2, (3 * rows) // 4})
        t2 = time.perf_counter()
        exact = []
        for i in pick:
            y = i * row_step
            m, _, _, _ = oracle.render(mode, *args, seed=seed, rows=(y, y + 1), nthreads=nthreads)
            exact.append(bool(np.array_equal(m[0], gpu_rows[i])))
        parity = {"against": "oracle MODE_REF64 (the Clojure path in double), same rows, same seed",
                  "draws": "independent (the kernel's loop-free samplers vs the reference's rejection loops)"
                           if direct else "the same (RT_FLAG_REJECTION_SAMPLERS)",
                  "rows": f"0,{row_step},...", "stats": st, "bounds": bounds, "checks": ok,
                  "mirror_rows": {"mode": "MODE_MIRROR32" + (" | DIRECT" if direct else ""),
                                  "rows": [i * row_step for i in pick], "bit_exact": exact,
                                  "seconds": time.perf_counter() - t2},
                  "pass": all(ok.values()) and all(exact)}
    return res, parity


# the statistics build of each product traversal (the diagnostic library), and
# body pairs per leaf of its tree
STATS_OF = {16: (17, 2), 18: (19, 4), 12: (13, 1), 5: (7, 0)}


def stats_leg(scene, cam, p, device, out_numel):
    """One untimed launch of the statistics build of the same frame, scene and
    traversal in the diagnostic library: counted executed flops per segment
    (fma = 2), BVH node / leaf / exact-test counts, wave-level events."""
    d = diag_lib()
    ds = C.c_void_p()
    check(d.rt_scene_upload(device, C.byref(scene.c), C.byref(ds)))
    try:
        v = lib_resolved_variant(scene, device)
        sv, pairs_per_leaf = STATS_OF.get(v, (None, None))
        if sv is None:
            return None
        old = d.rt_set_variant(sv)
        out = torch.empty(out_numel, dtype=torch.float32, device=torch.device("cuda", device))
        cnt = torch.zeros(2, dtype=torch.int64, device=out.device)
        dbg = (C.c_uint64 * 32)()
        try:
            check(d.rt_debug_stats(dbg))   # clear
            s = torch.cuda.current_stream(out.device)
            check(d.rt_launch(ds, C.byref(cam), C.byref(p), C.c_void_p(out.data_ptr()), C.c_void_p(cnt.data_ptr()),
                              C.c_void_p(s.cuda_stream)))
            torch.cuda.synchronize()
            check(d.rt_debug_stats(dbg))
        finally:
            d.rt_set_variant(old)
        segs, smp = (float(x) for x in cnt.cpu().tolist())
    finally:
        d.rt_scene_free(ds)
    wi = max(dbg[0], 1)
    res = {"stats_variant": sv, "flops_per_segment": dbg[18] / segs, "segments_per_sample": segs / smp,
           "per_wave_iter": {"wave_iters_per_sample": wi / smp, "lanes_active": dbg[1] / wi / 64.0,
                             "fresh_blocks": dbg[16] / wi, "fresh_lanes": dbg[17] / max(dbg[16], 1),
                             "random_unit_trips": dbg[14] / wi, "disk_trips": dbg[15] / wi,
                             "dielectric_blocks": dbg[19] / wi, "dielectric_lanes": dbg[20] / max(dbg[19], 1),
                             "lambert_metal_blocks": dbg[21] / wi,
                             "lambert_metal_lanes": dbg[22] / max(dbg[21], 1),
                             "sums_blocks": dbg[23] / wi, "refills": dbg[24] / wi, "claims": dbg[25] / wi,
                             "drain_checks": dbg[26] / wi}}
    if v != 5:
        res.update({"nodes": dbg[2] / segs, "leaf_pairs": pairs_per_leaf * dbg[3] / segs,
                    "exact_tests": dbg[4] / segs})
        res["per_wave_iter"].update({"trav_steps": dbg[6] / wi, "trav_lane_eff": dbg[7] / max(dbg[6], 1) / 64.0,
                                     "leaf_passes": dbg[12] / wi, "exact_passes": dbg[13] / wi})
    return res


_resolved = {}


def lib_resolved_variant(scene, device):
    return _resolved[(id(scene), device)]


# the product kernel in a rocprofv3 CSV: trace_kernel<SRC, SCAN, false, NW>
# (the statistics build's STATS = true launches are not the product's)
PRODUCT_KERNEL = re.compile(r"trace_kernel<[^>]*\bfalse\b")


def _pmc_avg(pmc_dir, passes, counters):
    """Per-dispatch averages of PMC counters over the product kernel's
    launches (trace_kernel, not the stats build) in the committed rocprofv3
    passes (profiles/pmc.sh; one counter group per pass)."""
    acc = {}
    for name in passes:
        f = pmc_dir / f"{name}.csv"
        if not f.exists():
            return None
        for r in csv.DictReader(open(f)):
            if PRODUCT_KERNEL.search(r["Kernel_Name"]) and r["Counter_Name"] in counters:
                acc.setdefault(r["Counter_Name"], []).append((int(r.get("Dispatch_Id") or 0),
                                                              int(r.get("Grid_Size") or 0), float(r["Counter_Value"])))
    if any(c not in acc for c in counters):
        return None
    # the median launch of the timed frames: the pass's last launches, all of
    # one grid (the recorded order: the units alone).  The launches before
    # them include plain-order ones -- a new shape's, with tile sharing's
    # helper workgroups in a larger grid and its HBM sums (C1: 20 vs 10.7 MB
    # written; the first-launch leg's 5 pairs) -- which are left out
    out = {}
    for c, v in acc.items():
        v = sorted(v)
        grid = v[-1][1]
        k = len(v)
        while k > 0 and v[k - 1][1] == grid:
            k -= 1
        out[c] = statistics.median(x for _, _, x in v[k:])
    return out


def pmc_traffic(pmc_dir):
    """HBM bytes per launch (FETCH_SIZE and WRITE_SIZE in their own passes, KB
    units; gfx950's FETCH_SIZE counts half the bytes of wide streaming reads ->
    x2, MI355X_MICROARCH.md §HBM)."""
    v = _pmc_avg(pmc_dir, ("fetch", "write"), ("FETCH_SIZE", "WRITE_SIZE"))
    if v is None:
        return None
    return {"bytes": (2.0 * v["FETCH_SIZE"] + v["WRITE_SIZE"]) * 1024.0, "fetch_bytes_x2": 2048.0 * v["FETCH_SIZE"],
            "write_bytes": 1024.0 * v["WRITE_SIZE"], "source": str(pmc_dir.relative_to(ROOT))}


def pmc_valu(pmc_dir, n_simd=1024, n_xcd=8):
    """VALU issue picture of the same launches (profiles/pmc.sh passes valu1,
    valu2, waits).  On gfx950 a SIMD issues up to two VALU
    instructions per quad-cycle (4 shader cycles): the full-rate ops (fp32
    fma/add/mul, 32-bit add/logic, v_mov, right shifts) dual-issue, the rest
    (packed and 64-bit ops, compares, selects, conversions, min/max, left
    shifts, and ANY instruction with an SGPR operand) take a quad-cycle of
    their own, transcendentals two (measured: profiles/r05/valu/).
      valu_busy       = quad-cycles with >= 1 VALU issue / SIMD quad-cycles
                      = (SQ_ACTIVE_INST_VALU - SQ_ACTIVE_INST_VALU2) / (SIMDs x cycles / 4)
      dual_issue      = SQ_ACTIVE_INST_VALU2 / those busy quad-cycles
      valu_pipe_util  = SQ_INSTS_VALU x 2 / (SIMDs x cycles): the pipe as if every
                        instruction took 2 cycles (a lower bound: single-port ops take 4)
      lanes_active    = SQ_THREAD_CYCLES_VALU / SQ_INSTS_VALU / 64
      salu_per_valu   = SQ_INSTS_SALU / SQ_INSTS_VALU
      wait_dep, wait_issue, issuing = SQ_WAIT_ANY, SQ_WAIT_INST_ANY,
                        SQ_ACTIVE_INST_ANY as shares of SQ_WAVE_CYCLES (wave residency)."""
    v1 = _pmc_avg(pmc_dir, ("valu1",), ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_VALU2", "SQ_INSTS_VALU",
                                        "SQ_THREAD_CYCLES_VALU", "GRBM_GUI_ACTIVE"))
    v2 = _pmc_avg(pmc_dir, ("valu2",), ("SQ_INSTS_SALU", "SQ_INSTS_BRANCH", "GRBM_GUI_ACTIVE"))
    v3 = _pmc_avg(pmc_dir, ("waits",), ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                        "GRBM_GUI_ACTIVE"))
    if v1 is None:
        return None
    cyc = v1["GRBM_GUI_ACTIVE"] / n_xcd
    quads = n_simd * cyc / 4.0
    busy_q = v1["SQ_ACTIVE_INST_VALU"] - v1["SQ_ACTIVE_INST_VALU2"]
    out = {"valu_busy": busy_q / quads, "dual_issue": v1["SQ_ACTIVE_INST_VALU2"] / busy_q,
           "valu_pipe_util": v1["SQ_INSTS_VALU"] * 2.0 / (n_simd * cyc),
           "lanes_active": v1["SQ_THREAD_CYCLES_VALU"] / v1["SQ_INSTS_VALU"] / 64.0,
           "valu_insts": v1["SQ_INSTS_VALU"], "source": str(pmc_dir.relative_to(ROOT))}
    if v2 is not None:
        out["salu_per_valu"] = v2["SQ_INSTS_SALU"] / v1["SQ_INSTS_VALU"]
        out["branch_per_valu"] = v2["SQ_INSTS_BRANCH"] / v1["SQ_INSTS_VALU"]
    if v3 is not None:
        wc = v3["SQ_WAVE_CYCLES"]
        out.update(wait_dep=v3["SQ_WAIT_ANY"] / wc, wait_issue=v3["SQ_WAIT_INST_ANY"] / wc,
                   issuing=v3["SQ_ACTIVE_INST_ANY"] / wc,
                   mean_waves_per_simd=wc * 4.0 / n_simd / (v3["GRBM_GUI_ACTIVE"] / n_xcd))
    return out


def occupancy(ds, p):
    o = (C.c_int * 4)()
    check(lib.rt_launch_occupancy(ds, C.byref(p), o))
    # o[0]: resident workgroups per CU in 256-thread units (4 waves each; the
    # 8-body-leaf variants run 512-thread workgroups: half as many, 8 waves)
    threads = {18: 512, 19: 512, 24: 512, 26: 1024}.get(o[3], 256)
    return {"limit_waves_per_simd": min(8.0, o[0] * 4 / 4.0), "workgroups_per_cu": o[0] * 256 // threads,
            "threads_per_workgroup": threads, "vgprs": o[1],
            "lds_bytes_per_wg": o[2], "variant": o[3], "hw_max_waves_per_simd": 8}


PARTS = ("upload_ms", "setup_ms", "enqueue_ms", "wait_ms", "scatter_ms", "other_ms")


def end_to_end(scene, cam, W, H, spp, depth, seed, n_dev, reps=7, warm=3):
    """rt_render, the product entry point the JNI shim calls: the scene cache
    (the first call uploads and builds the BVHs), the N-device fan-out (a
    task per device on the library's host worker pool), D2H straight into
    the rows of one caller buffer.  The first call of the process (rt_cache_clear() first, so it
    pays the scene upload, the BVH builds and the device context set-up, as
    the reference's one-frame `-main` does), `warm` untimed calls (the
    adaptive tile order converges over ~3 launches: tools/e2e_calls.py), then
    `reps` timed calls into one reused framebuffer, as a renderer drawing
    frames runs, whose median is the value (min and max beside it).  `parts`
    are rt_stats' host clocks of the slowest device's share; they add up to
    total_ms.  `bytes`: the same calls through rt_render_u8 (write-color! on
    the device, a quarter of the copy back), checked equal to rt_quantize of
    the float frame."""
    import numpy as np
    visible = lib.rt_device_count()
    flags = (RT_FLAG_SHARDS_ON_DEVICE0 if n_dev > visible else 0) | SAMPLER_FLAGS
    lib.rt_cache_clear()
    first = {}
    t0 = time.perf_counter()
    out = R.render(scene, cam, W, H, spp, depth, seed=seed, n_devices=n_dev, flags=flags, stats=first)
    first_wall = (time.perf_counter() - t0) * 1e3
    for _ in range(warm):
        R.render(scene, cam, W, H, spp, depth, seed=seed, n_devices=n_dev, flags=flags, out=out)
    runs = []
    for _ in range(reps):
        st = {}
        t0 = time.perf_counter()
        out = R.render(scene, cam, W, H, spp, depth, seed=seed, n_devices=n_dev, flags=flags, stats=st, out=out)
        st["wall_ms"] = (time.perf_counter() - t0) * 1e3
        runs.append(st)
    runs.sort(key=lambda r: r["total_ms"])
    med = runs[len(runs) // 2]
    # rt_render_u8: the frame as write-color!'s bytes (the PPM's), quantised on the device
    b8 = None
    u8_runs = []
    for i in range(warm + reps):
        st = {}
        b8 = R.render(scene, cam, W, H, spp, depth, seed=seed, n_devices=n_dev, flags=flags, stats=st, out=b8, u8=True)
        if i >= warm:
            u8_runs.append(st)
    u8_runs.sort(key=lambda r: r["total_ms"])
    u8_med = u8_runs[len(u8_runs) // 2]
    u8_equal = bool(np.array_equal(b8, R.write_color(out)))

    # frames in flight through the product entry (rt_render_submit ..
    # rt_render_wait): a frame loop keeping `nfl` frames submitted, each into
    # its own framebuffer; frame k+1's shards start on the devices while
    # frame k's rows come back
    nfl = 2
    bufs = [np.empty_like(out) for _ in range(nfl)]
    for i in range(warm):
        R.render_async(scene, cam, W, H, spp, depth, seed=seed, n_devices=n_dev, flags=flags, out=bufs[i % nfl]).wait()
    n_frames = max(4 * reps, 8)
    pending = []
    t0 = time.perf_counter()
    for i in range(n_frames):
        if len(pending) == nfl:
            pending.pop(0).wait()
        pending.append(R.render_async(scene, cam, W, H, spp, depth, seed=seed, n_devices=n_dev, flags=flags,
                                      out=bufs[i % nfl]))
    last = {}
    for f in pending[:-1]:
        f.wait()
    pending[-1].wait(stats=last)
    async_s = time.perf_counter() - t0
    async_equal = all(bool(np.array_equal(b, out)) for b in bufs)
    inflight = {"entry": "rt_render_submit .. rt_render_wait (include/rt.h)", "frames_in_flight": nfl,
                "frames": n_frames, "seconds": async_s, "ms_per_frame": async_s / n_frames * 1e3,
                "value": W * H * spp * n_frames / async_s / 1e6, "unit": "Mray-samples/s",
                "kernel_ms_max_last": last.get("kernel_ms"), "equals_rt_render": async_equal,
                "note": "a frame loop through the product entry: each frame submitted while the one before is still "
                        "on the devices (its shards' launches split for two rounds of workgroups, "
                        "RT_FLAG_STREAMED), waited on in order, every frame into one of two framebuffers; the "
                        "host wall clock over all frames"}

    def parts(r):
        return {k: r[k] for k in PARTS}

    return {"entry": "rt_render (include/rt.h)", "n_devices": med["n_devices"],
            "shards_on_device0": bool(flags & RT_FLAG_SHARDS_ON_DEVICE0), "statistic": f"median of {reps} calls",
            "total_ms": med["total_ms"], "total_ms_min": runs[0]["total_ms"], "total_ms_max": runs[-1]["total_ms"],
            "kernel_ms_max": med["kernel_ms"], "kernel_ms_mean": med["kernel_ms_mean"],
            "imbalance": med["kernel_ms"] / med["kernel_ms_mean"], "d2h_ms": med["d2h_ms"],
            "gather_ms": med["gather_ms"], "scene_cached": med["scene_cached"], "parts": parts(med),
            "value": W * H * spp / (med["total_ms"] * 1e-3) / 1e6, "unit": "Mray-samples/s",
            "first_call": {"total_ms": first["total_ms"], "parts": parts(first), "kernel_ms_max": first["kernel_ms"],
                           "d2h_ms": first["d2h_ms"], "scene_cached": first["scene_cached"],
                           "python_wall_ms": first_wall,
                           "note": "the process's first rt_render after rt_cache_clear(): scene upload + BVH builds "
                                   "(upload_ms), the device context (setup_ms: stream, events, framebuffer, pinned "
                                   "counters), the launch enqueue (enqueue_ms; the first launch of a kernel loads "
                                   "its code object), the device work (wait_ms: kernel in plain tile order + D2H)"},
            "bytes": {"entry": "rt_render_u8 (include/rt.h)", "statistic": f"median of {reps} calls",
                      "total_ms": u8_med["total_ms"], "kernel_ms_max": u8_med["kernel_ms"],
                      "d2h_ms": u8_med["d2h_ms"], "equals_rt_quantize_of_rt_render": u8_equal,
                      "note": "d2h_ms includes the quantise kernel"},
            "frames_in_flight": inflight, "repeats": reps, "warm_calls": warm}, out


def first_process(wl, spp, depth, seed, n_dev):
    """The reference's own usage, one frame per process (`clojure -M:main`,
    raytracing.clj:95-177): lib/rt_main, the C++ host of the C ABI, run as a
    fresh child process on this workload (the cover scene), --json: the HIP
    runtime's start-up (first rt_device_count), rt_render's parts on a cold
    library (scene upload + BVHs, device context, first launch = code-object
    load, kernel in plain tile order + D2H), quantise and the PPM write.
    `next_process`: a second fresh process right after it.  (On a fresh box
    the first such child has paid ~140 ms more in its first allocation +
    launch + sync -- prepare_ms.queue -- than the ones after it,
    profiles/r06/final/bench_reps.jsonl: the runtime's, not the library's.)"""
    import subprocess
    import tempfile
    exe = ROOT / "raytracing-clj_amd" / "lib" / "rt_main"
    if wl["scene"] != "cover11" or not exe.exists():
        return None
    extra = ["--rejection-samplers"] if SAMPLER_FLAGS & RT_FLAG_REJECTION_SAMPLERS else []

    def one():
        with tempfile.TemporaryDirectory() as td:
            t0 = time.perf_counter()
            r = subprocess.run([str(exe), str(spp), str(depth), "--scene", "cover", "--width", str(wl["width"]),
                                "--seed", str(seed), "--gpus", str(n_dev), "--out", str(Path(td) / "scene.ppm"),
                                "--json"] + extra, capture_output=True, text=True, timeout=300)
            wall = (time.perf_counter() - t0) * 1e3
        if r.returncode != 0:
            return {"error": (r.stdout + r.stderr)[-400:]}
        d = json.loads(r.stdout.strip().splitlines()[-1])
        d["child_wall_ms"] = wall
        return d
    d = one()
    if "error" in d:
        return d
    d["command"] = f"rt_main {spp} {depth} --scene cover --width {wl['width']} --seed {seed} --gpus {n_dev} --json"
    nxt = one()
    d["next_process"] = nxt if "error" in nxt else {
        k: nxt[k] for k in ("process_ms", "device_count_ms", "prepare_ms", "prepare_wait_ms", "render_ms",
                            "write_ms", "png_ms", "child_wall_ms")}
    return d



def rank_summary(per_rank, inflight, other_nf, steps, warmup):
    """The cross-rank part of the line from every rank's own record: both
    throughput bases at every N (single_frame: one frame at a time per rank;
    pipelined: 2 frames in flight per rank), `scaling_basis` naming the one
    `value` is (--inflight), and per rank its device (ordinal, UUID, PCI bus:
    a SCALE line shows N distinct devices), rows and times."""
    bases = {}
    for nf, el_key, smp_key in ((inflight, "elapsed_s", "samples"), (other_nf, "other_elapsed_s", "other_samples")):
        if nf is None:
            continue
        el = max(r[el_key] for r in per_rank)
        sm = sum(r[smp_key] for r in per_rank)
        bases["single_frame" if nf == 1 else "pipelined"] = {
            "value": sm / el / 1e6, "unit": "Mray-samples/s", "ms_per_frame": el / steps * 1e3,
            "streams_per_rank": nf, "steps": steps, "warmup": warmup * nf}
    mpf = [r["ms_per_frame"] for r in per_rank]
    per = {"rank": [r["rank"] for r in per_rank], "device": [r["device"] for r in per_rank],
           "device_uuid": [r["device_uuid"] for r in per_rank], "pci_bus_id": [r["pci_bus_id"] for r in per_rank],
           "distinct_devices": len({(r["device_uuid"], r["pci_bus_id"], r["device"]) for r in per_rank}),
           "kernel_ms_avg": [r["kernel_ms_avg"] for r in per_rank], "rows": [r["rows"] for r in per_rank],
           "ms_per_frame": mpf, "imbalance": max(mpf) / (sum(mpf) / len(mpf)),
           "elapsed_ms": [r["elapsed_s"] * 1e3 for r in per_rank],
           "elapsed_with_closing_barrier_ms": max(r["elapsed_barrier_s"] for r in per_rank) * 1e3}
    return {"scaling_basis": "single_frame" if inflight == 1 else "pipelined",
            "single_frame": bases.get("single_frame"), "pipelined": bases.get("pipelined"), "per_rank": per}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus != world and world > 1:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    if a.gpus > 1 and world == 1:
        raise SystemExit("for --gpus N > 1 launch with torch.distributed.run --nproc-per-node N")
    ndev = lib.rt_device_count()
    if not torch.cuda.is_available() or ndev <= 0:
        raise SystemExit("bench.py needs a GPU (MI355X); no device visible")
    # one rank per GPU; more ranks than GPUs only for rehearsals (ranks share)
    device = local % ndev
    torch.cuda.set_device(device)
    dev = torch.device("cuda", device)
    # The render exchanges nothing between ranks (pixels/samples are
    # independent; RNG keyed by (seed, pixel, sample)): the only cross-rank
    # traffic is the barrier and the timing scalars, on the host over gloo
    # (BENCH_DIST_BACKEND=nccl moves them to RCCL).
    backend = os.environ.get("BENCH_DIST_BACKEND", "gloo")
    if world > 1:
        # C-level banners (gloo prints "connected to N peer ranks") go to
        # stderr: stdout carries exactly one JSON line
        saved = os.dup(1)
        sys.stdout.flush()
        os.dup2(2, 1)
        try:
            dist.init_process_group(backend=backend)
            dist.barrier()
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
    check(lib.rt_set_variant(a.variant))
    check(lib.rt_set_schedule(a.schedule))

    wl = dict(WORKLOADS[a.workload])
    if a.spp:
        wl["spp"] = a.spp
    W = wl["width"]
    H = R.image_height(W)
    spp, depth = wl["spp"], wl["depth"]
    scene = scenes.cover_c4() if wl["scene"] == "c4" else scenes.cover(11, 42)
    cam = scenes.cover_camera(W, H)

    ds = C.c_void_p()
    check(lib.rt_scene_upload(device, C.byref(scene.c), C.byref(ds)))
    _resolved[(id(scene), device)] = lib.rt_resolve_variant(ds)
    p = rt_params(**shard_params(world, rank, W, H, spp, depth, a.seed, a.scaling))
    p.flags |= SAMPLER_FLAGS
    rows = check(lib.rt_rows_out(C.byref(p)))
    assert rows == len(shard_rows(H, p.row_tile or 8, p.tile_first, p.tile_step))
    # frames in flight: frame k on streams[k % nf], each stream its own
    # output buffer (and, in the library, its own tile-order record and split
    # sums); the frames are independent, so frame k+1's workgroups take the
    # slots frame k's tail frees.  `value` is timed with
    # --inflight frames in flight (1 by default, at every N: single-frame
    # throughput); the other basis (2 if --inflight is 1) is timed the same
    # way after it and reported beside it (single_frame / pipelined)
    inflight = max(1, a.inflight)
    other_nf = (2 if inflight == 1 else 1) if a.pipelined == "auto" else None
    n_streams = max(inflight, other_nf or 1)
    streams = [torch.cuda.Stream(dev) for _ in range(n_streams)]
    outs = [torch.empty(rows * W * 3, dtype=torch.float32, device=dev) for _ in range(n_streams)]
    out = outs[0]
    counters = torch.zeros(2, dtype=torch.int64, device=dev)
    stream = streams[0]
    sh = C.c_void_p(stream.cuda_stream)
    shs = [C.c_void_p(x.cuda_stream) for x in streams]

    def params_for(nf):
        q = rt_params(**shard_params(world, rank, W, H, spp, depth, a.seed, a.scaling))
        q.flags |= SAMPLER_FLAGS
        if nf > 1:
            q.flags |= RT_FLAG_STREAMED
        return q

    def step(k=0, params=p, nf=1):
        check(lib.rt_launch(ds, C.byref(cam), C.byref(params), C.c_void_p(outs[k % nf].data_ptr()),
                            C.c_void_p(counters.data_ptr()), shs[k % nf]))

    def barrier():
        if world > 1:
            dist.barrier()

    # one frame at a time on one stream (no RT_FLAG_STREAMED): the kernel's
    # own duration, which the roofline and the rocprof average use
    single_ms = None
    if a.warmup > 0:
        for _ in range(2):
            step(0, p)
        n1 = max(3, min(20, a.steps))
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n1)]
        for e0, e1 in ev:
            e0.record(stream)
            step(0, p)
            e1.record(stream)
        torch.cuda.synchronize()
        single_ms = sum(e0.elapsed_time(e1) for e0, e1 in ev) / n1
    # a new shape's first launch (no tile costs yet: tiles in plain dispatch
    # order, as a process's first frame runs), timed once the GPU is warm:
    # after a launch of another shape (8 rows fewer), which makes this frame's
    # shape new again.  Alternated with the same with the schedule off
    # (rt_set_schedule(1)), also after another shape's launch, 9 pairs (C1;
    # one for the other workloads); the medians are reported (single C1
    # launches move by +-0.1 ms)
    first_ms = plain_ms = None
    first_all, plain_all = [], []
    if a.warmup > 0 and a.schedule == 0 and p.row_end - p.row_begin > 16 and a.first_launch == "auto":
        other = type(p).from_buffer_copy(p)
        other.row_end = p.row_end - 8

        def new_shape_launch(sched):
            check(lib.rt_set_schedule(sched))
            step(0, other)
            torch.cuda.synchronize()
            g0, g1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            g0.record(stream)
            step(0, p)
            g1.record(stream)
            torch.cuda.synchronize()
            return g0.elapsed_time(g1)

        new_shape_launch(a.schedule)   # (untimed: the first pair's launches)
        for r in range(9 if a.workload == "c1" else 1):   # (one pair for the long frames)
            for sched in ((a.schedule, 1) if r % 2 == 0 else (1, a.schedule)):
                (first_all if sched == a.schedule else plain_all).append(new_shape_launch(sched))
        first_ms = statistics.median(first_all)
        plain_ms = statistics.median(plain_all)
        check(lib.rt_set_schedule(a.schedule))
        step(0, p)   # (the record again, for the timed steps)

    def timed(nf):
        """W * nf warm-up frames, then exactly K frames bracketed by barrier +
        synchronize; this rank's elapsed time, per-frame spans, counters."""
        pq = params_for(nf)
        for k in range(a.warmup * nf):
            step(k, pq, nf)
        torch.cuda.synchronize()
        counters.zero_()
        starts = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps)]
        ends = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps)]
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(a.steps):
            s_k = streams[k % nf]
            starts[k].record(s_k)
            step(k, pq, nf)
            ends[k].record(s_k)
        torch.cuda.synchronize()
        # each rank's own steps, from the common barrier to its last kernel's
        # end; the max over ranks is the job's time (the closing barrier itself,
        # a host round trip of every rank, is not render time: elapsed_barrier_s)
        t1 = time.perf_counter()
        barrier()
        spans = [s.elapsed_time(e) for s, e in zip(starts, ends)]
        cnt = counters.to("cpu").tolist()
        return {"elapsed_s": t1 - t0, "elapsed_barrier_s": time.perf_counter() - t0, "spans": spans,
                "segments": cnt[0], "samples": cnt[1]}

    main_t = timed(inflight)
    other_t = timed(other_nf) if other_nf else None
    kern_ms = main_t["spans"]
    props = torch.cuda.get_device_properties(dev)
    mine = {"rank": rank, "device": device, "device_name": props.name,
            "device_uuid": str(getattr(props, "uuid", "")), "pci_bus_id": getattr(props, "pci_bus_id", None),
            "local_rank": local, "visible_devices": ndev,
            "elapsed_s": main_t["elapsed_s"], "elapsed_barrier_s": main_t["elapsed_barrier_s"],
            "kernel_ms_avg": single_ms if single_ms is not None else sum(kern_ms) / len(kern_ms),
            "launch_span_ms_avg": sum(kern_ms) / len(kern_ms),
            "kernel_ms_max": max(kern_ms), "rows": rows, "segments": main_t["segments"],
            "samples": main_t["samples"], "first_launch_ms": first_ms, "plain_ms": plain_ms,
            "first_launch_all": first_all, "plain_all": plain_all,
            "ms_per_frame": main_t["elapsed_s"] / a.steps * 1e3,
            "other_elapsed_s": other_t["elapsed_s"] if other_t else None,
            "other_samples": other_t["samples"] if other_t else None}
    per_rank = [mine]
    if world > 1:
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
    elapsed = max(r["elapsed_s"] for r in per_rank)
    segs_total = sum(r["segments"] for r in per_rank)
    samples_total = sum(r["samples"] for r in per_rank)
    kern_avg_ms = mine["kernel_ms_avg"]
    summary = rank_summary(per_rank, inflight, other_nf, a.steps, a.warmup)
    # sustained load: as many single-stream frames as fit the requested seconds
    # at the slowest rank's rate, every rank at once
    sustained = None
    if a.sustained > 0:
        frames = max(1, int(a.sustained * 1e3 / max(r["ms_per_frame"] for r in per_rank)))
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(frames):
            step(0, p)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        barrier()
        els = [el]
        if world > 1:
            els = [None] * world
            dist.all_gather_object(els, el)
        sustained = {"seconds": max(els), "frames": frames,
                     "value": sum(r["rows"] for r in per_rank) * W * spp * frames / max(els) / 1e6,
                     "unit": "Mray-samples/s", "ms_per_frame": max(els) / frames * 1e3,
                     "note": "back-to-back frames on one stream per rank after the timed steps, for the "
                             "requested seconds: the rate under a long load (clocks, power)"}

    res = None
    if rank == 0:
        occ = occupancy(ds, p)
        stats = stats_leg(scene, cam, p, device, rows * W * 3) if a.stats == "auto" else None
        value = samples_total / elapsed / 1e6
        seg_per_sample = segs_total / max(samples_total, 1)
        # the dominant (only) kernel, per launch on rank 0
        launch_samples = rows * W * spp
        launch_segs = seg_per_sample * launch_samples
        kms = [r["kernel_ms_avg"] for r in per_rank]
        pmc_dir = PMC_DIRS.get(a.workload) if (not a.spp and a.variant == 0 and world == 1) else None
        traffic = pmc_traffic(pmc_dir) if pmc_dir else None
        valu = pmc_valu(pmc_dir) if pmc_dir else None
        bf_flops = launch_segs * (FLOPS_PER_SPHERE * len(scene) + FLOPS_PER_SEGMENT_NOMINAL)
        bf_tflops = bf_flops / (kern_avg_ms * 1e-3) / 1e12
        roof = {"bound": "valu", "achieved": None, "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s", "frac": None,
                "traffic": traffic["bytes"] if traffic else None}
        if stats is not None:
            fl = stats["flops_per_segment"]
            tflops = launch_segs * fl / (kern_avg_ms * 1e-3) / 1e12
            roof.update(achieved=tflops, frac=tflops / PEAK_FP32_TFLOPS, flops_per_segment=fl,
                        flops_source=f"counted: executed fp32 flops per lane (fma = 2), one untimed launch of the "
                                     f"statistics build (variant {stats['stats_variant']}, lib/librtclj_diag.so) of "
                                     f"the same frame")
        if valu is not None:
            roof.update({k: valu[k] for k in ("valu_busy", "dual_issue", "valu_pipe_util", "lanes_active",
                                              "salu_per_valu", "wait_dep", "wait_issue", "issuing") if k in valu})
        roof["note"] = ("VALU-issue bound: branchy per-ray fp32 work, no GEMM shape (MFMA unused), HBM not binding "
                        "(hbm_roofline). peak = the fp32 vector rate (157.3 TF/s: 2 flops x 32 lanes per cycle per "
                        "SIMD, i.e. v_fma_f32 dual-issued). PMC of the same launch: valu_busy = share of SIMD "
                        "quad-cycles issuing a VALU instruction, dual_issue = share of those issuing two; "
                        "single-port instructions (compares, selects, conversions, min/max, packed ops, SGPR "
                        "operands) take a quad-cycle alone, so the pipe is full while frac stays low -- "
                        "lanes_active of the 64 lanes do work per instruction (divergence). valu_pipe_util = "
                        "SQ_INSTS_VALU x 2 / SIMD cycles assumes every instruction dual-issues (a lower bound).")
        roof["brute_force_equivalent"] = {
            "tflops": bf_tflops, "frac": bf_tflops / PEAK_FP32_TFLOPS,
            "note": f"SURVEY.md §8d's formula (17 x {len(scene)} bodies + 100 per segment) prices the linear scan; "
                    f"the BVH tests ~1/19 of those bodies and returns the scan's hits bit for bit "
                    f"(tests/test_gpu_parity.py::test_bvh_bit_exact_on_full_c1_and_reference), so at "
                    f"{bf_tflops / PEAK_FP32_TFLOPS:.2f}x of peak that formula does not apply to this kernel"}
        hbm_bytes = rows * W * 12 + len(scene) * 32
        gbs = hbm_bytes / (kern_avg_ms * 1e-3) / 1e9
        res = {
            "metric": METRIC if (a.workload == "c1" and not a.spp) else metric_for(W, H, spp, depth), "value": value, "unit": "Mray-samples/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": elapsed / a.steps * 1e3, "higher_is_better": True,
            "scaling": a.scaling, "vs_baseline": None, "dtype": "fp32",
            "data": f"synthetic: RTIOW cover scene ({len(scene)} bodies, generator seed 42), render seed {a.seed}",
            "config": {"workload": wl["name"] if not a.spp else f"{wl['name']} (spp override {spp})",
                       "width": W, "height": H, "spp": spp, "max_depth": depth, "bodies": len(scene),
                       "parallelism": ("row-tile 8 x%d (strong)" % world) if a.scaling == "strong"
                       else ("sample-stripe x%d (weak)" % world), "variant": a.variant,
                       "tile_schedule": "adaptive longest-first" if a.schedule == 0 else "dispatch order",
                       "samplers": "loop-free (default)" if a.samplers == "direct"
                       else "rejection (RT_FLAG_REJECTION_SAMPLERS)"},
            "roofline": roof,
            "hbm_roofline": {"bound": "hbm", "achieved": gbs, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                             "frac": gbs / PEAK_HBM_GBS, "traffic": traffic["bytes"] if traffic else None,
                             "traffic_detail": traffic,
                             "note": "non-binding: algorithmic bytes/launch = W*rows*12 (fp32 RGB written once) + "
                                     "bodies*32 (scene read); traffic = PMC FETCH_SIZE x2 + WRITE_SIZE per launch. "
                                     "Beyond the algorithmic bytes: the 12-byte pixels' partial 64-B lines, and the tile "
                                     "sharing's global atomics (each wave's batch claims on its tile's word, the helper "
                                     "workgroups' owner-table reads and shared tiles' sums; DESIGN.md §3.1), not "
                                     "re-reads"},
            "valu": valu, "occupancy": occ, "stats_build": stats,
            "kernel_ms_avg": kern_avg_ms, "launch_span_ms_max": mine["kernel_ms_max"],
            "dispatch_order": {"kernel_ms": mine["first_launch_ms"],
                               "plain_schedule_off_ms": mine["plain_ms"],
                               "kernel_ms_all": mine["first_launch_all"],
                               "plain_schedule_off_ms_all": mine["plain_all"],
                               "note": "the first launch of a new shape (no tile costs yet: tiles in plain dispatch "
                                       "order, as a process's first frame runs), timed after the GPU is warm, right "
                                       "after a launch of another shape; plain_schedule_off_ms: the same frame with "
                                       "the schedule off (rt_set_schedule(1)), also a new shape; medians of 9 "
                                       "alternated pairs (events around the whole rt_launch: its fills and kernels); "
                                       "the timed steps dispatch longest first by the previous launches' per-tile "
                                       "durations (each added to half the record before it)"},
            "scaling_basis": summary["scaling_basis"], "single_frame": summary["single_frame"],
            "pipelined": summary["pipelined"],
            "frames_in_flight": {"streams": inflight, "rt_launch_flags": "RT_FLAG_STREAMED" if inflight > 1 else 0,
                                 "launch_span_ms_avg": mine["launch_span_ms_avg"],
                                 "note": "timed frames go round-robin to this many streams (independent frames: "
                                         "the next frame's workgroups take the slots this frame's tail frees); "
                                         "kernel_ms_avg and the roofline are the same frame launched alone on one "
                                         "stream; launch_span_ms_avg = each timed frame's start-to-end on its stream "
                                         "(spans overlap)"},
            "per_rank": summary["per_rank"],
            "segments_per_sample": seg_per_sample, "samples_per_step": samples_total / a.steps,
            "kernel": "rtclj::trace_kernel<SRC,SCAN,STATS> (default: BVH with 4-body leaves in LDS, 8x8-pixel "
                      "sample pool per 256-thread workgroup, fixed-point colour sums in LDS)",
            "sustained": sustained, "end_to_end": None, "cpu_baseline": None, "parity": None,
        }
    if a.e2e == "auto":
        # the product fan-out over world devices, timed on rank 0 while the
        # other ranks wait at the barrier
        barrier()
        if rank == 0:
            res["end_to_end"], frame = end_to_end(scene, cam, W, H, spp, depth, a.seed, world)
            if world == 1:
                res["end_to_end"]["first_process"] = first_process(wl, spp, depth, a.seed, world)
        barrier()
    if rank == 0:
        if a.cpu_baseline == "auto" and world == 1:
            import numpy as np
            gpu_rows = segs_rows = None
            if a.scaling == "strong":
                # the GPU frame's rows 0, s, 2s, ... and their own segment count
                # (one untimed launch of just those rows: 1-row tiles, stride s)
                pr = rt_params(width=W, height=H, row_begin=0, row_end=H, spp=spp, max_depth=depth, seed=a.seed,
                               row_tile=1, tile_first=0, tile_step=a.cpu_row_step, flags=SAMPLER_FLAGS)
                nr = check(lib.rt_rows_out(C.byref(pr)))
                o2 = torch.empty(nr * W * 3, dtype=torch.float32, device=dev)
                c2 = torch.zeros(2, dtype=torch.int64, device=dev)
                check(lib.rt_launch(ds, C.byref(cam), C.byref(pr), C.c_void_p(o2.data_ptr()),
                                    C.c_void_p(c2.data_ptr()), sh))
                torch.cuda.synchronize()
                gpu_rows = o2.cpu().numpy().reshape(nr, W, 3)
                full = out.cpu().numpy().reshape(H, W, 3)
                assert np.array_equal(gpu_rows, full[::a.cpu_row_step]), "row launch != the timed frame's rows"
                segs_rows = float(c2[0].item())
            res["cpu_baseline"], res["parity"] = cpu_baseline(scene, cam, W, H, spp, depth, a.seed, a.cpu_row_step,
                                                              a.cpu_threads, gpu_rows, segs_rows)
        print(json.dumps(res), flush=True)
    lib.rt_scene_free(ds)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
