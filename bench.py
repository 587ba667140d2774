#!/usr/bin/env python3
"""bench.py — Mray-samples/s of the MI355X trace kernel on BASELINE.json's C1.

Workload (BASELINE.json configs[1], the metric's own config): the RTIOW cover
scene (grid 11 -> 484 bodies, generator seed 42) at 1200x675, 100 spp,
depth 50, fp32, render seed 1.  A "step" renders one full frame's share:

  * --scaling weak (default): every rank renders the whole 1200x675 frame
    with its own 100-sample stripe (samples [100*rank, 100*rank+100)), so
    per-GPU work is fixed; ranks share nothing (no collective on the data
    path; the RNG is keyed by (seed, pixel, sample)).
  * --scaling strong: the single 100-spp frame is split into interleaved
    8-row tiles, tile t on rank t % N (the north_star row-tile shard).

Inputs (scene table, camera) are resident in HBM before timing; the frame
stays on the device (host gather is not in `value`).  Timing: W untimed
warm-up steps, then K steps bracketed by barrier + synchronize, max over
ranks; kernel duration from HIP events on the launch stream.

Run:  python bench.py [--gpus N --steps K --warmup W]
      torchrun --nproc-per-node N bench.py --gpus N ...   (N > 1)
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import platform
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "raytracing-clj_amd"))

import torch  # noqa: E402  (first: librtclj.so then binds to torch's HIP runtime)
import torch.distributed as dist  # noqa: E402

import rtclj  # noqa: E402
from rtclj import scenes  # noqa: E402
from rtclj._lib import check, lib, rt_params  # noqa: E402
from rtclj.shard import shard_params, shard_rows  # noqa: E402

METRIC = "Mray-samples/sec at 1200×675×100spp depth50; achieved HBM GB/s vs peak"
# executed fp32 flops (fma = 2) of the BVH traversal, per event:
# node = 2 children x 6 slab planes x (sub + mul); leaf pair = 2 bodies x 16;
# exact body test (sqrt, root choice) = 4
FLOPS_NODE, FLOPS_LEAF_PAIR, FLOPS_EXACT = 24, 32, 4
PMC_DEFAULT = ROOT / "profiles" / "r01" / "pmc_v16k"
PEAK_FP32_TFLOPS = 157.3   # MI355X_MICROARCH.md: peak FP32 vector (= fp32 MFMA) rate
PEAK_HBM_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E peak (spec)
FLOPS_PER_SPHERE = 17      # per-body test, a and r^2 hoisted, fma = 2
FLOPS_PER_SEGMENT = 100    # per-segment hit/scatter/sky work (nominal)

WORKLOADS = {
    "c1": dict(width=1200, spp=100, depth=50, grid=11, name="C1 RTIOW cover 1200x675 100spp depth50"),
    "c2": dict(width=3840, spp=500, depth=50, grid=11, name="C2 cover 3840x2160 500spp depth50"),
    "c4": dict(width=7680, spp=2000, depth=64, grid=16, name="C4 cover(1025) 7680x4320 2000spp depth64"),
}


def parse():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scaling", choices=["weak", "strong"], default="weak")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c1")
    ap.add_argument("--spp", type=int, default=None, help="override the workload's spp (not a bench line)")
    ap.add_argument("--variant", type=int, default=0, help="kernel variant (rt_set_variant)")
    ap.add_argument("--lpp", type=int, default=0, help="lanes per pixel (rt_set_lanes_per_pixel; 0 auto)")
    ap.add_argument("--schedule", type=int, default=0,
                    help="tile schedule (rt_set_schedule): 0 adaptive longest-first, 1 plain dispatch order")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    ap.add_argument("--cpu-row-step", type=int, default=2, help="CPU baseline samples rows 0, s, 2s, ...")
    ap.add_argument("--cpu-threads", type=int, default=16)
    return ap.parse_args()


def cpu_baseline(scene, cam, w, h, spp, depth, seed, row_step, threads):
    """The oracle's fp64 reference-semantics mode (the C++ restatement of the
    Clojure path) on a bounded row sample of the same frame, on host cores."""
    sys.path.insert(0, str(ROOT))
    import numpy as np
    import oracle
    nthreads = max(1, min(threads, os.cpu_count() or 1))
    t0 = time.perf_counter()
    _, _, segs, samples = oracle.render(oracle.MODE_REF64, scene.sphere.astype(np.float64), scene.kind,
                                        scene.mat.astype(np.float64), cam.as_list(), cam.defocus, w, h, spp, depth,
                                        seed=seed, row_step=row_step, nthreads=nthreads)
    dt = time.perf_counter() - t0
    rows = (h + row_step - 1) // row_step
    cpu = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    # the reference's own setting: a pool of 2 threads (raytracing.clj:157),
    # on a 16x sparser row sample (about the same CPU time)
    step2 = row_step * 16
    t1 = time.perf_counter()
    _, _, _, samples2 = oracle.render(oracle.MODE_REF64, scene.sphere.astype(np.float64), scene.kind,
                                      scene.mat.astype(np.float64), cam.as_list(), cam.defocus, w, h, spp, depth,
                                      seed=seed, row_step=step2, nthreads=min(2, nthreads))
    dt2 = time.perf_counter() - t1
    return {"value": samples / dt / 1e6, "unit": "Mray-samples/s", "cores": nthreads, "kind": "port",
            "sample": f"rows 0,{row_step},{2 * row_step},... ({rows} rows x {w} px x {spp} spp = {samples} samples) "
                      f"of the same frame, fp64 reference semantics (oracle MODE_REF64), {dt:.1f} s",
            "seconds": dt, "segments_per_sample": segs / max(samples, 1), "cpu_model": cpu,
            "host": platform.node(),
            "two_threads": {"value": samples2 / dt2 / 1e6, "cores": min(2, nthreads),
                            "sample": f"every {step2}th row ({samples2} samples), {dt2:.1f} s: the reference's "
                                      f"pool-size 2 (raytracing.clj:157)"}}


# traversal variant -> (its stats build, body pairs per leaf)
BVH_STATS = {0: (17, 2), 16: (17, 2), 17: (17, 2), 18: (19, 4), 19: (19, 4), 11: (13, 1), 13: (13, 1), 14: (15, 1), 15: (15, 1)}


def bvh_counters(ds, cam, p, out, counters, sh, variant):
    """One untimed launch of the stats build of the same frame and traversal
    (variant 17 for the default 16, 13 for 11): per-segment node visits,
    leaf pair tests, exact tests (rt_debug_stats)."""
    sv, pairs_per_leaf = BVH_STATS[lib.rt_resolve_variant(ds)]
    old = lib.rt_set_variant(sv)
    try:
        dbg = (C.c_uint64 * 16)()
        check(lib.rt_debug_stats(dbg))                  # clear
        counters.zero_()
        check(lib.rt_launch(ds, C.byref(cam), C.byref(p), C.c_void_p(out.data_ptr()),
                            C.c_void_p(counters.data_ptr()), sh))
        torch.cuda.synchronize()
        check(lib.rt_debug_stats(dbg))
        segs = float(counters[0].item())
    finally:
        lib.rt_set_variant(old)
    wi = max(dbg[0], 1)
    return {"nodes": dbg[2] / segs, "leaf_pairs": pairs_per_leaf * dbg[3] / segs, "exact_tests": dbg[4] / segs,
            "stats_variant": sv,
            # wave-level events per wave loop iteration (what the VALU issues for)
            "per_wave_iter": {"wave_iters_per_sample": wi / max(float(counters[1].item()), 1.0),
                              "lanes_active": dbg[1] / wi / 64.0, "trav_steps": dbg[6] / wi,
                              "trav_lane_eff": dbg[7] / max(dbg[6], 1) / 64.0,
                              "leaf_passes": dbg[12] / wi, "exact_passes": dbg[13] / wi,
                              "random_unit_trips": dbg[14] / wi, "disk_trips": dbg[15] / wi}}


def _pmc_avg(passes, counters):
    """Per-dispatch averages of PMC counters over the timed kernel's launches
    (trace_kernel, not its stats build) in the committed rocprofv3 passes."""
    import csv
    acc = {}
    for name in passes:
        f = PMC_DEFAULT / f"{name}.csv"
        if not f.exists():
            return None
        for r in csv.DictReader(open(f)):
            if "trace_kernel" in r["Kernel_Name"] and "false>" in r["Kernel_Name"] and r["Counter_Name"] in counters:
                acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    if any(c not in acc for c in counters):
        return None
    return {c: sum(v) / len(v) for c, v in acc.items()}


def pmc_traffic():
    """HBM bytes per launch from the committed rocprofv3 PMC passes (separate
    FETCH_SIZE / WRITE_SIZE runs, KB units; gfx950 FETCH_SIZE counts half the
    bytes of wide streaming reads -> x2, MI355X_MICROARCH.md §HBM)."""
    v = _pmc_avg(("fetch", "write"), ("FETCH_SIZE", "WRITE_SIZE"))
    if v is None:
        return None, None
    return (2.0 * v["FETCH_SIZE"] + v["WRITE_SIZE"]) * 1024.0, str(PMC_DEFAULT.relative_to(ROOT))


def occupancy(ds, p, with_pmc, n_simd=1024, n_xcd=8):
    """Resident waves per SIMD: the launch's limit (HIP occupancy query with its
    dynamic LDS; VGPRs) and the measured mean over the timed kernel's launches
    from the committed PMC pass (SQ_WAVE_CYCLES in 4-cycle units summed over
    the SIMDs, vs GRBM_GUI_ACTIVE summed over the XCDs)."""
    o = (C.c_int * 4)()
    check(lib.rt_launch_occupancy(ds, C.byref(p), o))
    limit = min(8.0, o[0] * 4 / 4.0)   # 256-thread workgroups per CU x 4 waves / 4 SIMDs
    res = {"limit_waves_per_simd": limit, "workgroups_per_cu": o[0], "vgprs": o[1], "lds_bytes_per_wg": o[2],
           "lanes_per_pixel_shape": o[3], "hw_max_waves_per_simd": 8}
    v = _pmc_avg(("waves",), ("SQ_WAVE_CYCLES", "GRBM_GUI_ACTIVE")) if with_pmc else None
    if v is not None:
        mean = v["SQ_WAVE_CYCLES"] * 4.0 / n_simd / (v["GRBM_GUI_ACTIVE"] / n_xcd)
        res.update({"mean_waves_per_simd": mean, "frac_of_limit": mean / limit, "frac_of_hw_max": mean / 8.0,
                    "source": str(PMC_DEFAULT.relative_to(ROOT))})
    return res


def pmc_valu(n_simd=1024, n_xcd=8):
    """VALU issue picture of the same launches: the fraction of cycles each
    SIMD issues a VALU instruction (SQ_ACTIVE_INST_VALU, 4-cycle units,
    summed over the SIMDs, vs GRBM_GUI_ACTIVE summed over the XCDs) and the
    mean fraction of the 64 lanes active per VALU instruction."""
    v = _pmc_avg(("insts", "waves"), ("SQ_ACTIVE_INST_VALU", "SQ_INSTS_VALU", "SQ_THREAD_CYCLES_VALU",
                                      "GRBM_GUI_ACTIVE"))
    if v is None:
        return None
    busy = v["SQ_ACTIVE_INST_VALU"] * 4.0 / n_simd / (v["GRBM_GUI_ACTIVE"] / n_xcd)
    lanes = v["SQ_THREAD_CYCLES_VALU"] / v["SQ_INSTS_VALU"] / 64.0
    return {"issue_busy": busy, "lanes_active": lanes, "valu_insts": v["SQ_INSTS_VALU"],
            "source": str(PMC_DEFAULT.relative_to(ROOT)),
            "note": "the binding limit: VALU issue slots (a wave64 instruction takes 4 cycles whatever its "
                    "active lanes); issue_busy ~1 = every SIMD issues a VALU instruction every 4 cycles "
                    "(SQ_ACTIVE_INST_VALU counts per wave, so overlapping multi-cycle instructions can read "
                    "a little above 1); executed-flop frac = issue_busy x lanes_active x (flops per issued "
                    "lane-instruction)"}


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
    # traffic is the barrier and the max/sum of three timing scalars, done on
    # the host over gloo (BENCH_DIST_BACKEND=nccl moves them to RCCL).
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
    red_dev = dev if backend == "nccl" else torch.device("cpu")
    lib.rt_set_variant(a.variant)
    lib.rt_set_lanes_per_pixel(a.lpp)
    lib.rt_set_schedule(a.schedule)

    wl = dict(WORKLOADS[a.workload])
    if a.spp:
        wl["spp"] = a.spp
    W = wl["width"]
    H = rtclj.raytracing.image_height(W)
    spp, depth = wl["spp"], wl["depth"]
    scene = scenes.cover(wl["grid"], 42)
    cam = scenes.cover_camera(W, H)

    ds = C.c_void_p()
    check(lib.rt_scene_upload(device, C.byref(scene.c), C.byref(ds)))
    p = rt_params(**shard_params(world, rank, W, H, spp, depth, a.seed, a.scaling))
    rows = check(lib.rt_rows_out(C.byref(p)))
    assert rows == len(shard_rows(H, p.row_tile or 8, p.tile_first, p.tile_step))
    out = torch.empty(rows * W * 3, dtype=torch.float32, device=dev)
    counters = torch.zeros(2, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)
    sh = C.c_void_p(stream.cuda_stream)

    def step():
        check(lib.rt_launch(ds, C.byref(cam), C.byref(p), C.c_void_p(out.data_ptr()),
                            C.c_void_p(counters.data_ptr()), sh))

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    counters.zero_()
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps)]
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(a.steps):
        starts[k].record(stream)
        step()
        ends[k].record(stream)
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = [s.elapsed_time(e) for s, e in zip(starts, ends)]
    cnt = counters.to("cpu").tolist()
    local_stats = torch.tensor([elapsed, max(kern_ms), sum(kern_ms) / len(kern_ms)], dtype=torch.float64)
    tot = torch.tensor([float(cnt[0]), float(cnt[1])], dtype=torch.float64)
    if world > 1:
        ls, tt = local_stats.to(red_dev), tot.to(red_dev)
        dist.all_reduce(ls, op=dist.ReduceOp.MAX)
        dist.all_reduce(tt, op=dist.ReduceOp.SUM)
        local_stats, tot = ls.cpu(), tt.cpu()
    elapsed, kern_max_ms, kern_avg_ms = local_stats.tolist()
    segs_total, samples_total = tot.tolist()
    bvh = (bvh_counters(ds, cam, p, out, counters, sh, a.variant)
           if rank == 0 and lib.rt_resolve_variant(ds) in BVH_STATS else None)
    # the committed PMC passes were taken on C1's default launch: only that
    # workload's line quotes them
    pmc_ok = a.workload == "c1" and not a.spp and a.variant == 0 and a.lpp == 0 and a.scaling == "weak"
    occ = occupancy(ds, p, pmc_ok) if rank == 0 else None
    lib.rt_scene_free(ds)

    if rank == 0:
        samples_per_step = samples_total / a.steps
        value = samples_per_step * a.steps / elapsed / 1e6
        seg_per_sample = segs_total / max(samples_total, 1)
        # dominant kernel, per launch on this rank (rank-0 share at N>1)
        launch_samples = rows * W * spp
        launch_segs = seg_per_sample * launch_samples
        bf_flops = launch_segs * (FLOPS_PER_SPHERE * len(scene) + FLOPS_PER_SEGMENT)
        bf_tflops = bf_flops / (kern_avg_ms * 1e-3) / 1e12
        if bvh is not None:
            per_seg = (FLOPS_NODE * bvh["nodes"] + FLOPS_LEAF_PAIR * bvh["leaf_pairs"] +
                       FLOPS_EXACT * bvh["exact_tests"] + FLOPS_PER_SEGMENT)
            work = (f"BVH traversal, executed fp32 work per segment = 24 x {bvh['nodes']:.2f} nodes + "
                    f"32 x {bvh['leaf_pairs']:.2f} leaf pairs (the big bodies' leaf included) + "
                    f"4 x {bvh['exact_tests']:.2f} exact tests + 100 = {per_seg:.0f} flops "
                    f"(counters: one untimed stats launch)")
        else:
            per_seg = FLOPS_PER_SPHERE * len(scene) + FLOPS_PER_SEGMENT
            work = f"linear scan, executed fp32 work per segment = 17 x {len(scene)} bodies + 100"
        tflops = launch_segs * per_seg / (kern_avg_ms * 1e-3) / 1e12
        hbm_bytes = rows * W * 12 + len(scene) * 32
        gbs = hbm_bytes / (kern_avg_ms * 1e-3) / 1e9
        traffic, traffic_src = pmc_traffic() if pmc_ok else (None, "no committed PMC pass for this workload")
        res = {
            "metric": METRIC, "value": value, "unit": "Mray-samples/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": elapsed / a.steps * 1e3, "higher_is_better": True,
            "scaling": a.scaling, "vs_baseline": None, "dtype": "fp32",
            "data": f"synthetic: RTIOW cover scene (grid {wl['grid']}, {len(scene)} bodies, generator seed 42), "
                    f"render seed {a.seed}",
            "config": {"workload": wl["name"] if not a.spp else f"{wl['name']} (spp override {spp})",
                       "width": W, "height": H, "spp_per_gpu": spp, "max_depth": depth, "bodies": len(scene),
                       "parallelism": ("sample-stripe x%d (weak)" % world) if a.scaling == "weak"
                       else ("row-tile 8 x%d (strong)" % world), "variant": a.variant,
                       "tile_schedule": "adaptive longest-first" if a.schedule == 0 else "dispatch order"},
            "roofline": {"bound": "mfma", "achieved": tflops, "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                         "frac": tflops / PEAK_FP32_TFLOPS, "traffic": traffic,
                         "note": f"compute-bound fp32 on the VALU (branchy per-ray FP work, no GEMM shape: MFMA unused); "
                                 f"peak = the fp32 dense peak (vector = MFMA for fp32); {work}. "
                                 f"Brute-force-equivalent (SURVEY §8d: 17 x {len(scene)} + 100 per segment): "
                                 f"{bf_tflops:.1f} TF/s. traffic = HBM bytes/launch from {traffic_src} "
                                 f"(FETCH x2 + WRITE)"},
            "hbm_roofline": {"bound": "hbm", "achieved": gbs, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                             "frac": gbs / PEAK_HBM_GBS, "traffic": traffic,
                             "note": "non-binding: algorithmic bytes/launch = W*rows*12 (fp32 RGB) + bodies*32"},
            "valu": pmc_valu() if pmc_ok else None,
            "occupancy": occ,
            "bvh_per_segment": bvh,
            "kernel_ms_avg": kern_avg_ms, "kernel_ms_max": kern_max_ms,
            "segments_per_sample": seg_per_sample, "samples_per_step": samples_per_step,
            "kernel": "rtclj::trace_kernel<SRC,SCAN,LPP> (variant %d; default = 16: BVH with 4-body leaves in LDS, 8x8-pixel sample pool per workgroup)" % a.variant,
            "cpu_baseline": None,
        }
        if a.cpu_baseline == "auto" and world == 1:
            res["cpu_baseline"] = cpu_baseline(scene, cam, W, H, spp, depth, a.seed, a.cpu_row_step, a.cpu_threads)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
