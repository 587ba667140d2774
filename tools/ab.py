#!/usr/bin/env python3
"""A/B kernel variants on one GPU, interleaved rounds in one process
(cdna_hip_programming.md §5.4 rule 24).  Prints per-variant median/min kernel
ms and Msamples/s on a BASELINE workload, checks every variant's frame is
bit-identical to the first, and decodes the stats build (variant 3).
--persistent launches through rt_launch on one uploaded scene (as bench.py
does), so the adaptive tile order applies after each variant's first launch
(one untimed warm-up launch per variant and round).

  python tools/ab.py --variants 1 2 3 --rounds 3 [--width 1200 --spp 100]
"""
import argparse
import ctypes as C
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "raytracing-clj_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (before the library: torch's HIP runtime must serve the process)

from rtclj import raytracing as R, scenes  # noqa: E402
from rtclj._lib import check, diag_lib  # noqa: E402

lib = diag_lib()   # the diagnostic build holds every variant (same ABI, same bits)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", nargs="+", default=["16", "18"], help="kernel variants, e.g. 16 17 11")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--width", type=int, default=1200)
    ap.add_argument("--spp", type=int, default=100)
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--grid", type=int, default=11)
    ap.add_argument("--scene", choices=["cover", "reference"], default="cover")
    ap.add_argument("--json", default=None)
    ap.add_argument("--persistent", action="store_true",
                    help="rt_launch on one uploaded scene (adaptive tile order active), like bench.py")
    a = ap.parse_args()
    w = a.width
    h = R.image_height(w)
    if a.scene == "cover":
        sc, cam = scenes.cover(a.grid), scenes.cover_camera(w, h)
    else:
        sc, cam = R.Scene.from_bodies(R.hittables), R.camera(w, h, **R.REFERENCE_CAMERA)
    if a.persistent:
        import torch
        from rtclj._lib import rt_params
        ds = C.c_void_p()
        check(lib.rt_scene_upload(0, C.byref(sc.c), C.byref(ds)))
        p = rt_params(width=w, height=h, row_begin=0, row_end=h, spp=a.spp, max_depth=a.depth, seed=1)
        out = torch.empty(h * w * 3, dtype=torch.float32, device="cuda")
        cnt = torch.zeros(2, dtype=torch.int64, device="cuda")
        stream = torch.cuda.current_stream()

        def launch(v, st):
            # warm-up: records this variant's tile durations for the timed launch's order
            check(lib.rt_launch(ds, C.byref(cam), C.byref(p), C.c_void_p(out.data_ptr()), None,
                                C.c_void_p(stream.cuda_stream)))
            if v in (3, 6, 7, 10, 13, 15, 17, 19):
                check(lib.rt_debug_stats((C.c_uint64 * 32)()))   # count the timed launch only
            cnt.zero_()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            check(lib.rt_launch(ds, C.byref(cam), C.byref(p), C.c_void_p(out.data_ptr()),
                                C.c_void_p(cnt.data_ptr()), C.c_void_p(stream.cuda_stream)))
            e1.record(stream)
            torch.cuda.synchronize()
            st["kernel_ms"] = e0.elapsed_time(e1)
            st["segments"], st["samples"] = int(cnt[0]), int(cnt[1])
            return out.cpu().numpy().reshape(h, w, 3)
    cfgs = [int(x) for x in a.variants]
    names = a.variants
    times = {v: [] for v in names}
    ref = None
    stats = {}
    for r in range(a.rounds):
        for name, v in zip(names, cfgs):
            check(lib.rt_set_variant(v))
            st = {}
            if a.persistent:
                img = launch(v, st)
            else:
                img = R.render(sc, cam, w, h, spp=a.spp, max_depth=a.depth, seed=1, stats=st, library=lib)
            times[name].append(st["kernel_ms"])
            stats[name] = st
            if ref is None:
                ref = img
            elif not np.array_equal(img, ref):
                print(f"variant {name}: frame differs from variant {names[0]}!", flush=True)
                sys.exit(1)
            if v in (3, 6, 7, 10, 13, 15, 17, 19):
                d = (C.c_uint64 * 32)()
                check(lib.rt_debug_stats(d))
                d = list(d)
                stats["dbg"] = d
                stats["dbg_variant"] = name
                nw = int(d[5])
                wv = np.zeros(4 * 65536, np.uint64)
                check(lib.rt_debug_waves(0, wv.ctypes.data_as(C.POINTER(C.c_uint64)), 65536))
                stats["waves"] = wv.reshape(-1, 4)[:nw].copy()
    out = {"workload": f"{a.scene} {w}x{h} spp{a.spp} depth{a.depth}", "variants": {}}
    samples = w * h * a.spp
    for v in names:
        med = statistics.median(times[v])
        out["variants"][v] = {"median_ms": med, "min_ms": min(times[v]), "Msamples_s": samples / med / 1e3,
                              "all_ms": times[v]}
        print(f"variant {v}: median {med:8.3f} ms  min {min(times[v]):8.3f}  {samples / med / 1e3:8.1f} Msamples/s")
    seg = stats[names[0]]["segments"] / stats[names[0]]["samples"]
    print(f"segments/sample {seg:.4f}")
    if "dbg" in stats:
        it, lanes, sph, blk, blk_lanes, waves = stats["dbg"][:6]
        segs_total = stats[names[0]]["segments"]
        if stats["dbg_variant"] in ("13", "15", "17", "19"):
            tw, tl = stats["dbg"][6], stats["dbg"][7]
            print(json.dumps({"bvh_nodes_per_segment": sph / segs_total, "bvh_leaves_per_segment": blk / segs_total,
                              "bvh_considers_per_segment": blk_lanes / segs_total,
                              "trav_wave_iters_per_wave_iter": tw / it, "trav_lane_eff": tl / max(64 * tw, 1),
                              "trav_lanes_active_frac_of_loop_lanes": tl / max(tw * (lanes / it), 1),
                              "leaf_passes_per_trav_iter": stats["dbg"][12] / max(tw, 1),
                              "exact_passes_per_trav_iter": stats["dbg"][13] / max(tw, 1),
                              "lanes_per_leaf_pass": blk / max(stats["dbg"][12], 1),
                              "lanes_per_exact_pass": blk_lanes / max(stats["dbg"][13], 1)}))
        info = {"wave_iters": it, "simd_eff_loop": lanes / (64 * it), "iters_per_wave": it / waves,
                "block_rate": blk / max(sph, 1), "lanes_per_block": blk_lanes / max(blk, 1), "waves": waves}
        wv = stats["waves"]
        t0 = wv[:, 0].min()
        st_, en = (wv[:, 0] - t0) / 100.0, (wv[:, 1] - t0) / 100.0    # us
        life = en - st_
        grid = np.linspace(0, en.max(), 41)
        occ = [int(((st_ <= g) & (en > g)).sum()) for g in grid]
        cu = ((wv[:, 2] >> 8) & 0xF) | (((wv[:, 2] >> 13) & 0x3) << 4) | (((wv[:, 2] >> 12) & 1) << 6)
        xcc = wv[:, 3] & 0xF
        info.update(kernel_us=float(en.max()), life_us_mean=float(life.mean()), life_us_max=float(life.max()),
                    life_us_min=float(life.min()), resident_waves_over_time=occ,
                    max_resident=int(max(occ)), start_last_us=float(st_.max()),
                    distinct_cu_xcc=int(len(set(zip(cu.tolist(), xcc.tolist())))))
        cyc = stats["dbg"][8:12]
        tot = max(sum(cyc), 1)
        info["clock_split"] = {"camera": cyc[0] / tot, "hit_search": cyc[1] / tot, "shade": cyc[2] / tot,
                               "accumulate": cyc[3] / tot}
        info["variant"] = stats["dbg_variant"]
        out["stats"] = info
        print(json.dumps(info))
    if a.json:
        Path(a.json).write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
