#!/usr/bin/env python3
"""Bit-equality of two kernel variants on the GPU (an A/B candidate against
the default): renders the same frames under each and compares the float
bits and the segment counts.  Cases: C1's frame at 16 spp, ragged sizes, a
row range, eight shards on device 0 (split launches), realm, spp > 255
(wrap counts).  RTCLJ_LIBRARY selects the build.

  python tools/variant_eq.py --a 22 --b 24
"""
import argparse
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "raytracing-clj_amd"))
from rtclj import raytracing as R, scenes  # noqa: E402
from rtclj._lib import RT_FLAG_REALM, RT_FLAG_SHARDS_ON_DEVICE0, lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--a", type=int, default=22)
    ap.add_argument("--b", type=int, default=24)
    a = ap.parse_args()
    cover = scenes.cover(11)
    ref = R.Scene.from_bodies(R.hittables)
    cases = [
        ("c1 16spp", cover, scenes.cover_camera(1200, 675), 1200, 675, dict(spp=16)),
        ("ragged 37x21", ref, R.camera(37, 21, **R.REFERENCE_CAMERA), 37, 21, dict(spp=9, max_depth=10)),
        ("rows 100-333", cover, scenes.cover_camera(640, 360), 640, 360, dict(spp=12, rows=(100, 333))),
        ("8 shards", cover, scenes.cover_camera(1200, 675), 1200, 675,
         dict(spp=24, n_devices=8, flags=RT_FLAG_SHARDS_ON_DEVICE0)),
        ("realm", ref, R.camera(200, 112, **R.REFERENCE_CAMERA), 200, 112, dict(spp=8, flags=RT_FLAG_REALM)),
        ("spp 300", cover, scenes.cover_camera(96, 54), 96, 54, dict(spp=300)),
        ("c4 scene", scenes.cover_c4(), scenes.cover_camera(320, 180), 320, 180, dict(spp=40, max_depth=64)),
        ("c4 scene rows", scenes.cover_c4(), scenes.cover_camera(7680, 4320), 7680, 4320,
         dict(spp=4, max_depth=64, rows=(2000, 2040))),
    ]
    bad = 0
    for name, sc, cam, w, h, kw in cases:
        outs = []
        for v in (a.a, a.b):
            old = lib.rt_set_variant(v)
            assert old >= 0, lib.rt_last_error()
            st = {}
            img = R.render(sc, cam, w, h, seed=5, stats=st, **kw)
            lib.rt_set_variant(old)
            outs.append((img, st))
        (x, sx), (y, sy) = outs
        eq = x.shape == y.shape and np.array_equal(x.view(np.uint32), y.view(np.uint32))
        seg = sx.get("segments") == sy.get("segments")
        print(f"{name:14s} bits {'equal' if eq else 'DIFFER'}  segments {sx.get('segments')} / {sy.get('segments')}"
              f"  variants {sx.get('variant')} / {sy.get('variant')}", flush=True)
        bad += (not eq) + (not seg)
    print("ALL EQUAL" if bad == 0 else f"{bad} MISMATCHES")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
