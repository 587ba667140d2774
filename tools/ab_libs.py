#!/usr/bin/env python3
"""A/B whole library builds on one GPU: alternates `bench.py` runs (one
process each, RTCLJ_LIBRARY selects the build) for R rounds and prints the
median kernel ms per build.  Every run has its own time limit; the first
failing run ends the script (no retries).

  python tools/ab_libs.py --libs raytracing-clj_amd/lib/ab_base.so raytracing-clj_amd/lib/librtclj.so \
      --rounds 3 [--out gpurun_out/ab.jsonl] [-- extra bench.py args]
"""
import argparse
import json
import os
import statistics
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def main():
    argv = sys.argv[1:]
    extra = []
    if "--" in argv:
        k = argv.index("--")
        argv, extra = argv[:k], argv[k + 1:]
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", nargs="+", required=True)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--out", default=None)
    ap.add_argument("--variants", nargs="+", type=int, default=None,
                    help="per --libs entry: its bench.py --variant (default 0 for every one)")
    a = ap.parse_args(argv)
    variants = a.variants or [0] * len(a.libs)
    assert len(variants) == len(a.libs), "--variants: one per --libs entry"
    runs = [(lib, v, f"{Path(lib).name}:v{v}" if v else Path(lib).name) for lib, v in zip(a.libs, variants)]
    res = {name: [] for _, _, name in runs}
    res_plain = {name: [] for _, _, name in runs}   # dispatch_order: the frame in plain tile order
    out = open(a.out, "a") if a.out else None
    for r in range(a.rounds):
        for lib, v, name in runs:
            env = dict(os.environ, RTCLJ_LIBRARY=str(Path(lib).resolve()))
            cmd = [sys.executable, str(ROOT / "bench.py"), "--cpu-baseline", "off", "--steps", str(a.steps),
                   "--warmup", "2", "--variant", str(v)] + extra
            p = subprocess.run(["timeout", "-k", "10", "240"] + cmd, env=env, capture_output=True, text=True)
            if p.returncode != 0:
                print(f"run failed ({p.returncode}) for {lib}:\n{p.stderr[-3000:]}", flush=True)
                sys.exit(p.returncode)
            line = json.loads(p.stdout.strip().splitlines()[-1])
            ms = line["kernel_ms_avg"]
            res[name].append(ms)
            plain = (line.get("dispatch_order") or {}).get("kernel_ms")
            if plain is not None:
                res_plain[name].append(plain)
            print(f"round {r} {name:24s} kernel {ms:.3f} ms  plain order {plain}  "
                  f"{line['value']:.0f} Msamples/s", flush=True)
            if out:
                out.write(json.dumps({"round": r, "lib": name, "kernel_ms_avg": ms, "occupancy": line.get("occupancy"),
                                      "value": line["value"], "bvh": line.get("bvh_per_segment"),
                                      "plain_ms": plain,
                                      "args": extra}) + "\n")
                out.flush()
    for name, v in res.items():
        print(f"{name:24s} median {statistics.median(v):.3f} ms  min {min(v):.3f}  runs {v}")
        if res_plain[name]:
            print(f"{name:24s} plain order median {statistics.median(res_plain[name]):.3f} ms")


if __name__ == "__main__":
    main()
