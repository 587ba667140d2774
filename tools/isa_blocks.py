#!/usr/bin/env python3
"""Per-block VALU counts of a trace kernel from the marked ISA listing
(make -C raytracing-clj_amd isa-marks: RT_MARK in trace_kernel.h), priced by
tools/isa_cost.py's issue classes, and -- with the statistics build's events
per wave iteration (a bench.py line's stats_build.per_wave_iter) -- the
estimated VALU instructions and busy quad-cycles per wave iteration by block
(DESIGN.md §9).  An instruction belongs to the last marker above it in the
listing (layout order), so a block's count is its static code: a loop inside a
block (the claim loop of refill, the compaction step's scan) counts once.

  python tools/isa_blocks.py [--isa lib/isa/trace_marks.s] [--kernel NAME_SUBSTR]
                             [--bench line.json] [--pmc-valu-per-iter N]
"""
import argparse
import json
import re
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tools"))
from isa_cost import classify  # noqa: E402

# variant 22: trace_kernel<SRC_LDS, SCAN_BVHQ7, false, 4, 0>
DEFAULT_KERNEL = "_ZN5rtclj12trace_kernelILi1ELi8ELb0ELi4ELi0EEEvNS_5KArgsE"


# blocks whose code the compiler copies per call site (the leaf lambda is
# inlined at the big-body loop and at both leaf children of a node step): one
# pass runs one copy, so a pass costs the smallest copy; what a larger copy
# holds beyond it is code the compiler laid out there -- in the big-body
# loop's copy of `exact`, the tree walk's ray set-up (slab offsets, 1/u,
# padding: read from the listing), which runs once per segment -- and goes to
# EXCESS_TO
PER_COPY = ("leaf", "exact_tail", "exact", "exact_accept")
EXCESS_TO = "tree_setup"
TAIL_SPLIT = re.compile(r"v_bitop3_b32.*bitop3:0xa8")


def blocks(isa, kernel):
    lines = Path(isa).read_text().split("\n")
    start = next(i for i, ln in enumerate(lines) if ln.startswith(kernel + ":"))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    cur = "prologue"
    out = {}
    copies = {}   # per PER_COPY block: one count dict per copy
    zero = {"D": 0, "S": 0, "T": 0, "SALU": 0}
    hot = cur   # the last block before a "cold" marker
    for ln in lines[start:end]:
        m = re.search(r";@@ (\w+)", ln)
        if m:
            cur = m.group(1)
            if cur != "cold":
                hot = cur
            if cur in PER_COPY:
                copies.setdefault(cur, []).append(dict(zero))
            continue
        # a rare branch ("cold") is its own basic block: the next label goes
        # back to the block it branched from
        if cur == "cold" and re.match(r"\.LBB", ln):
            cur = hot   # (a PER_COPY block goes on in the same copy)
        # the exact-test loop is rotated: its tail (root choice, acceptance,
        # the next candidate) is laid out right after the leaf pass, whose
        # last instruction merges the candidate mask (v_bitop3 0xa8)
        if cur == "leaf" and TAIL_SPLIT.search(ln):
            k0 = classify(ln)
            if k0:
                copies["leaf"][-1][k0] += 1
            cur = hot = "exact_tail"
            copies.setdefault(cur, []).append(dict(zero))
            continue
        k = classify(ln)
        b = copies[cur][-1] if cur in PER_COPY else out.setdefault(cur, dict(zero))
        if k:
            b[k] += 1
        elif re.match(r"\s+s_", ln):
            b["SALU"] += 1
    for k, cs in copies.items():
        small = min(cs, key=lambda c: c["D"] + c["S"] + c["T"])
        out[k] = dict(small, copies=len(cs))
        ex = out.setdefault(EXCESS_TO, dict(zero))
        for c in cs:
            for f in zero:
                ex[f] += c[f] - small[f]
    return out


def qc(b):
    """busy quad-cycles of one pass: dual-issuable 0.5, single-port 1, transcendental 2"""
    return b["D"] * 0.5 + b["S"] + 2 * b["T"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--isa", default=str(ROOT / "raytracing-clj_amd" / "lib" / "isa" / "trace_marks.s"))
    ap.add_argument("--kernel", default=DEFAULT_KERNEL)
    ap.add_argument("--bench", default=None, help="a bench.py JSON line with stats_build (events per wave iteration)")
    ap.add_argument("--pmc-valu-per-iter", type=float, default=None,
                    help="measured VALU instructions per wave iteration (PMC SQ_INSTS_VALU / wave iterations)")
    ap.add_argument("--iters-per-wave", type=float, default=69.0,
                    help="wave iterations per wave (C1: 3.53 M per launch over 12,750 tiles x 4 waves)")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    bl = blocks(a.isa, a.kernel)
    print(f"{'block':18s} {'D':>5s} {'S':>5s} {'T':>3s} {'VALU':>5s} {'quad-cycles':>11s} {'SALU':>5s}")
    for k, b in bl.items():
        note = f"  (one copy of {b['copies']}; the rest in {EXCESS_TO})" if "copies" in b else ""
        print(f"{k:18s} {b['D']:5.0f} {b['S']:5.0f} {b['T']:3.0f} {b['D'] + b['S'] + b['T']:5.0f} {qc(b):11.1f} "
              f"{b['SALU']:5.0f}{note}")
    res = {"static": bl}
    if a.bench:
        line = json.loads(Path(a.bench).read_text().strip().splitlines()[-1])
        pw = line["stats_build"]["per_wave_iter"]
        # events per wave iteration of each block (the statistics build's
        # counters; 1 = once per wave iteration)
        # once per wave (prologue, epilogue, the compaction step, the outer
        # loop): 1 / (wave iterations per wave), from the frame's units
        per_wave = 1.0 / a.iters_per_wave
        ev = {"iteration": 1.0, "camera": pw["fresh_blocks"], "setup": 1.0, "bigleaf": 1.0, "tree_setup": 1.0,
              "node": pw["trav_steps"], "leaf": pw["leaf_passes"], "exact": pw["exact_passes"],
              "exact_accept": pw["exact_passes"], "exact_tail": pw["exact_passes"], "hit": 1.0,
              "lambert_metal": pw["lambert_metal_blocks"], "dielectric": pw["dielectric_blocks"],
              "sums": pw.get("sums_blocks", 1.0), "refill": pw.get("refills", 1.0), "claim": pw.get("claims", 1.0),
              "drain_check": pw.get("drain_checks", 1.0),
              "compaction": 1.0, "loop": per_wave, "epilogue": per_wave, "prologue": per_wave,
              "compact_step": per_wave, "rejection_disk": 0.0, "rejection_sphere": 0.0, "cold": 0.0}
        tot_v = tot_q = 0.0
        rows = []
        for k, b in bl.items():
            e = ev.get(k, 0.0)
            v = e * (b["D"] + b["S"] + b["T"])
            q = e * qc(b)
            tot_v += v
            tot_q += q
            rows.append((k, e, v, q))
        print(f"\nper wave iteration (events x static count; {line['stats_build']['stats_variant']}'s counters):")
        print(f"{'block':18s} {'events':>7s} {'VALU':>7s} {'quad-cyc':>8s} {'share':>6s}")
        for k, e, v, q in sorted(rows, key=lambda r: -r[3]):
            if e:
                print(f"{k:18s} {e:7.2f} {v:7.1f} {q:8.1f} {q / tot_q:6.1%}")
        print(f"{'total':18s} {'':7s} {tot_v:7.1f} {tot_q:8.1f}")
        if a.pmc_valu_per_iter:
            print(f"measured (PMC) VALU per wave iteration {a.pmc_valu_per_iter:.1f}: the estimate covers "
                  f"{tot_v / a.pmc_valu_per_iter:.1%}")
        res["per_wave_iter"] = {k: {"events": e, "valu": v, "quad_cycles": q} for k, e, v, q in rows}
        res["total_valu"] = tot_v
        res["total_quad_cycles"] = tot_q
    if a.json:
        Path(a.json).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
