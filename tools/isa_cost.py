#!/usr/bin/env python3
"""Price gfx950 ISA lines by VALU issue class (profiles/r05/valu_cost.txt):
D = dual-issuable full-rate op (0.5 quad-cycle when paired), S = single-port
(1 quad-cycle), T = transcendental (2).  Prints per-range counts.
  python tools/isa_cost.py file.s start:end [start:end ...]
"""
import re
import sys

DUAL = {"v_fma_f32", "v_fmac_f32", "v_add_f32", "v_sub_f32", "v_subrev_f32", "v_mul_f32", "v_fmamk_f32",
        "v_fmaak_f32", "v_mov_b32", "v_add_u32", "v_sub_u32", "v_subrev_u32", "v_and_b32", "v_or_b32", "v_xor_b32",
        "v_not_b32", "v_bitop3_b32", "v_lshrrev_b32", "v_ashrrev_i32", "v_lshlrev_b16"}
TRANS = {"v_sqrt_f32", "v_rcp_f32", "v_rsq_f32", "v_exp_f32", "v_log_f32"}


def classify(line):
    m = re.match(r"\s+(v_[a-z0-9_]+)", line)
    if not m:
        return None
    op = m.group(1)
    base = re.sub(r"_(e32|e64|sdwa|dpp)$", "", op)
    if base in TRANS:
        return "T"
    if base in DUAL:
        # any SGPR source operand makes an instruction single-port (measured:
        # v_fma/add/mul/sub_f32, v_add_u32, v_xor, v_bitop3 with an SGPR
        # operand all take a whole quad-cycle; inline constants and literals do not)
        ops = line.split(";")[0].split(None, 1)[1] if len(line.split(None, 1)) > 1 else ""
        srcs = ops.split(",")[1:]
        if any(re.match(r"\s*-?\|?(s\d+|s\[|vcc|exec)", x) for x in srcs):
            return "S"
        return "D"
    if base.startswith("v_readlane") or base.startswith("v_writelane") or base.startswith("v_readfirstlane"):
        return "S"
    return "S"


def main():
    lines = open(sys.argv[1]).read().split("\n")
    verbose = "-v" in sys.argv
    for rng in [x for x in sys.argv[2:] if x != "-v"]:
        a, b = (int(x) for x in rng.split(":"))
        c = {"D": 0, "S": 0, "T": 0}
        salu = 0
        for ln in lines[a - 1:b]:
            k = classify(ln)
            if k:
                c[k] += 1
                if verbose and k != "D":
                    print(f"      {k} {ln.strip()}")
            elif re.match(r"\s+s_", ln):
                salu += 1
        q = c["D"] * 0.5 + c["S"] + 2 * c["T"]
        print(f"{rng:>12}: D {c['D']:3d}  S {c['S']:3d}  T {c['T']:2d}  -> {q:6.1f} quad-cycles (paired)  "
              f"{c['D'] + c['S'] + 2 * c['T']:4d} (unpaired)   SALU/branch {salu}")


if __name__ == "__main__":
    main()
