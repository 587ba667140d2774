#!/usr/bin/env python3
"""Summarise committed rocprofv3 PMC passes (profiles/pmc.sh) of the product
kernel: per-dispatch medians of every counter over trace_kernel<..., false>
launches, plus the derived VALU / occupancy / HBM figures bench.py reports.

  python tools/pmc_summary.py profiles/r02/pmc_c1 [kernel_stats.csv]
"""
import csv
import re
import statistics
import sys
from pathlib import Path


def main():
    d = Path(sys.argv[1])
    acc = {}
    for f in sorted(d.glob("*.csv")):
        for r in csv.DictReader(open(f)):
            if re.search(r"trace_kernel<[^>]*\bfalse\b", r["Kernel_Name"]):
                acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    # the median launch, as bench.py takes it (the timed frames' recorded order)
    avg = {k: statistics.median(v) for k, v in acc.items()}
    lines = [f"== {d}  (per-dispatch averages over the product kernel's launches)"]
    for k in sorted(avg):
        lines.append(f"  {k:26s} {avg[k]:.4g}")
    g = avg.get("GRBM_GUI_ACTIVE")
    if g:
        cyc = g / 8
        if "SQ_ACTIVE_INST_VALU2" in avg:
            busy = avg["SQ_ACTIVE_INST_VALU"] - avg["SQ_ACTIVE_INST_VALU2"]
            lines.append(f"  valu_busy    = (ACTIVE_INST_VALU - ACTIVE_INST_VALU2) / (1024 SIMDs x cycles/4) = "
                         f"{busy / (1024 * cyc / 4):.3f}")
            lines.append(f"  dual_issue   = ACTIVE_INST_VALU2 / busy quad-cycles = {avg['SQ_ACTIVE_INST_VALU2'] / busy:.3f}")
        if "SQ_INSTS_VALU" in avg:
            lines.append(f"  valu_pipe_util = SQ_INSTS_VALU*2 / (1024 x cycles) = {avg['SQ_INSTS_VALU'] * 2 / 1024 / cyc:.3f}")
        if "SQ_INSTS_SALU" in avg and "SQ_INSTS_VALU" in avg:
            lines.append(f"  salu_per_valu = {avg['SQ_INSTS_SALU'] / avg['SQ_INSTS_VALU']:.3f}")
        if "SQ_WAIT_ANY" in avg and "SQ_WAVE_CYCLES" in avg:
            wc = avg["SQ_WAVE_CYCLES"]
            lines.append(f"  wait_dep {avg['SQ_WAIT_ANY'] / wc:.3f}  wait_issue {avg['SQ_WAIT_INST_ANY'] / wc:.3f}  "
                         f"issuing {avg.get('SQ_ACTIVE_INST_ANY', 0) / wc:.3f} (of wave residency)")
        if "SQ_WAVE_CYCLES" in avg:
            lines.append(f"  waves/SIMD   = SQ_WAVE_CYCLES*4/1024 / (GRBM_GUI_ACTIVE/8) = "
                         f"{avg['SQ_WAVE_CYCLES'] * 4 / 1024 / cyc:.3f}")
    if "SQ_THREAD_CYCLES_VALU" in avg and "SQ_INSTS_VALU" in avg:
        lines.append(f"  lanes_active = SQ_THREAD_CYCLES_VALU / SQ_INSTS_VALU / 64 = "
                     f"{avg['SQ_THREAD_CYCLES_VALU'] / avg['SQ_INSTS_VALU'] / 64:.3f}")
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        lines.append(f"  HBM bytes/launch = FETCH_SIZE*2 + WRITE_SIZE (KB units) = "
                     f"{(2 * avg['FETCH_SIZE'] + avg['WRITE_SIZE']) * 1024 / 1e6:.3f} MB")
    if len(sys.argv) > 2:
        for r in csv.DictReader(open(sys.argv[2])):
            if "trace_kernel" in r.get("Name", ""):
                lines.append(f"  kernel {r['Name'][:60]}: calls {r['Calls']} avg {float(r['AverageNs']) / 1e6:.3f} ms")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
