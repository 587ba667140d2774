#!/usr/bin/env python3
"""Per-launch PMC counters of the trace kernel from rocprofv3 counter CSVs
(one per pass, e.g. of tools/launch_frames.py): for each file, each
counter's value per trace_kernel dispatch, in dispatch order, and the HBM
bytes per launch (FETCH_SIZE x 2 + WRITE_SIZE, KB units; the gfx950 x2 of
MI355X_MICROARCH.md) of the last dispatch when both are present.

  python tools/pmc_frames.py DIR/*.csv
"""
import csv
import json
import sys
from collections import defaultdict


def main():
    per = defaultdict(dict)   # counter -> {dispatch: value}
    for f in sys.argv[1:]:
        for r in csv.DictReader(open(f)):
            kn = r["Kernel_Name"]
            if not ("trace_kernel" in kn or "sorted_kernel" in kn) or ("trace_kernel" in kn and "true>" in kn):
                continue
            d = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0)
            c = r["Counter_Name"]
            per[c][d] = per[c].get(d, 0.0) + float(r["Counter_Value"])
    res = {c: [v[k] for k in sorted(v)] for c, v in per.items()}
    if "FETCH_SIZE" in res and "WRITE_SIZE" in res:
        res["hbm_bytes_last"] = (2.0 * res["FETCH_SIZE"][-1] + res["WRITE_SIZE"][-1]) * 1024.0
        res["write_bytes_last"] = res["WRITE_SIZE"][-1] * 1024.0
        res["fetch_bytes_x2_last"] = res["FETCH_SIZE"][-1] * 2048.0
    if "SQ_INSTS_VALU" in res and "SQ_THREAD_CYCLES_VALU" in res:
        res["lanes_active_last"] = res["SQ_THREAD_CYCLES_VALU"][-1] / res["SQ_INSTS_VALU"][-1] / 64.0
    if "SQ_ACTIVE_INST_VALU" in res and "GRBM_GUI_ACTIVE" in res:
        res["issue_busy_last"] = res["SQ_ACTIVE_INST_VALU"][-1] * 4.0 / 1024 / (res["GRBM_GUI_ACTIVE"][-1] / 8)
    if "SQ_WAVE_CYCLES" in res and "GRBM_GUI_ACTIVE" in res:
        res["waves_per_simd_last"] = res["SQ_WAVE_CYCLES"][-1] * 4.0 / 1024 / (res["GRBM_GUI_ACTIVE"][-1] / 8)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
