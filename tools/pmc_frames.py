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
            if "trace_kernel" not in r["Kernel_Name"] or "true>" in r["Kernel_Name"]:
                continue
            d = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0)
            c = r["Counter_Name"]
            per[c][d] = per[c].get(d, 0.0) + float(r["Counter_Value"])
    res = {c: [v[k] for k in sorted(v)] for c, v in per.items()}
    if "FETCH_SIZE" in res and "WRITE_SIZE" in res:
        res["hbm_bytes_last"] = (2.0 * res["FETCH_SIZE"][-1] + res["WRITE_SIZE"][-1]) * 1024.0
        res["write_bytes_last"] = res["WRITE_SIZE"][-1] * 1024.0
        res["fetch_bytes_x2_last"] = res["FETCH_SIZE"][-1] * 2048.0
    print(json.dumps(res))


if __name__ == "__main__":
    main()
