#!/usr/bin/env python3
"""Summarise rocprofv3 counter CSVs of the timed trace kernel (not its stats
build, `...true>`): tools/pmc_summary.py DIR [DIR ...]"""
import collections
import csv
import glob
import sys

for d in sys.argv[1:]:
    agg = collections.defaultdict(list)
    dur = []
    for f in glob.glob(f"{d}/*/prof_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "trace_kernel" in r["Kernel_Name"] and "false>" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for f in glob.glob(f"{d}/*/prof_kernel_stats.csv"):
        for r in csv.DictReader(open(f)):
            if "trace_kernel" in r["Name"] and "false>" in r["Name"]:
                dur.append(float(r["AverageNs"]))
    print(f"== {d}  kernel avg {sum(dur) / max(len(dur), 1) / 1e6:.2f} ms")
    for k in sorted(agg):
        v = agg[k]
        print(f"  {k:26s} {sum(v) / len(v):.4g}")
