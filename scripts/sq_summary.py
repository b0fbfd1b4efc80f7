#!/usr/bin/env python3
"""Per-launch averages of every counter in gpurun_out/<dir>/*/*_counter_collection.csv for one kernel
(argv[2], default trace_pool; the timed variant, not the count_work one)."""
import collections
import csv
import glob
import sys

d = sys.argv[1]
kernel = sys.argv[2] if len(sys.argv) > 2 else "trace_pool"
tot = {}
for f in sorted(glob.glob(f"gpurun_out/{d}/*/*_counter_collection.csv")):
    agg, disp = collections.defaultdict(float), set()
    for r in csv.DictReader(open(f)):
        if kernel not in r["Kernel_Name"] or "true> >" in r["Kernel_Name"]:
            continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
        disp.add(r["Dispatch_Id"])
    for c, v in agg.items():
        tot[c] = v / max(len(disp), 1)
for c in sorted(tot):
    print(f"{c:32s} {tot[c]:.4g}")
