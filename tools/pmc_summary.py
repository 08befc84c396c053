#!/usr/bin/env python3
"""Reduce rocprofv3 --pmc counter_collection.csv files to per-dispatch counter sums of one kernel (dev tool)."""
import collections
import csv
import glob
import re
import sys

pattern = sys.argv[1] if len(sys.argv) > 1 else "scan_kernel"
for d in sys.argv[2:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        agg = collections.OrderedDict()
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if not re.search(pattern, r["Kernel_Name"]):
                    continue
                k = int(r["Dispatch_Id"])
                agg.setdefault(k, {"kernel": re.search(pattern, r["Kernel_Name"]).group(0)})
                agg[k][r["Counter_Name"]] = agg[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        for k, v in agg.items():
            print(d.split("/")[-1], k, v["kernel"], " ".join(f"{a}={b:.6g}" for a, b in v.items() if a != "kernel"))
