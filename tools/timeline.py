#!/usr/bin/env python3
"""Timeline of the last dispatches in a rocprofv3 --kernel-trace csv directory: start offset, duration and the idle gap
before each kernel (dev tool: where a query's wall time goes between kernels).

usage: timeline.py <dir> [last-n]"""
import csv
import glob
import re
import sys

d, n = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows = []
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    with open(f) as fh:
        rows += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(fh)]
for f in glob.glob(f"{d}/**/*memory_copy_trace.csv", recursive=True):  # with --memory-copy-trace
    with open(f) as fh:
        rows += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                  "copy " + r.get("Direction", "?") + " " + r.get("Size", r.get("Bytes", ""))) for r in csv.DictReader(fh)]
rows.sort()
rows = rows[-n:]
t0, prev = rows[0][0], rows[0][0]
for s, e, k in rows:
    name = re.sub(r"\(.*", "", k)[-60:]
    print(f"{(s - t0) / 1e3:10.1f} us  dur {(e - s) / 1e3:9.1f}  gap {(s - prev) / 1e3:8.1f}  {name}")
    prev = e
