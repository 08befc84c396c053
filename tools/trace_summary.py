#!/usr/bin/env python3
"""Per-kernel duration summary from a rocprofv3 --kernel-trace csv directory (dev tool).

usage: trace_summary.py <dir> <kernel-substring>"""
import csv
import glob
import statistics
import sys

d, pat = sys.argv[1], sys.argv[2]
durs = []
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            if pat in r["Kernel_Name"]:
                durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
if not durs:
    print(f"no dispatch of {pat}")
    sys.exit(0)
print(f"kernel {pat}: dispatches {len(durs)} mean_ms {statistics.mean(durs):.4f} "
      f"median_ms {statistics.median(durs):.4f} min_ms {min(durs):.4f} max_ms {max(durs):.4f}")
