#!/usr/bin/env python3
"""Per-kernel duration summary from a rocprofv3 --kernel-trace csv directory (dev tool).

usage: trace_summary.py <dir> <kernel-regex>  (one line per matching kernel template)"""
import collections
import csv
import glob
import re
import statistics
import sys

d, pat = sys.argv[1], sys.argv[2]
durs = collections.defaultdict(list)
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            m = re.search(pat, r["Kernel_Name"])
            if m:
                durs[m.group(0)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
if not durs:
    print(f"no dispatch of {pat}")
    sys.exit(0)
for k, v in sorted(durs.items()):
    print(f"kernel {k}: dispatches {len(v)} mean_ms {statistics.mean(v):.4f} "
          f"median_ms {statistics.median(v):.4f} min_ms {min(v):.4f} max_ms {max(v):.4f}")
