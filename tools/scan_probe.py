#!/usr/bin/env python3
"""Dev tool: decompose scan-kernel time over query shapes on synthetic AdAnalytics segments (device-generated).

usage: python tools/scan_probe.py [--segments 32] [--reps 5]
Prints one line per query: scan kernel ms (HIP events), rows/s of the kernel, matched docs."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--segments", type=int, default=32)
    ap.add_argument("--rows", type=int, default=7_812_500)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--only", default="")
    ap.add_argument("--workload", choices=("adanalytics", "ssb"), default="adanalytics")
    args = ap.parse_args()
    import numpy as np
    import torch
    from pinot_amd import synth
    from pinot_amd.gpu import GpuEngine
    from pinot_amd.plan import Table
    from pinot_amd.query import parse
    from pinot_amd.segment import ImmutableSegment
    eng = GpuEngine(0)
    segs = []
    table = None
    for s in range(args.segments):
        specs = synth.SSB_LINEORDER if args.workload == "ssb" else synth.ADANALYTICS
        dcs = synth.make_columns_torch(specs, s, args.rows, torch.device("cuda"))
        seg = ImmutableSegment(f"a{s}", args.rows, {dc.spec.name: dc.meta_column() for dc in dcs})
        segs.append(seg)
        if table is None:
            table = Table("adAnalytics", [seg])
        eng.register_device_segment(seg, table, dcs)
    table = Table("adAnalytics", segs)
    ids = ", ".join(str((i * 7919 + 13) % 1_000_000) for i in range(1000))
    f3 = "lo_orderdate BETWEEN 8035 AND 8399 AND lo_discount BETWEEN 1 AND 3 AND lo_quantity < 25"
    qs = {
        "ssb_count": f"SELECT COUNT(*) FROM t WHERE {f3}",
        "ssb_date": "SELECT COUNT(*) FROM t WHERE lo_orderdate BETWEEN 8035 AND 8399",
        "ssb_sum_small": f"SELECT SUM(lo_discount * lo_quantity) FROM t WHERE {f3}",
        "ssb_sum_price": f"SELECT SUM(lo_extendedprice) FROM t WHERE {f3}",
        "ssb_q11": synth.ssb_q11_query(),
        "ssb_dense_price": "SELECT SUM(lo_extendedprice) FROM t",
    } if args.workload == "ssb" else {
        "count": "SELECT COUNT(*) FROM t",
        "in_only": f"SELECT COUNT(*) FROM t WHERE accountId IN ({ids})",
        "range_only": "SELECT COUNT(*) FROM t WHERE daysSinceEpoch BETWEEN 18000 AND 18089",
        "range_acct": "SELECT COUNT(*) FROM t WHERE accountId BETWEEN 1000 AND 500000",
        "range_narrow": "SELECT COUNT(*) FROM t WHERE accountId BETWEEN 1000 AND 1999",
        "in_100": "SELECT COUNT(*) FROM t WHERE accountId IN (" + ids.split(", 1")[0] + ")",
        "sum_dense": "SELECT SUM(clicks) FROM t",
        "gb_dense": "SELECT daysSinceEpoch, SUM(clicks) FROM t GROUP BY daysSinceEpoch",
        "config2": synth.adanalytics_query(1000),
        "c2_filter": f"SELECT COUNT(*) FROM t WHERE daysSinceEpoch BETWEEN 18000 AND 18089 AND accountId IN ({ids})",
        "c2_gb_count": f"SELECT daysSinceEpoch, COUNT(*) FROM t WHERE daysSinceEpoch BETWEEN 18000 AND 18089 "
                       f"AND accountId IN ({ids}) GROUP BY daysSinceEpoch",
        "c2_sum": f"SELECT SUM(clicks), SUM(impressions) FROM t WHERE daysSinceEpoch BETWEEN 18000 AND 18089 "
                  f"AND accountId IN ({ids})",
    }
    rows = args.segments * args.rows
    for name, sql in qs.items():
        if args.only and name not in args.only.split(","):
            continue
        plan = eng.make_plan(table, parse(sql))
        r = eng.run_plan(plan)
        ks, hs = [], []
        t0 = time.perf_counter()
        for _ in range(args.reps):
            r = eng.run_plan(plan)
            t = eng.last_timing()
            ks.append(t.prefilter_ms + t.scan_ms)
            hs.append((t.host_compile_ms, t.prepass_ms, t.prefilter_ms, t.scan_ms, t.execute_wall_ms,
                       t.finalize_wall_ms))
        wall = (time.perf_counter() - t0) / args.reps * 1e3
        k = float(np.median(ks))
        print(f"{name:12s} scan {k:8.3f} ms  {rows / k / 1e6:9.3f} Grows/s  wall {wall:8.3f} ms  "
              f"matched {r.stats.num_docs_scanned}  host/pre/filt/scan/exec/fin ms "
              + "/".join(f"{x:.3f}" for x in np.median(np.array(hs), axis=0)), flush=True)


if __name__ == "__main__":
    main()
