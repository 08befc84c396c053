#!/usr/bin/env python3
"""Benchmark of the north-star workload (BASELINE.json config 2):

    SELECT daysSinceEpoch, SUM(clicks), SUM(impressions) FROM adAnalytics
    WHERE daysSinceEpoch BETWEEN 18000 AND 18089 AND accountId IN (<1 000 ids>)
    GROUP BY daysSinceEpoch ORDER BY daysSinceEpoch LIMIT 400

over 1 B synthetic rows per GPU (128 Pinot-format segments x 7 812 500 rows, generated on the device by
pinot_amd.synth, resident in HBM before the timed region).  A step = one pg_execute of the query over all of this
GPU's segments (host plan compile + filter pre-pass + fused scan/aggregate kernel + result decode); at N > 1 each rank
runs its own 128 segments (weak scaling) and the ranks merge their dense partial state with RCCL all-reduces
(pinot_amd.combine).  Rank 0 prints ONE JSON line.

`roofline` is for the dominant kernel (scan_kernel): algorithmic bytes per launch (forward-index bytes of the four
columns + dictionary bytes of the aggregated / grouped columns) / its HIP-event duration measured on the
stream it runs on.  `cpu_baseline` times the C restatement of the Pinot CPU operators (oracle/, "port") on a bounded
sample of the same segments, single-threaded, on rank 0 at N = 1 only.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=("adanalytics", "ssb"), default="adanalytics",
                    help="adanalytics = config 2 (the headline metric); ssb = config 3 (SSB Q1.1 shape, 96 segments/GPU)")
    ap.add_argument("--segments", type=int, default=None, help="segments per GPU (default: the workload's)")
    ap.add_argument("--rows", type=int, default=7_812_500, help="rows per segment")
    ap.add_argument("--in-ids", type=int, default=1000)
    ap.add_argument("--cpu-sample-segments", type=int, default=2)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", "scan_traffic.json"),
                    help="PMC HBM traffic of the scan kernel for this workload (tools/profile_bench.sh)")
    args = ap.parse_args()
    ssb = args.workload == "ssb"
    if args.segments is None:
        args.segments = 96 if ssb else 128

    import numpy as np
    import torch

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from pinot_amd import synth
    from pinot_amd.combine import merge_partials_across_ranks
    from pinot_amd.gpu import GpuEngine
    from pinot_amd.plan import Table
    from pinot_amd.query import parse
    from pinot_amd.segment import ImmutableSegment

    eng = GpuEngine(local)
    dev = torch.device("cuda", local)
    segs, dev_cols_sample = [], []
    t_gen = time.time()
    specs = synth.SSB_LINEORDER if ssb else synth.ADANALYTICS
    tname = "lineorder" if ssb else "adAnalytics"
    table_cols = {s.name: i for i, s in enumerate(specs)}
    fwd_bytes = 0
    dict_bytes = 0
    table = None
    for s in range(args.segments):
        gidx = rank * args.segments + s
        dcs = synth.make_columns_torch(specs, gidx, args.rows, dev)
        seg = ImmutableSegment(f"{tname}_{gidx}", args.rows, {dc.spec.name: dc.meta_column() for dc in dcs})
        segs.append(seg)
        if table is None:
            table = Table(tname, [seg])
        eng.register_device_segment(seg, table, dcs)
        fwd_bytes += sum((args.rows * dc.bits + 7) // 8 for dc in dcs)
        # dictionaries the scan decodes: aggregated / grouped columns (config 2: all but accountId; config 3: the two
        # SUM operands)
        dec = ("lo_extendedprice", "lo_discount") if ssb else ("daysSinceEpoch", "clicks", "impressions")
        dict_bytes += sum(4 * dc.cardinality for dc in dcs if dc.spec.name in dec)
        if s < args.cpu_sample_segments and rank == 0 and world == 1 and not args.no_cpu:
            dev_cols_sample.append((seg, [dc.host_column() for dc in dcs]))
        del dcs
    torch.cuda.synchronize()
    table = Table(tname, segs)
    assert table.column_ids == table_cols
    gen_s = time.time() - t_gen

    q = parse(synth.ssb_q11_query() if ssb else synth.adanalytics_query(args.in_ids))
    plan = eng.make_plan(table, q)
    if world > 1 and plan.key_spaces:
        ks = plan.key_spaces[0]  # the dense key space must be identical on every rank for the all-reduce
        kk = torch.tensor([ks.kind, ks.cardinality, ks.base], dtype=torch.int64, device=dev)
        allk = [torch.empty_like(kk) for _ in range(world)]
        dist.all_gather(allk, kk)
        assert all(torch.equal(kk, x) for x in allk), "key spaces differ across ranks"

    def step():
        if world == 1:
            return eng.run_plan(plan)
        p = eng.run_partial(plan)
        return merge_partials_across_ranks(eng, plan, p)

    for _ in range(args.warmup):
        res = step()
    scan_ms = []
    parts = {k: [] for k in ("host_compile_ms", "prepass_ms", "scan_ms", "execute_wall_ms", "finalize_wall_ms")}
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
        tm = eng.last_timing()
        scan_ms.append(tm.scan_ms)
        for k, v in parts.items():
            v.append(getattr(tm, k))
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    if dist:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())

    rows_per_gpu = args.segments * args.rows
    total_rows = rows_per_gpu * world * args.steps
    value = total_rows / el
    scan_avg_ms = float(np.mean(scan_ms))
    alg_bytes = fwd_bytes + dict_bytes
    achieved = alg_bytes / (scan_avg_ms * 1e-3) / 1e9

    cpu = None
    parity = None
    if rank == 0 and world == 1 and not args.no_cpu and dev_cols_sample:
        from oracle.oracle import OracleEngine
        orc = OracleEngine(threads=1)
        hsegs = [ImmutableSegment(seg.name, args.rows, {c.name: c for c in cols}) for seg, cols in dev_cols_sample]
        ht = Table(tname, hsegs)
        o = orc.execute(ht, q)  # warm
        reps, tc0 = 0, time.perf_counter()
        while True:
            o = orc.execute(ht, q)
            reps += 1
            if time.perf_counter() - tc0 >= args.cpu_seconds:
                break
        cpu_el = time.perf_counter() - tc0
        cpu = {"value": reps * len(hsegs) * args.rows / cpu_el, "unit": "rows/s", "cores": 1, "kind": "port",
               "sample": f"{len(hsegs)} of the {args.segments} segments ({len(hsegs) * args.rows} rows), same query, "
                         f"{reps} runs of oracle/pinot_oracle.c (restated Pinot CPU operators), 1 thread"}
        # parity on the sample: device result over the same segments
        dplan = eng.make_plan(table, q, segments=[seg for seg, _ in dev_cols_sample])
        d = eng.run_plan(dplan)
        parity = bool(d.rows == o.rows and d.stats.num_docs_scanned == o.stats.num_docs_scanned)

    traffic = traffic_bytes = None
    try:  # measured by rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over this same command (tools/profile_bench.sh)
        tj = json.load(open(args.traffic_file))
        tc = tj.get("config") or {}
        if (not ssb and tc.get("rows_per_gpu") == args.segments * args.rows and tc.get("in_list_size") == args.in_ids
                and tj.get("traffic_bytes_per_launch")):
            traffic_bytes = float(tj["traffic_bytes_per_launch"])
            traffic = traffic_bytes / (scan_avg_ms * 1e-3) / 1e9
    except (OSError, ValueError):
        pass

    if rank == 0:
        out = {
            "metric": ("rows/sec for filter + SUM(a*b) over SSB lineorder (config 3, secondary line)" if ssb else
                       "rows/sec for filter+group-by SUM over 1B rows; % of HBM roofline, 1–8 GPUs"),
            "value": value, "unit": "rows/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": el / args.steps * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "int64", "data": "synthetic (pinot_amd.synth, seed 42, Pinot segment format, device-generated)",
            "config": {"workload": ("SSB config 3 (Q1.1 shape): SUM(lo_extendedprice * lo_discount) WHERE lo_orderdate "
                                    "BETWEEN (365 of 2557 days) AND lo_discount BETWEEN 1 AND 3 AND lo_quantity < 25"
                                    if ssb else
                                    "AdAnalytics config 2: SUM(clicks), SUM(impressions) WHERE daysSinceEpoch BETWEEN "
                                    "(90 of 365 days) AND accountId IN (1000 ids) GROUP BY daysSinceEpoch"),
                       "rows_per_gpu": rows_per_gpu, "segments_per_gpu": args.segments,
                       "rows_per_segment": args.rows, "in_list_size": None if ssb else args.in_ids,
                       "parallelism": f"segments x{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "scan_kernel", "kernel_ms": scan_avg_ms, "algorithmic_bytes": alg_bytes,
                         "traffic_bytes_per_launch": traffic_bytes},
            "cpu_baseline": cpu,
            "parity_sample": parity,
            "step_breakdown_ms": {k: round(float(np.mean(v)), 4) for k, v in parts.items()},
            "groups": len(res.rows), "docs_matched": res.stats.num_docs_scanned, "datagen_s": round(gen_s, 1),
        }
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
