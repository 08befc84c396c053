#!/usr/bin/env python3
"""Benchmark of the segment query hot path on synthetic Pinot-format segments (BASELINE.json).

Workloads (`--workload`; the default is the headline metric):
  adanalytics  config 2 (north star): SELECT daysSinceEpoch, SUM(clicks), SUM(impressions) FROM adAnalytics
               WHERE daysSinceEpoch BETWEEN 18000 AND 18089 AND accountId IN (<1 000 ids>)
               GROUP BY daysSinceEpoch ORDER BY daysSinceEpoch LIMIT 400 -- 128 segments x 7 812 500 rows per GPU
  ssb          config 3: SSB Q1.1 shape, SUM(lo_extendedprice * lo_discount) under 3 dictionary filters -- 96 segments
               per GPU (768 over 8 GPUs = 6 B rows)
  highcard     config 4: SELECT userId, DISTINCTCOUNT(itemId) ... GROUP BY userId ORDER BY DISTINCTCOUNT(itemId) DESC,
               userId LIMIT 100 (10 M users x 1 000 items, numGroupsLimit 10 M) -- 128 segments per GPU

Segments are generated on the device (pinot_amd.synth) and resident in HBM before the timed region.  A step = one
query over all of this GPU's segments: host plan compile + filter pre-pass + fused scan/aggregate kernel + device
finalize (+ at N > 1 the cross-GPU merge, pinot_amd.combine).  Weak scaling: every rank scans its own segments.
`--gpus N` without a torchrun environment launches N rank processes (torch.distributed.run) before touching a GPU.

`roofline`: the hot path's kernels (the selective stream over the driving filter leaves + the fused scan over its
survivors, or the fused scan alone when no leaf prefix is selective):
algorithmic bytes per query (forward-index bytes of the touched columns + dictionary bytes of the decoded columns,
SURVEY §8(d)) / their summed HIP-event durations on the stream they run on; `traffic` from the rocprofv3
FETCH_SIZE / WRITE_SIZE passes of tools/profile_bench.sh (profiles/traffic_<workload>.json).
`cpu_baseline`: the C restatement of the Pinot CPU operators (oracle/, "port") on a bounded sample of the same segments,
at Pinot's default combine parallelism (CombineOperatorUtils.java:38-50) and at every core this process may use; rank 0
at N = 1 only.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s
HEADLINE_METRIC = "rows/sec for filter+group-by SUM over 1B rows; % of HBM roofline, 1–8 GPUs"


def workloads(args):
    from pinot_amd import synth
    return {
        "adanalytics": dict(
            specs=synth.ADANALYTICS, table="adAnalytics", segments=128, trim=False,
            query=synth.adanalytics_query(args.in_ids), decoded=("daysSinceEpoch", "clicks", "impressions"),
            metric=HEADLINE_METRIC,
            desc="AdAnalytics config 2: SUM(clicks), SUM(impressions) WHERE daysSinceEpoch BETWEEN (90 of 365 days) "
                 f"AND accountId IN ({args.in_ids} ids) GROUP BY daysSinceEpoch"),
        "ssb": dict(
            specs=synth.SSB_LINEORDER, table="lineorder", segments=96, trim=False, query=synth.ssb_q11_query(),
            decoded=("lo_extendedprice", "lo_discount"),
            metric="rows/sec for filter + SUM(a*b) over SSB lineorder (config 3, secondary line)",
            desc="SSB config 3 (Q1.1 shape): SUM(lo_extendedprice * lo_discount) WHERE lo_orderdate BETWEEN "
                 "(365 of 2557 days) AND lo_discount BETWEEN 1 AND 3 AND lo_quantity < 25"),
        "highcard": dict(
            specs=synth.HIGHCARD, table="events", segments=128, trim=True,
            query=synth.highcard_query() + " OPTION(numGroupsLimit=10000000)", decoded=("userId", "itemId"),
            metric="rows/sec for high-cardinality group-by DISTINCTCOUNT (config 4, secondary line)",
            desc="config 4: SELECT userId, DISTINCTCOUNT(itemId) GROUP BY userId (10 M users x 1 000 items) "
                 "ORDER BY DISTINCTCOUNT(itemId) DESC, userId LIMIT 100, numGroupsLimit 10 M"),
    }


def launch_ranks(n):
    """N rank processes through torch.distributed.run (this process has not touched a GPU); exit with its code."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.call(cmd))


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=("adanalytics", "ssb", "highcard"), default="adanalytics")
    ap.add_argument("--segments", type=int, default=None, help="segments per GPU (default: the workload's)")
    ap.add_argument("--rows", type=int, default=7_812_500, help="rows per segment")
    ap.add_argument("--in-ids", type=int, default=1000)
    ap.add_argument("--cpu-sample-segments", type=int, default=None)
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="per CPU leg")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--traffic-file", default=None, help="PMC HBM traffic of the scan kernel (tools/profile_bench.sh)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        launch_ranks(args.gpus)

    import numpy as np
    import torch

    W = workloads(args)[args.workload]
    if args.segments is None:
        args.segments = W["segments"]
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
    want_cpu = rank == 0 and world == 1 and not args.no_cpu
    cores = len(os.sched_getaffinity(0))
    nproc = os.cpu_count()
    pinot_threads = max(1, min(10, cores // 2))  # CombineOperatorUtils.MAX_NUM_THREADS_PER_QUERY on this host
    n_sample = min(args.segments, args.cpu_sample_segments or max(4, min(16, cores)))
    segs, host_sample = [], []
    t_gen = time.time()
    fwd_bytes = dict_bytes = 0
    table = None
    for s in range(args.segments):
        gidx = rank * args.segments + s
        dcs = synth.make_columns_torch(W["specs"], gidx, args.rows, dev)
        seg = ImmutableSegment(f"{W['table']}_{gidx}", args.rows, {dc.spec.name: dc.meta_column() for dc in dcs})
        segs.append(seg)
        if table is None:
            table = Table(W["table"], [seg])
        eng.register_device_segment(seg, table, dcs)
        fwd_bytes += sum((args.rows * dc.bits + 7) // 8 for dc in dcs)
        dict_bytes += sum(4 * dc.cardinality for dc in dcs if dc.spec.name in W["decoded"])
        if want_cpu and s < n_sample:
            host_sample.append(ImmutableSegment(seg.name, args.rows, {dc.spec.name: dc.host_column() for dc in dcs}))
        del dcs
    torch.cuda.synchronize()
    table = Table(W["table"], segs)
    gen_s = time.time() - t_gen

    q = parse(W["query"])
    t_low = time.perf_counter()
    plan = eng.make_plan(table, q, flags=0, trim=W["trim"])
    lowering_ms = (time.perf_counter() - t_low) * 1e3
    if world > 1:
        for ks in plan.key_spaces:  # packed keys merge across ranks only over identical key spaces
            kk = torch.tensor([ks.kind, ks.cardinality, ks.base], dtype=torch.int64, device=dev)
            allk = [torch.empty_like(kk) for _ in range(world)]
            dist.all_gather(allk, kk)
            assert all(torch.equal(kk, x) for x in allk), "key spaces differ across ranks"

    def step():
        if world == 1:
            return eng.run_plan(plan)
        return merge_partials_across_ranks(eng, plan, eng.run_partial(plan))

    for _ in range(args.warmup):
        res = step()
    scan_ms = []
    parts = {k: [] for k in ("host_compile_ms", "prepass_ms", "prefilter_ms", "scan_ms", "execute_wall_ms",
                             "finalize_ms", "finalize_wall_ms")}
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
        tm = eng.last_timing()
        scan_ms.append(tm.prefilter_ms + tm.scan_ms)  # the hot path's kernels: selective stream + fused scan
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
    value = rows_per_gpu * world * args.steps / el
    scan_avg_ms = float(np.mean(scan_ms))
    alg_bytes = fwd_bytes + dict_bytes
    achieved = alg_bytes / (scan_avg_ms * 1e-3) / 1e9

    cpu = parity = None
    if want_cpu and host_sample:
        from oracle.oracle import OracleEngine
        ht = Table(W["table"], host_sample)
        hq = parse(W["query"])
        from pinot_amd.plan import CPlan
        orc = OracleEngine()
        cplan = CPlan(ht, hq, host_sample, list(range(1, len(host_sample) + 1)))
        legs = {}
        for name, threads in (("pinot_default", min(len(host_sample), pinot_threads)),
                              ("all_cores", min(len(host_sample), cores))):
            v, runs = orc.time_segments(cplan, host_sample, threads, args.cpu_seconds)
            legs[name] = {"value": v, "threads": threads, "runs": runs}
        best = max(legs.values(), key=lambda x: x["value"])
        cpu = {"value": best["value"], "unit": "rows/s", "cores": best["threads"], "kind": "port",
               "label": "restated Pinot CPU path (oracle/pinot_oracle.c, per-segment operators)",
               "sample": f"{len(host_sample)} of the {args.segments} segments ({len(host_sample) * args.rows} rows), "
                         f"same query; per-segment filter -> projection -> aggregation in C, segments as parallel "
                         f"combine tasks; the value-keyed merge of the per-segment results is not timed",
               "legs": legs, "nproc": nproc, "cores_available": cores, "cpu_model": cpu_model()}
        if W["table"] != "events":  # parity on the sample (config 4's 5 M groups per segment are tested smaller)
            o = orc.execute(ht, hq)
            d = eng.run_plan(eng.make_plan(table, q, segments=segs[:len(host_sample)], flags=0))
            parity = bool(d.rows == o.rows and d.stats.num_docs_scanned == o.stats.num_docs_scanned)

    traffic = traffic_bytes = None
    tf = args.traffic_file or os.path.join(ROOT, "profiles", f"traffic_{args.workload}.json")
    try:  # rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over this same command (tools/profile_bench.sh)
        tj = json.load(open(tf))
        tc = tj.get("config") or {}
        if tc.get("rows_per_gpu") == rows_per_gpu and tc.get("workload") == W["desc"] and \
                tj.get("traffic_bytes_per_launch"):
            traffic_bytes = float(tj["traffic_bytes_per_launch"])
            traffic = traffic_bytes / (scan_avg_ms * 1e-3) / 1e9
    except (OSError, ValueError):
        pass

    if rank == 0:
        out = {
            "metric": W["metric"], "value": value, "unit": "rows/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "int64",
            "data": "synthetic (pinot_amd.synth, seed 42, Pinot segment format, device-generated)",
            "config": {"workload": W["desc"], "rows_per_gpu": rows_per_gpu, "segments_per_gpu": args.segments,
                       "rows_per_segment": args.rows,
                       "in_list_size": args.in_ids if args.workload == "adanalytics" else None,
                       "parallelism": f"segments x{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "stream_kernel + scan_kernel" if tm.scan_launches > 1 else "scan_kernel",
                         "kernel_ms": scan_avg_ms,
                         "algorithmic_bytes": alg_bytes,
                         "traffic_bytes_per_launch": traffic_bytes,
                         # the bytes actually moved (PMC) over the same time: below `frac` when the AND short-circuits
                         "traffic_frac": traffic / HBM_PEAK_GBS if traffic is not None else None},
            "cpu_baseline": cpu,
            "parity_sample": parity,
            "step_breakdown_ms": {k: round(float(np.mean(v)), 4) for k, v in parts.items()},
            "host_plan_lowering_ms": round(lowering_ms, 3),
            "groups": len(res.rows), "docs_matched": res.stats.num_docs_scanned, "datagen_s": round(gen_s, 1),
        }
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
