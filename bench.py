#!/usr/bin/env python3
"""Benchmark of the segment query hot path on synthetic Pinot-format segments (BASELINE.json).

Workloads (`--workload`; the default is the headline metric):
  adanalytics  config 2 (north star): SELECT daysSinceEpoch, SUM(clicks), SUM(impressions) FROM adAnalytics
               WHERE daysSinceEpoch BETWEEN 18000 AND 18089 AND accountId IN (<1 000 ids>)
               GROUP BY daysSinceEpoch ORDER BY daysSinceEpoch LIMIT 400 -- 128 segments x 7 812 500 rows per GPU
  ssb          config 3: SSB Q1.1 shape, SUM(lo_extendedprice * lo_discount) under 3 dictionary filters -- 96 segments
               per GPU (768 over 8 GPUs = 6 B rows)
  highcard     config 4: SELECT userId, DISTINCTCOUNT(itemId) ... GROUP BY userId ORDER BY DISTINCTCOUNT(itemId) DESC,
               userId LIMIT 100 (10 M users x 1 000 items) -- 128 segments per GPU, under the server instance config
               SURVEY §8(d) prescribes for the reference: num.groups.limit 10 M (no per-segment truncation) and
               groupby.trim.threshold = MAX_TRIM_THRESHOLD (no lossy resize during the combine); the step returns the
               server's result, the top getTableCapacity(100, 5 000) = 5 000 groups with their value sets
  index        config 5: COUNT(*), COUNTMV(mvTags) under a sorted-index range, an OR of two inverted-index leaves, an
               inverted NOT_EQ and an inverted IN -- 32 segments per GPU (256 over 8 GPUs = 2 B rows)

Segments are generated on the device (pinot_amd.synth) and resident in HBM before the timed region.  A step = one
query over all of this GPU's segments through the relocatable plan image (pg_execute_image): host plan compile +
filter pre-pass + fused scan/aggregate kernel + device finalize + the result's arrays (keys, values, counts, value
sets: what the server's DataTable holds) copied into numpy (+ at N > 1 the cross-GPU merge, pinot_amd.combine).  The
value-keyed Python dict view of those arrays (DeviceResult.rows) is built on first access, outside the step: the parity
check after the timed region reads it.  Weak scaling: every rank scans its own segments.
`--gpus N` without a torchrun environment launches N rank processes (torch.distributed.run) before touching a GPU.

`roofline`: the hot path's kernels (the selective stream over the driving filter leaves + the fused scan over its
survivors, or the fused scan alone when no leaf prefix is selective), timed with HIP events on the stream they run on.
`achieved` = the bytes the executed plan must read / that time: every column read for all docs in full (the streamed
driving leaf, a full scan's columns) + for a column read only for the docs that passed earlier filter stages, the
128-byte lines holding those docs' values (expected lines of uniformly spread survivors, with the survivor counts of the
plan's own filter prefixes measured by COUNT(*) queries before timing), at the width the device reads (dictIds, or the
decoded value image of a large dictionary).  SURVEY §8(d)'s algorithmic bytes (every touched column in full) are kept
as `algorithmic_bytes` / `algorithmic_frac`: a short-circuiting AND never reads most of them, so that ratio is not
bounded by the peak.  `traffic` = PMC bytes (FETCH_SIZE x 2 + WRITE_SIZE per query, tools/profile_bench.sh) from
profiles/traffic_<workload>.json, used only when it was measured on this very libpinot_gpu.so (md5 stamp).
`cpu_baseline`: the C restatement of the Pinot CPU operators (oracle/, "port": per-segment filter with later AND
children on the survivors only, projection of the matching docs, aggregation) over min(#segments, 128, cores) of the
same segments, at Pinot's default combine parallelism (CombineOperatorUtils.java:38-50) and at one thread per segment up
to every core this process may use; rank 0 at N = 1 only.
`parity_full`: the last timed step's result itself (same plan, flags and trim) against the oracle over EVERY segment of
the line (the server's combined result under the same instance config); `parity_sample` re-plans 16 segments.
`--split-table`: the workload's table (128 segments for config 2 / 4) divided over the N ranks (16 per GPU
at N = 8): strong scaling of the 1 B-row query.
"""
import argparse
import hashlib
import json
import math
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
    """`trim`: "server" = the group-by result a Pinot server returns (GroupByOrderByCombineOperator: the top
    getTableCapacity(limit, 5 000) groups under the ORDER BY).  `config`: the server instance's settings
    (InstanceConfig; default = InstancePlanMakerImplV2's defaults).  `stages`: the executed plan's read pattern, in evaluation order: (filter the docs passed so far, or None = every
    doc; [(column, "ids" | "values")] read for those docs).  "ids" = the packed dictIds; "values" = what an aggregation /
    key reads (the decoded value image of a large non-identity dictionary, else the dictIds)."""
    from pinot_amd import synth
    from pinot_amd.plan import MAX_TRIM_THRESHOLD, InstanceConfig
    ids = ", ".join(str((i * 7919 + 13) % 1_000_000) for i in range(args.in_ids))
    return {
        "adanalytics": dict(
            specs=synth.ADANALYTICS, table="adAnalytics", segments=128, trim="server",
            query=synth.adanalytics_query(args.in_ids), decoded=("daysSinceEpoch", "clicks", "impressions"),
            metric=HEADLINE_METRIC,
            desc="AdAnalytics config 2: SUM(clicks), SUM(impressions) WHERE daysSinceEpoch BETWEEN (90 of 365 days) "
                 f"AND accountId IN ({args.in_ids} ids) GROUP BY daysSinceEpoch",
            stages=[(None, [("accountId", "ids")]),                       # the selective stream
                    (f"accountId IN ({ids})", [("daysSinceEpoch", "ids")]),  # list scan: the range leaf + group key
                    ("*", [("clicks", "values"), ("impressions", "values")])]),
        "ssb": dict(
            specs=synth.SSB_LINEORDER, table="lineorder", segments=96, trim=False, query=synth.ssb_q11_query(),
            decoded=("lo_extendedprice", "lo_discount"),
            metric="rows/sec for filter + SUM(a*b) over SSB lineorder (config 3, secondary line)",
            desc="SSB config 3 (Q1.1 shape): SUM(lo_extendedprice * lo_discount) WHERE lo_orderdate BETWEEN "
                 "(365 of 2557 days) AND lo_discount BETWEEN 1 AND 3 AND lo_quantity < 25",
            stages=[(None, [("lo_orderdate", "ids")]),
                    ("lo_orderdate BETWEEN 8035 AND 8399", [("lo_discount", "ids")]),
                    ("lo_orderdate BETWEEN 8035 AND 8399 AND lo_discount BETWEEN 1 AND 3", [("lo_quantity", "ids")]),
                    ("*", [("lo_extendedprice", "values")])]),
        "highcard": dict(
            specs=synth.HIGHCARD, table="events", segments=128, trim="server", flags="VALUE_SETS",
            query=synth.highcard_query(), decoded=("userId", "itemId"),
            config=InstanceConfig(num_groups_limit=10_000_000, groupby_trim_threshold=MAX_TRIM_THRESHOLD),
            metric="rows/sec for high-cardinality group-by DISTINCTCOUNT (config 4, secondary line)",
            desc="config 4: SELECT userId, DISTINCTCOUNT(itemId) GROUP BY userId (10 M users x 1 000 items) "
                 "ORDER BY DISTINCTCOUNT(itemId) DESC, userId LIMIT 100, numGroupsLimit 10 M",
            stages=[(None, [("userId", "values"), ("itemId", "values")])]),
        "index": dict(
            specs=None, make=synth.make_index_columns_torch, table="idx", segments=synth.INDEX_SEGMENTS_PER_GPU,
            trim=False, query=synth.index_query(), decoded=(),
            metric="rows/sec for sorted + inverted index filters (5 predicates) + COUNTMV (config 5, secondary line)",
            desc="config 5: COUNT(*), COUNTMV(mvTags) WHERE sortedCol BETWEEN (40 %) AND (inv1 = x OR inv2 IN (20)) "
                 "AND inv3 <> y AND inv4 IN (2000) -- sorted index, 4 bitmap inverted indexes, MV column",
            stages=None),
    }


DECODE_MIN_CARD = 1 << 17  # pg_runtime.hip kDecodeMinCard: larger INT / LONG dictionaries get a decoded value image


def read_width(dc, use):
    """Bits per doc the device reads of synthetic column `dc` for a use (pg_runtime.hip build_decoded)."""
    lo, hi = int(dc.dict_values[0]), int(dc.dict_values[-1])
    identity = hi - lo + 1 == dc.cardinality
    if use == "ids" or identity or dc.cardinality < DECODE_MIN_CARD:
        return dc.bits
    return max(1, (hi - lo).bit_length())


def lines_bytes(num_docs, width, needed):
    """Bytes of the 128-byte lines holding `needed` uniformly spread docs' values of a `width`-bit column."""
    total = (num_docs * width + 7) // 8
    if needed >= num_docs:
        return total
    lines = (total + 127) // 128
    per_line = 1024.0 / width
    p = 1.0 - (1.0 - needed / num_docs) ** per_line
    return min(total, 128.0 * lines * p)


def index_plan_bytes(eng, table, plan, index_meta, rows, sql):
    """Config 5: the bytes its plan must read, on SURVEY §8(d)'s definition.  Per segment: the serialized roaring
    bytes of the dictIds the inverted leaves select, within the 64 K-doc keys of the sorted leaf's doc range (the
    fused index count decodes only those keys' containers; docs are uniform over the keys, so the range's share of
    each bitmap), the sorted index's (start, end) pairs, and the value counts of the docs in that range at 4 bits per
    doc (the count column COUNTMV reads, the device's form of the MV start-of-row bitmap, <= 0.5 B / doc).  No doc bitmap
    is written or read: the leaves are decoded in LDS (pg_index.hip).  Returns (plan bytes, SURVEY §8(d) algorithmic
    bytes = every referenced roaring byte + sorted pairs + the start-of-row bitmap over the sorted range,
    [docs in the sorted range, matched docs])."""
    import numpy as np
    where = sql.split(" WHERE ")[1]
    sp = [p for p in plan.query.filter.leaves() if p.column == "sortedCol"][0]
    in_range = int(eng.execute(table, f"SELECT COUNT(*) FROM {table.name} WHERE sortedCol BETWEEN {sp.lower} AND "
                                      f"{sp.upper}").rows[()][0])
    matched = int(eng.execute(table, f"SELECT COUNT(*) FROM {table.name} WHERE {where}").rows[()][0])
    S = len(index_meta)
    frac_range = in_range / (S * rows)
    total = alg = 0.0
    for si, meta in enumerate(index_meta):
        ref = 0
        for li, lw in enumerate(plan.lowered[si]):
            offs = meta[plan.leaf_preds[li].column][0]
            if offs is None or lw.ids is None:
                continue
            ids = np.asarray(lw.ids, dtype=np.int64)
            ref += int((offs[ids + 1] - offs[ids]).sum())
        pairs = 8 * meta["sortedCol"][1]
        total += frac_range * ref + pairs + frac_range * rows / 2
        alg += ref + pairs + frac_range * meta["mvTags"][2] / 8
    return total, alg, [in_range, matched]


def full_parity(W, q, res, host_all, cfg, threads) -> bool:
    """The timed plan's own result (`res`: same flags, trim and instance config) against the oracle over every segment
    of the line: the server's combined result (GroupByOrderByCombineOperator / AggregationOnlyCombineOperator under
    `cfg`), rows and docs scanned.  Config 4 (~10 M users with value sets): the oracle's per-segment (user, item) pairs
    merged by value in a bitmap of every (user, item), then the server's top getTableCapacity rows under the ORDER BY
    with their item sets."""
    import numpy as np
    from concurrent.futures import ThreadPoolExecutor
    from oracle.oracle import OracleEngine
    from pinot_amd.plan import CPlan, Table, group_trim
    orc = OracleEngine(threads=threads)
    table = Table(W["table"], host_all)
    if W["table"] != "events":
        o = orc.execute(table, q, server=W["trim"] == "server", config=cfg)
        return bool(res.rows == o.rows and res.stats.num_docs_scanned == o.stats.num_docs_scanned)
    cp = CPlan(table, q, host_all, list(range(1, len(host_all) + 1)), config=cfg)
    users_card = table.key_space("userId")
    items = table.key_space("itemId")
    from pinot_amd import abi
    assert users_card.kind == items.kind == abi.PG_KEY_VALUE_OFFSET
    ub, ib = users_card.base, items.base
    seen = np.zeros((users_card.cardinality, items.cardinality), dtype=bool)
    with ThreadPoolExecutor(threads) as ex:
        for u, v in ex.map(lambda i: orc.distinct_pairs(cp, i, host_all[i]), range(len(host_all))):
            seen[u - ub, v - ib] = True
    counts = seen.sum(axis=1)
    users = np.nonzero(counts)[0]
    size = group_trim(q, cfg).server_size
    top = users[np.lexsort((users, -counts[users]))[:size]]
    want = {(int(x + ub),): {int(i + ib) for i in np.nonzero(seen[x])[0]} for x in top}
    got = res.rows
    return bool(got.keys() == want.keys() and all(got[k][0] == want[k] for k in want) and
                res.stats.num_docs_scanned == sum(sg.num_docs for sg in host_all))


def lib_md5():
    from pinot_amd import gpu
    with open(gpu.LIB_PATH, "rb") as f:
        return hashlib.md5(f.read()).hexdigest()


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


def vary_literals(sql: str, k: int) -> str:
    """The query with every integer literal of its WHERE clause shifted by k (a same-shape query, other literals)."""
    import re
    head, sep, rest = sql.partition(" WHERE ")
    if not sep:
        return sql
    cut = min([i for i in (rest.find(" GROUP BY "), rest.find(" ORDER BY "), rest.find(" LIMIT ")) if i >= 0] or
              [len(rest)])
    where = re.sub(r"(?<![\w.])(\d+)(?![\w.])", lambda m: str(int(m.group(1)) + k), rest[:cut])
    return head + sep + where + rest[cut:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=("adanalytics", "ssb", "highcard", "index"), default="adanalytics")
    ap.add_argument("--segments", type=int, default=None, help="segments per GPU (default: the workload's)")
    ap.add_argument("--split-table", action="store_true",
                    help="divide the workload's table (--table-segments) over the ranks: strong scaling")
    ap.add_argument("--table-segments", type=int, default=None)
    ap.add_argument("--rows", type=int, default=7_812_500, help="rows per segment")
    ap.add_argument("--in-ids", type=int, default=1000)
    ap.add_argument("--cpu-sample-segments", type=int, default=None)
    ap.add_argument("--cpu-seconds", type=float, default=6.0, help="per CPU leg")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--inflight", type=int, default=4,
                    help="queries in flight in the timed loop (host threads, each with its own stream): one query's "
                         "host work (lowering to the device plan, launches, result decode; at N > 1 the cross-rank "
                         "merge) overlaps the other queries' kernels, as concurrent queries on a server do; 1 = serial")
    ap.add_argument("--no-full-parity", action="store_true",
                    help="skip the oracle check of the timed result over every segment (parity_full)")
    ap.add_argument("--traffic-file", default=None, help="PMC HBM traffic of the hot-path kernels (tools/profile_bench.sh)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        launch_ranks(args.gpus)

    import numpy as np
    import torch

    W = workloads(args)[args.workload]
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.split_table:
        total = args.table_segments or W["segments"]
        if total % world:
            raise SystemExit(f"--split-table: {total} segments do not divide over {world} ranks")
        args.segments = total // world
    elif args.segments is None:
        args.segments = W["segments"]
    # PG_BENCH_SHARE_GPU=1 (rehearsal of the N-rank path on a one-GPU box): every rank on device 0, gloo collectives
    share = os.environ.get("PG_BENCH_SHARE_GPU") == "1"
    if share:
        local = 0
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if share:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    import ctypes as C

    from pinot_amd import abi, synth
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
    n_sample = min(args.segments, args.cpu_sample_segments or max(16, min(128, cores)))
    segs, host_all = [], []  # host copies of every segment (rank 0, N = 1): the CPU leg's sample and the full parity
    t_gen = time.time()
    fwd_bytes = dict_bytes = 0
    widths = {}  # column -> [(bits of dictIds, bits of values)] per segment
    index_meta = []  # config 5: per segment {column: (inverted-index offsets, cardinality, num values)}
    table = None
    for s in range(args.segments):
        gidx = rank * args.segments + s
        dcs = W["make"](gidx, args.rows, dev) if W.get("make") else \
            synth.make_columns_torch(W["specs"], gidx, args.rows, dev)
        seg = ImmutableSegment(f"{W['table']}_{gidx}", args.rows, {dc.spec.name: dc.meta_column() for dc in dcs})
        segs.append(seg)
        if table is None:
            table = Table(W["table"], [seg])
        eng.register_device_segment(seg, table, dcs)
        if W["stages"] is not None:
            fwd_bytes += sum((args.rows * dc.bits + 7) // 8 for dc in dcs)
            dict_bytes += sum(4 * dc.cardinality for dc in dcs if dc.spec.name in W["decoded"])
            for dc in dcs:
                widths.setdefault(dc.spec.name, []).append((read_width(dc, "ids"), read_width(dc, "values")))
        else:  # index path: keep what the byte model needs (inverted-index offset headers, MV value counts)
            index_meta.append({dc.spec.name: (dc.inv_be[:4 * (dc.cardinality + 1)].cpu().numpy().view(">u4")
                                              .astype(np.int64) if dc.inv_be is not None else None,
                                              dc.cardinality, dc.num_values) for dc in dcs})
        if want_cpu and (s < n_sample or not args.no_full_parity):
            host_all.append(ImmutableSegment(seg.name, args.rows, {dc.spec.name: dc.host_column() for dc in dcs}))
        del dcs
    torch.cuda.synchronize()
    table = Table(W["table"], segs)
    gen_s = time.time() - t_gen

    q = parse(W["query"])
    t_low = time.perf_counter()
    # config 4's server result carries the DISTINCTCOUNT intermediate as the reference's Set of values per kept group
    # (what GroupByOrderByCombineOperator hands the broker); the other workloads have no DISTINCTCOUNT
    flags = abi.PG_PLAN_VALUE_SETS if W.get("flags") == "VALUE_SETS" else 0
    cfg = W.get("config")
    plan = eng.make_plan(table, q, flags=flags, trim=W["trim"], config=cfg)
    lowering_cold_ms = (time.perf_counter() - t_low) * 1e3
    # host lowering of a cache miss with the table's per-column caches warm (the server case: segments loaded once,
    # every query lowered): queries of the same shape with other filter literals, fully lowered (make_plan, no plan
    # cache), and the shape cache's re-lowering of only the leaves (CPlan.relower); outside the timed region
    low, relow = [], []
    for k in range(1, 6):
        qk = parse(vary_literals(W["query"], k))
        t1 = time.perf_counter()
        pk = eng.make_plan(table, qk, flags=flags, trim=W["trim"], config=cfg)
        pk.image()
        low.append((time.perf_counter() - t1) * 1e3)
        t1 = time.perf_counter()
        plan.relower(qk, eng.dict_id_sets).image()
        relow.append((time.perf_counter() - t1) * 1e3)
    lowering_ms = float(np.median(low))
    if world > 1:
        for ks in plan.key_spaces:  # packed keys merge across ranks only over identical key spaces
            kk = torch.tensor([ks.kind, ks.cardinality, ks.base], dtype=torch.int64, device=dev)
            allk = [torch.empty_like(kk) for _ in range(world)]
            dist.all_gather(allk, kk)
            assert all(torch.equal(kk, x) for x in allk), "key spaces differ across ranks"

    # survivors of the plan's filter prefixes (outside the timed region): the bytes the executed plan must read
    rows_per_gpu = args.segments * args.rows
    plan_bytes, stage_docs, counted = 0.0, [], set()
    if W["stages"] is None:
        plan_bytes, fwd_bytes, stage_docs = index_plan_bytes(eng, table, plan, index_meta, args.rows, W["query"])
    for filt, cols in W["stages"] or []:
        if filt is None:
            n = rows_per_gpu
        else:
            where = W["query"].split(" WHERE ")[1].split(" GROUP BY ")[0] if filt == "*" else filt
            n = int(eng.execute(table, f"SELECT COUNT(*) FROM {W['table']} WHERE {where}").rows[()][0])
        stage_docs.append(n)
        for c, use in cols:
            if c in counted:
                continue
            counted.add(c)
            for w_ids, w_vals in widths[c]:
                plan_bytes += lines_bytes(args.rows, w_ids if use == "ids" else w_vals, n / args.segments)

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
    # each step's HIP-event phase times land in a preallocated struct (one ctypes call per step inside the timed
    # region); they are summed up after it
    tms = (abi.pg_timing * args.steps)()
    last_timing = eng.lib.pg_last_timing
    t0 = time.perf_counter()
    for i in range(args.steps):
        res = step()
        last_timing(C.byref(tms[i]))
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    serial_ms = el / args.steps * 1e3
    inflight = args.inflight
    if inflight > 1:
        # the same K steps with `inflight` queries in flight: host threads run the per-GPU part of whole queries (each
        # its own stream and parameter arena in the library) while this thread completes them in submission order --
        # at N > 1 the cross-rank merge (its collectives issued by this one thread, in the same order on every rank);
        # the kernel phase times above (one query at a time) stay the roofline's
        import threading
        from concurrent.futures import ThreadPoolExecutor
        gate = threading.Barrier(inflight)
        run = eng.run_plan if world == 1 else eng.run_partial

        def first(_):  # every pool thread makes its stream / arena before the timed region
            gate.wait()
            return run(plan)

        def complete(r):
            return r if world == 1 else merge_partials_across_ranks(eng, plan, r)

        with ThreadPoolExecutor(inflight) as ex:
            for f in [ex.submit(first, i) for i in range(inflight)]:
                complete(f.result())
            for f in [ex.submit(run, plan) for _ in range(args.warmup)]:
                complete(f.result())
            torch.cuda.synchronize()
            if dist:
                dist.barrier()
            t0 = time.perf_counter()
            futs = [ex.submit(run, plan) for _ in range(args.steps)]
            for f in futs:
                res = complete(f.result())
            torch.cuda.synchronize()
            if dist:
                dist.barrier()
            el = time.perf_counter() - t0
    if dist:
        t = torch.tensor([el], dtype=torch.float64, device="cpu" if share else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())

    for tm in tms:
        # the hot path's kernels: index pre-pass (IN-list LUTs, sorted / inverted / MV leaf bitmaps) + selective
        # stream + fused scan (+ the radix-partitioned group-by's passes, reported in scan_ms)
        scan_ms.append(tm.prepass_ms + tm.prefilter_ms + tm.scan_ms)
        for k, v in parts.items():
            v.append(getattr(tm, k))
    value = rows_per_gpu * world * args.steps / el
    # the kernels the last step ran (pg_last_trace), named for the roofline line
    path = set(eng.last_trace()["path"]) if world == 1 else set()
    kernels = [k for p, k in (("prepass", "prepass"), ("stream", "stream_kernel"), ("fused_scan", "scan_kernel"),
                              ("partitioned", "part_direct + part_split2s + part_aggregate"),
                              ("index_count", "index_count_kernel")) if p in path]
    scan_avg_ms = max(float(np.mean(scan_ms)), 1e-9)  # (0 only with the library's phase timings off)
    alg_bytes = fwd_bytes + dict_bytes
    achieved = plan_bytes / (scan_avg_ms * 1e-3) / 1e9
    alg_achieved = alg_bytes / (scan_avg_ms * 1e-3) / 1e9

    cpu = parity = parity_full = None
    host_sample = host_all[:n_sample]
    if want_cpu and host_sample:
        from oracle.oracle import OracleEngine
        from pinot_amd.plan import CPlan
        ht = Table(W["table"], host_sample)
        hq = parse(W["query"])
        orc = OracleEngine()
        cplan = CPlan(ht, hq, host_sample, list(range(1, len(host_sample) + 1)), config=cfg)
        legs = {}
        for name, threads in (("pinot_default", min(len(host_sample), pinot_threads)),
                              ("all_cores", min(len(host_sample), cores))):
            v, runs = orc.time_segments(cplan, host_sample, threads, args.cpu_seconds)
            legs[name] = {"value": v, "threads": threads, "runs": runs}
        best = max(legs.values(), key=lambda x: x["value"])
        cpu = {"value": best["value"], "unit": "rows/s", "cores": best["threads"], "kind": "port",
               "label": "restated Pinot CPU path (oracle/pinot_oracle.c, per-segment operators)",
               "sample": f"{len(host_sample)} of the {args.segments} segments ({len(host_sample) * args.rows} rows), "
                         f"same query; per-segment filter (later AND children on the survivors) -> projection of the "
                         f"matching docs -> aggregation in C, segments as parallel combine tasks; the value-keyed merge "
                         f"of the per-segment results is not timed",
               "legs": legs, "nproc": nproc, "cores_available": cores, "cpu_model": cpu_model()}
        if W["table"] != "events":  # parity on up to 16 sampled segments (value-keyed merge in Python)
            ps = host_sample[:16]
            o = orc.execute(Table(W["table"], ps), hq, config=cfg)
            d = eng.run_plan(eng.make_plan(table, q, segments=segs[:len(ps)], flags=0, config=cfg))
            parity = bool(d.rows == o.rows and d.stats.num_docs_scanned == o.stats.num_docs_scanned)
        else:  # config 4 on 2 full segments: the oracle's per-segment value sets merged by value (numpy), top rows
            from pinot_amd.plan import reduce_to_rows
            ps = host_sample[:2]
            pp = CPlan(Table(W["table"], ps), hq, ps, [1, 2], config=cfg)
            pk, pv = zip(*(orc.distinct_pairs(pp, i, sg) for i, sg in enumerate(ps)))
            pair = np.unique(np.concatenate(pk) * (1 << 20) + np.concatenate(pv))
            users, counts = np.unique(pair >> 20, return_counts=True)
            top = np.lexsort((users, -counts))[:q.limit]
            want = [[int(users[i]), int(counts[i])] for i in top]
            d = eng.run_plan(eng.make_plan(table, q, segments=segs[:2], flags=0, trim=True, config=cfg))
            parity = bool(reduce_to_rows(q, d)[1] == want)
        if not args.no_full_parity and len(host_all) == args.segments:
            t_par = time.perf_counter()
            parity_full = full_parity(W, q, res, host_all, cfg, min(cores, 64))
            parity_full_s = time.perf_counter() - t_par

    traffic = traffic_bytes = None
    traffic_note = None
    tf = args.traffic_file or os.path.join(ROOT, "profiles", f"traffic_{args.workload}.json")
    try:  # rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over this same command (tools/profile_bench.sh)
        tj = json.load(open(tf))
        tc = tj.get("config") or {}
        if tj.get("lib_md5") != lib_md5():
            traffic_note = f"{os.path.relpath(tf, ROOT)} measured on another build: not used"
        elif tc.get("rows_per_gpu") == rows_per_gpu and tc.get("workload") == W["desc"] and \
                tj.get("traffic_bytes_per_launch"):
            traffic_bytes = float(tj["traffic_bytes_per_launch"])
            traffic = traffic_bytes / (scan_avg_ms * 1e-3) / 1e9
    except (OSError, ValueError):
        pass

    if rank == 0:
        out = {
            "metric": W["metric"], "value": value, "unit": "rows/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3, "higher_is_better": True,
            "inflight": inflight, "serial_ms_per_step": round(serial_ms, 4),
            "step_plan_frac": plan_bytes / (el / args.steps) / 1e9 / HBM_PEAK_GBS,
            "inflight_note": "queries in flight in the timed loop: value / ms_per_step time K whole queries with "
                             f"{inflight} host threads issuing them (each its own stream), serial_ms_per_step the "
                             "same K queries one after another; kernel_ms and the roofline come from the serial pass",
            "scaling": "strong" if args.split_table else "weak",
            "vs_baseline": None, "dtype": "int64",
            "data": "synthetic (pinot_amd.synth, seed 42, Pinot segment format, device-generated)",
            "config": {"workload": W["desc"], "rows_per_gpu": rows_per_gpu, "segments_per_gpu": args.segments,
                       "rows_per_segment": args.rows,
                       "in_list_size": args.in_ids if args.workload == "adanalytics" else None,
                       "parallelism": f"segments x{world}" + (" (table split)" if args.split_table else "")},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": " + ".join(kernels) or ("stream_kernel + scan_kernel" if tm.scan_launches > 1
                                                           else "scan_kernel"),
                         "kernel_ms": scan_avg_ms,
                         "plan_bytes": plan_bytes, "stage_docs": stage_docs,
                         "algorithmic_bytes": alg_bytes, "algorithmic_frac": alg_achieved / HBM_PEAK_GBS,
                         "traffic_bytes_per_launch": traffic_bytes,
                         "traffic_frac": traffic / HBM_PEAK_GBS if traffic is not None else None,
                         "traffic_note": traffic_note},
            "cpu_baseline": cpu,
            "parity_full": parity_full,
            "parity_full_scope": None if parity_full is None else
            f"the last timed step's result vs the oracle over all {args.segments} segments "
            f"({round(parity_full_s, 1)} s)",
            "parity_sample": parity,
            "step_breakdown_ms": {k: round(float(np.mean(v)), 4) for k, v in parts.items()},
            "host_plan_lowering_ms": round(lowering_ms, 3),
            "host_plan_lowering_note": "median of 5 same-shape queries with other filter literals, plan + image, "
                                       "table caches warm, no plan cache; cold = the first plan on a new table; "
                                       "relower = the shape cache's hit (CPlan.relower)",
            "host_plan_lowering_cold_ms": round(lowering_cold_ms, 3),
            "host_plan_relower_ms": round(float(np.median(relow)), 3),
            "groups": len(res.rows), "docs_matched": res.stats.num_docs_scanned, "datagen_s": round(gen_s, 1),
            "lib_md5": lib_md5(),
        }
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
