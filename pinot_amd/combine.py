"""Cross-GPU combine: the MI355X replacement of the reference's partial-result merge.

In the reference one server merges its segments' partial results on the host:
AggregationOnlyCombineOperator.mergeResultsBlocks (operator/combine/AggregationOnlyCombineOperator.java:47-57) and
GroupByOrderByCombineOperator.processSegments -> IndexedTable.upsert (operator/combine/GroupByOrderByCombineOperator.java
:127-214, data/table/IndexedTable.java:103-118).  Here segments are sharded over the GPUs of a node (one process per
GPU); each GPU merges its own segments on device inside the fused scan (pg_execute_partial), and the ranks then merge
their partial states over RCCL / xGMI in one of two ways:

* dense all-reduce -- a small dense key space without DISTINCTCOUNT bitmaps: ONE SUM all-reduce of i64 (doc counts,
    integer sums, AVG counts, COUNTMV), the exact fixed-point sums as 32-bit limbs (pg_partials_copy) and the
    statistics, then MIN / MAX all-reduces of the order-preserving images; every rank holds the merged state (config 2:
    365 slots x 3 int64, latency-bound).  Double sums are exact integers in fixed point (SK_FX), so the merged sum has
    the same bits for every run, every rank count and every collective algorithm.
* row exchange -- hash states, large key spaces, DISTINCTCOUNT (bitmaps merge by OR, which RCCL cannot reduce):
    every rank exports its groups as rows bucketed by owner rank (pg_partials_export, owner = pg_key_owner(key)),
    the buckets go to their owners in one all_to_all, each owner inserts-and-merges what it received into a fresh
    table (pg_partials_merge: SUM / MIN / MAX / OR per state), finalizes ITS keys (ORDER BY trim included), and the
    per-owner results -- disjoint key sets, packed as flat byte buffers (keys, values, counts, value sets) -- are
    all-gathered to every rank as device buffers.  Per-link traffic is (N-1)/N of one rank's groups instead of N
    copies of the key space.  A library error on one rank (e.g. a merge table over the state budget) is agreed on by
    an all-reduce before the next collective, so every rank raises instead of the others waiting forever.

Statistics (ExecutionStatistics) are summed with one all_reduce.  `gather_merge_results` merges value-keyed host
results (oracle / DataTable-level) with the reference's AggregationFunction.merge (pinot_amd.plan.merge_intermediate).
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np

from . import abi
from .plan import ExecutionStats, IntermediateResult, default_row, merge_intermediate, top_groups

_STATS_FIELDS = ["num_docs_scanned", "num_entries_scanned_in_filter", "num_entries_scanned_post_filter",
                 "num_total_docs", "num_segments_processed", "num_segments_matched"]
DENSE_ALLREDUCE_MAX_BYTES = 64 << 20


def _is_gloo(group=None) -> bool:
    import torch.distributed as dist
    return dist.get_backend(group) == "gloo"


def _comm(t, group):
    """The tensor a collective runs on: the device tensor itself over RCCL, a host copy over gloo (CPU tests)."""
    return t.cpu() if _is_gloo(group) else t


def allreduce_state(state, group=None) -> None:
    """In-place merge of a dense partial state across ranks: SUM of the integer words (i64 state, the exact sums'
    32-bit limbs, statistics -- one buffer), MIN / MAX of the order-preserving images.  Every merge is an integer
    operation, so the result is the same bits on every rank, in every run, whatever algorithm RCCL picks (SURVEY.md
    §8(e): reproducible double SUMs)."""
    import torch.distributed as dist
    ops = {"i64": dist.ReduceOp.SUM, "mn": dist.ReduceOp.MIN, "mx": dist.ReduceOp.MAX, "stats": dist.ReduceOp.SUM}
    for name in ("i64", "mn", "mx", "stats"):
        t = state.get(name)
        if t is not None and t.numel():
            c = _comm(t, group)
            dist.all_reduce(c, op=ops[name], group=group)
            if c is not t:
                t.copy_(c)


def _all_gather_ints(vals, group, device):
    import torch
    import torch.distributed as dist
    t = torch.tensor(vals, dtype=torch.int64, device=device)
    c = _comm(t, group)
    out = [torch.empty_like(c) for _ in range(dist.get_world_size(group))]
    dist.all_gather(out, c, group=group)
    return [o.tolist() for o in out]


_FLAG_BITS = (abi.PG_RESULT_GROUPS_LIMIT_REACHED, abi.PG_RESULT_TRIM_THRESHOLD_REACHED)


def _layout_header(err, fp, flags, group, dev):
    """ONE fixed-size MAX all-reduce every step: [error flag | result flag bits | fingerprint | -fingerprint].  Every
    rank then holds the same maxima and minima, so every rank takes the same decision (raise, dense all-reduce or row
    exchange) even when one rank's state layout changed since the last step (a hash table regrown, a DENSE / HASH
    switch), and the OR of the ranks' PG_RESULT_* flags (the combined block's numGroupsLimitReached)."""
    import torch
    import torch.distributed as dist
    v = [1 if err is not None else 0] + [1 if flags & b else 0 for b in _FLAG_BITS] + fp + [-x for x in fp]
    t = torch.tensor(v, dtype=torch.int64, device=dev)
    c = _comm(t, group)
    dist.all_reduce(c, op=dist.ReduceOp.MAX, group=group)
    h = c.tolist()
    n, nb = len(fp), len(_FLAG_BITS)
    merged_flags = sum(b for b, x in zip(_FLAG_BITS, h[1:1 + nb]) if x)
    return h[0], merged_flags, h[1 + nb:1 + nb + n], [-x for x in h[1 + nb + n:]]


def merge_partials_across_ranks(engine, plan, p, group=None) -> IntermediateResult:
    """pg_execute_partial result `p` (this rank) -> merged over the process group -> finalized result (every rank
    returns the same merged result).  Consumes `p`.

    Per step: one MAX all-reduce of a fixed-size header (error flag, result flags, state-layout fingerprint,
    _layout_header), then for dense states the i64 state, the exact sums' limbs and the six statistics in ONE SUM
    all-reduce (config 2: that is all) and MIN / MAX all-reduces for MIN / MAX states; other states take the row
    exchange."""
    import torch
    from .gpu import check
    pc = p.contents
    dev = torch.device("cuda", torch.cuda.current_device())
    fp = [pc.mode, pc.num_slots, pc.n_i64, pc.n_fx, pc.n_min, pc.n_max, pc.bitmap_words, pc.layout, pc.fx_sig]
    st_host = [getattr(pc.stats, f) for f in _STATS_FIELDS]
    n = pc.num_slots
    ni = n * pc.n_i64
    nf = n * pc.n_fx * 4  # the exact sums as 32-bit limbs (pg_partials_copy)
    dense_mine = pc.mode == abi.PG_STATE_DENSE and pc.bitmap_words == 0 and \
        n * 8 * (pc.n_i64 + 4 * pc.n_fx + pc.n_min + pc.n_max) <= DENSE_ALLREDUCE_MAX_BYTES
    err = state = sums = None
    ptr = lambda t: C.c_void_p(t.data_ptr()) if t.numel() else None
    if dense_mine:
        # the library's copies run on its own stream (torch carries its own HIP runtime, so streams do not cross) and
        # return once done
        try:
            # i64 state | fx limbs | statistics: one SUM all-reduce
            sums = torch.empty(ni + nf + len(_STATS_FIELDS), dtype=torch.int64, device=dev)
            sums[ni + nf:].copy_(torch.tensor(st_host, dtype=torch.int64), non_blocking=False)
            state = {"i64": sums[:ni], "fx": sums[ni:ni + nf],
                     "mn": torch.empty(n * pc.n_min, dtype=torch.int64, device=dev),
                     "mx": torch.empty(n * pc.n_max, dtype=torch.int64, device=dev)}
            check(engine.lib.pg_partials_copy(p, abi.PG_COPY_OUT, ptr(state["i64"]), ptr(state["fx"]),
                                              ptr(state["mn"]), ptr(state["mx"]), None))
        except Exception as e:  # noqa: BLE001 -- agreed on below, raised on every rank
            err = e
    any_err, flags, hi, lo = _layout_header(err, fp, pc.flags, group, dev)
    if any_err:
        engine.lib.pg_partials_free(p)
        if err is not None:
            raise err
        raise RuntimeError("the cross-GPU merge failed on another rank")
    if hi[2:] != lo[2:]:
        engine.lib.pg_partials_free(p)
        raise ValueError(f"partial state layouts differ across ranks: max {hi}, min {lo} (a plan with PG_PLAN_F64_SUMS "
                         f"and table-global sum bounds, pg_agg.sum_exp)")
    pc.flags = flags
    dense_all = hi[:2] == lo[:2] and hi[0] == abi.PG_STATE_DENSE   # every rank dense over the same slots
    if not (dense_all and dense_mine):  # dense_mine is a function of the (now known equal) layout: same on all ranks
        return _exchange_rows(engine, plan, p, torch.tensor(st_host, dtype=torch.int64, device=dev), flags, group, dev)
    allreduce_state({"i64": sums, "mn": state["mn"], "mx": state["mx"]}, group)
    for f, v in zip(_STATS_FIELDS, sums[ni + nf:].cpu().tolist()):  # waits for the collectives
        setattr(pc.stats, f, int(v))
    if state["mn"].numel() or state["mx"].numel():
        torch.cuda.synchronize()
    try:
        check(engine.lib.pg_partials_copy(p, abi.PG_COPY_IN, ptr(state["i64"]), ptr(state["fx"]), ptr(state["mn"]),
                                          ptr(state["mx"]), None))
    except Exception:
        engine.lib.pg_partials_free(p)
        raise
    return engine.finalize_partial(plan, p)


def _agree(err, group, dev):
    """MAX-all-reduce of an error flag: every rank learns that some rank's library call failed (then all raise)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([1 if err is not None else 0], dtype=torch.int64, device=dev)
    c = _comm(t, group)
    dist.all_reduce(c, op=dist.ReduceOp.MAX, group=group)
    if err is not None:
        raise err
    if int(c.item()):
        raise RuntimeError("the cross-GPU merge failed on another rank")


def _pack_result(ra) -> np.ndarray:
    """One rank's finalized result arrays as a flat byte buffer: [G, K, A, num_distinct, has_sets, flags, merged,
    6 stats] int64 | keys uint32 | values float64 | counts int64 | offsets uint64 | ids uint32 (8-byte aligned
    sections)."""
    has = ra["offsets"] is not None
    nd = len(ra["ids"]) if has else 0
    parts = [np.array([ra["G"], ra["K"], ra["A"], nd, int(has), ra.get("flags", 0), ra.get("merged", 0)],
                      dtype=np.int64), ra["stats"].astype(np.int64),
             ra["keys"].astype(np.uint32).ravel(), ra["values"].astype(np.float64).ravel(),
             ra["counts"].astype(np.int64).ravel()]
    if has:
        parts += [ra["offsets"].astype(np.uint64), ra["ids"].astype(np.uint32)]
    out = bytearray()
    for a in parts:
        b = a.tobytes()
        out += b + bytes((-len(b)) % 8)
    return np.frombuffer(bytes(out), dtype=np.uint8)


def _unpack_result(buf: np.ndarray) -> dict:
    b = buf.tobytes()
    pos = 0

    def take(dtype, n):
        nonlocal pos
        a = np.frombuffer(b, dtype=dtype, count=n, offset=pos).copy()
        pos += -(-a.nbytes // 8) * 8
        return a
    G, K, A, nd, has, flags, merged = (int(x) for x in take(np.int64, 7))
    stats = take(np.int64, 6)
    keys = take(np.uint32, G * K).reshape(G, K)
    vals = take(np.float64, G * A).reshape(G, A)
    cnts = take(np.int64, G * A).reshape(G, A)
    offs = take(np.uint64, G * A + 1) if has else None
    ids = take(np.uint32, nd) if has else None
    return {"G": G, "K": K, "A": A, "keys": keys, "values": vals, "counts": cnts, "offsets": offs, "ids": ids,
            "stats": stats, "flags": flags, "merged": merged}


def _exchange_rows(engine, plan, p, stats, flags, group, dev) -> IntermediateResult:
    import torch
    import torch.distributed as dist
    pc = p.contents
    world = dist.get_world_size(group)
    rb = pc.row_bytes
    gloo = _is_gloo(group)
    err = q = None
    counts, send = [0] * world, None
    try:
        counts = engine.export_rows(p, world)  # rows per owner rank
    except Exception as e:  # noqa: BLE001 -- agreed on below, re-raised on every rank
        err = e
        engine.lib.pg_partials_free(p)
    _agree(err, group, dev)
    sc = torch.tensor(counts, dtype=torch.int64, device="cpu" if gloo else dev)
    rcounts = torch.empty_like(sc)
    dist.all_to_all_single(rcounts, sc, group=group)
    rcounts = rcounts.tolist()
    try:
        q = engine.create_like(p, max(sum(rcounts), 1))
        send = torch.empty(max(sum(counts), 1) * rb, dtype=torch.uint8, device=dev)
        engine.export_rows(p, world, C.c_void_p(send.data_ptr()), sum(counts))
    except Exception as e:  # noqa: BLE001
        err = e
        if q is not None:  # created, then the export failed: free the fresh table before every rank raises
            engine.lib.pg_partials_free(q)
            q = None
    finally:
        engine.lib.pg_partials_free(p)
    _agree(err, group, dev)
    recv = torch.empty(max(sum(rcounts), 1) * rb, dtype=torch.uint8, device=dev)
    s_in, r_in = (send.cpu(), torch.empty(recv.numel(), dtype=torch.uint8)) if gloo else (send, recv)
    dist.all_to_all_single(r_in[:sum(rcounts) * rb], s_in[:sum(counts) * rb],
                           output_split_sizes=[c * rb for c in rcounts], input_split_sizes=[c * rb for c in counts],
                           group=group)
    if gloo:
        recv.copy_(r_in)
    st = _comm(stats, group)
    dist.all_reduce(st, op=dist.ReduceOp.SUM, group=group)
    torch.cuda.synchronize()
    ra = None
    try:
        engine.merge_rows(q, C.c_void_p(recv.data_ptr()), sum(rcounts))
        for f, v in zip(_STATS_FIELDS, st.cpu().tolist()):
            setattr(q.contents.stats, f, int(v))
        q.contents.flags = flags & abi.PG_RESULT_GROUPS_LIMIT_REACHED  # the threshold is judged on the union below
        ra = engine.finalize_arrays(plan, q)  # this rank's keys (their ORDER BY trim included); frees q
        q = None
    except Exception as e:  # noqa: BLE001
        err = e
    finally:
        if q is not None:
            engine.lib.pg_partials_free(q)
    _agree(err, group, dev)
    # the owners' results (disjoint key sets) to every rank: sizes, then one all_gather of padded byte buffers
    mine = _pack_result(ra)
    sizes = _all_gather_ints([mine.size], group, dev)
    mx = max(s[0] for s in sizes)
    buf = torch.zeros(mx, dtype=torch.uint8, device="cpu" if gloo else dev)
    buf[:mine.size] = torch.from_numpy(mine.copy())
    outs = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(outs, buf, group=group)
    rows = {}
    res = None
    n_merged = 0  # the owners' key sets are disjoint: the combined table holds their sum
    for o, sz in zip(outs, sizes):
        ra_o = _unpack_result(o[:sz[0]].cpu().numpy())
        n_merged += ra_o["merged"]
        res = engine.decode(plan, ra_o)
        rows.update(res.rows)
    if not plan.query.group_by and () not in rows:  # no rank matched a doc
        rows[()] = default_row(res.aggregations)
    if plan.plan.flags & abi.PG_PLAN_EXACT_LIMIT and plan.plan.limit and len(rows) > plan.plan.limit:
        # the server's result size over the union of the owners' kept rows (each owner kept its own top `limit`)
        rows = top_groups(plan.query, res.aggregations, rows, plan.plan.limit)
    # every owner carries the statistics summed over the ranks
    thr = plan.plan.trim_threshold
    return IntermediateResult(res.aggregations, res.group_by, rows, ExecutionStats(*(int(x) for x in ra["stats"])),
                              bool(flags & abi.PG_RESULT_GROUPS_LIMIT_REACHED),
                              bool(plan.query.group_by and plan.query.order_by and thr and n_merged >= thr),
                              n_merged if plan.query.group_by else None)


def gather_merge_results(res: IntermediateResult, group=None) -> IntermediateResult:
    """Sparse merge: all_gather the value-keyed partials of every rank, merge by key in rank order (a fixed order,
    so double sums are reproducible), as GroupByOrderByCombineOperator merges per-segment blocks."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    parts = [None] * world
    dist.all_gather_object(parts, (res.rows, res.stats.__dict__), group=group)
    merged = {}
    stats = ExecutionStats()
    for rows, st in parts:
        for k, v in rows.items():
            merged[k] = merge_intermediate(res.aggregations, merged[k], v) if k in merged else v
        for f in _STATS_FIELDS:
            setattr(stats, f, getattr(stats, f) + st[f])
    if not res.group_by and () not in merged:
        merged[()] = default_row(res.aggregations)
    return IntermediateResult(res.aggregations, res.group_by, merged, stats)
