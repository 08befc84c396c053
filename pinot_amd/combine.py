"""Cross-GPU combine: the MI355X replacement of the reference's partial-result merge.

In the reference one server merges its segments' partial results on the host:
AggregationOnlyCombineOperator.mergeResultsBlocks (operator/combine/AggregationOnlyCombineOperator.java:47-57) and
GroupByOrderByCombineOperator.processSegments -> IndexedTable.upsert (operator/combine/GroupByOrderByCombineOperator.java
:127-214, data/table/IndexedTable.java:103-118).  Here segments are sharded over the GPUs of a node (one process per
GPU); each GPU merges its own segments on device inside the fused scan (pg_execute_partial), and the ranks then merge
their dense per-slot state with ONE collective per state array over RCCL / xGMI:

    i64   (doc counts, integer sums, AVG counts, COUNTMV)   all_reduce SUM
    f64   (floating-point sums)                            all_reduce SUM
    mn    (order-preserving int64 image of double MIN)      all_reduce MIN
    mx    (order-preserving int64 image of double MAX)      all_reduce MAX
    flags (DISTINCTCOUNT presence bytes)                    all_reduce MAX
    stats (ExecutionStatistics)                            all_reduce SUM

Sparse / high-cardinality keys use `gather_merge_results`: an all_gather of value-keyed partials merged with the
reference's own AggregationFunction.merge semantics (pinot_amd.plan.merge_intermediate).
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, Optional

import numpy as np

from . import abi
from .plan import ExecutionStats, IntermediateResult, merge_intermediate

_STATS_FIELDS = ["num_docs_scanned", "num_entries_scanned_in_filter", "num_entries_scanned_post_filter",
                 "num_total_docs", "num_segments_processed", "num_segments_matched"]


def allreduce_state(state: Dict[str, "torch.Tensor"], group=None) -> None:
    """In-place merge of a dense partial state across ranks (any backend: RCCL on GPU, gloo in CPU tests)."""
    import torch.distributed as dist
    ops = {"i64": dist.ReduceOp.SUM, "f64": dist.ReduceOp.SUM, "mn": dist.ReduceOp.MIN, "mx": dist.ReduceOp.MAX,
           "flags": dist.ReduceOp.MAX, "stats": dist.ReduceOp.SUM}
    for name in ("i64", "f64", "mn", "mx", "flags", "stats"):
        t = state.get(name)
        if t is not None and t.numel():
            dist.all_reduce(t, op=ops[name], group=group)


def merge_partials_across_ranks(engine, plan, p, group=None) -> IntermediateResult:
    """pg_execute_partial result `p` (this rank) -> all-reduced over the process group -> finalized result.

    The state leaves the library through pg_partials_copy into torch device tensors (RCCL operates on those), is
    reduced in place, and goes back with PG_COPY_IN before pg_partials_finalize decodes it."""
    import torch
    pc = p.contents
    dev = torch.device("cuda", torch.cuda.current_device())
    n = pc.num_slots
    state = {
        "i64": torch.empty(n * pc.n_i64, dtype=torch.int64, device=dev),
        "f64": torch.empty(n * pc.n_f64, dtype=torch.float64, device=dev),
        "mn": torch.empty(n * pc.n_min, dtype=torch.int64, device=dev),
        "mx": torch.empty(n * pc.n_max, dtype=torch.int64, device=dev),
        "flags": torch.empty(n * pc.flag_bytes_per_slot, dtype=torch.uint8, device=dev),
    }
    ptr = lambda t: C.c_void_p(t.data_ptr()) if t.numel() else None
    torch.cuda.synchronize()
    from .gpu import check
    check(engine.lib.pg_partials_copy(p, abi.PG_COPY_OUT, ptr(state["i64"]), ptr(state["f64"]), ptr(state["mn"]),
                                      ptr(state["mx"]), ptr(state["flags"]), None))
    state["stats"] = torch.tensor([getattr(pc.stats, f) for f in _STATS_FIELDS], dtype=torch.int64, device=dev)
    allreduce_state(state, group)
    torch.cuda.synchronize()
    check(engine.lib.pg_partials_copy(p, abi.PG_COPY_IN, ptr(state["i64"]), ptr(state["f64"]), ptr(state["mn"]),
                                      ptr(state["mx"]), ptr(state["flags"]), None))
    for f, v in zip(_STATS_FIELDS, state["stats"].cpu().tolist()):
        setattr(pc.stats, f, int(v))
    return engine.finalize_partial(plan, p)


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
            if v is None:
                continue
            merged[k] = merge_intermediate(res.aggregations, merged[k], v) if k in merged else v
        for f in _STATS_FIELDS:
            setattr(stats, f, getattr(stats, f) + st[f])
    if not res.group_by and () not in merged:
        merged[()] = None
    return IntermediateResult(res.aggregations, res.group_by, merged, stats)
