"""Python driver of the C oracle (oracle/pinot_oracle.c).  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and only
as the checker.  The product path (pinot_amd.gpu) never imports it.

Executes a lowered plan segment by segment with the restated Pinot operators, then merges the
per-segment results by VALUE key exactly like the combine operators do:
  AggregationOnlyCombineOperator.mergeResultsBlocks (operator/combine/AggregationOnlyCombineOperator.java:47-57),
  GroupByOrderByCombineOperator.processSegments -> IndexedTable.upsert (operator/combine/GroupByOrderByCombineOperator.java:127-214,
  data/table/IndexedTable.java:103-118), with DISTINCTCOUNT sets converted from dictIds to values at
  extraction (DistinctCountAggregationFunction.extractAggregationResult, function/DistinctCountAggregationFunction.java:252-310).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from concurrent.futures import ThreadPoolExecutor
from typing import List, Optional, Sequence

import numpy as np

from pinot_amd import abi
from pinot_amd.segment import _NP_BE
from pinot_amd.plan import (MAX_TRIM_THRESHOLD, CPlan, ExecutionStats, IntermediateResult, Table, default_row,
                            execute_filtered, final_value, group_trim, has_filtered_aggregations, merge_intermediate)
from pinot_amd.query import QueryContext, parse
from pinot_amd.segment import ImmutableSegment

_HERE = os.path.dirname(os.path.abspath(__file__))
# PINOT_ORACLE_LIB: the sanitizer build of the same source (tests/test_sanitizers.py)
LIB = os.environ.get("PINOT_ORACLE_LIB") or os.path.join(_HERE, "libpinot_oracle.so")
ORC_FWD_SV, ORC_FWD_SORTED, ORC_FWD_MV, ORC_FWD_RAW = 0, 1, 2, 3


class orc_column(C.Structure):
    _fields_ = [("dict", C.c_void_p), ("fwd", C.c_void_p), ("inv", C.c_void_p), ("inv_bytes", C.c_uint64),
                ("keymap", C.c_void_p), ("fwd_kind", C.c_uint32), ("data_type", C.c_uint32),
                ("num_docs", C.c_uint32), ("cardinality", C.c_uint32), ("bits", C.c_uint32),
                ("num_values", C.c_uint32), ("entry_bytes", C.c_uint32), ("pad", C.c_uint32),
                ("range", C.c_void_p), ("range_bytes", C.c_uint64)]


class orc_segment_result(C.Structure):
    _fields_ = [("stats", abi.pg_stats), ("num_groups", C.c_uint64), ("num_keys", C.c_uint32),
                ("num_aggs", C.c_uint32), ("key_dict_ids", C.POINTER(C.c_int32)),
                ("values", C.POINTER(C.c_double)), ("counts", C.POINTER(C.c_int64)),
                ("num_distinct", C.c_uint64), ("distinct_group_agg", C.POINTER(C.c_uint64)),
                ("distinct_dict_ids", C.POINTER(C.c_int32))]


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        lib = C.CDLL(LIB)
        lib.orc_execute_segment.argtypes = [C.POINTER(abi.pg_plan), C.c_uint32, C.POINTER(orc_column), C.c_uint64,
                                            C.POINTER(C.POINTER(orc_segment_result))]
        lib.orc_execute_segment.restype = C.c_int
        lib.orc_result_free.argtypes = [C.POINTER(orc_segment_result)]
        lib.orc_unpack.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint32, C.c_void_p]
        lib.orc_roaring_decode.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32]
        lib.orc_num_bits_per_value.argtypes = [C.c_int32]
        lib.orc_num_bits_per_value.restype = C.c_int
        _lib = lib
    return _lib


class _SegmentColumns:
    """orc_column array for one segment, indexed by table column id (keeps the byte buffers alive)."""

    def __init__(self, seg: ImmutableSegment, table: Table):
        n = len(table.column_ids)
        self.arr = (orc_column * max(n, 1))()
        self.keep = []
        for name, col in seg.columns.items():
            c = self.arr[table.column_ids[name]]
            if col.dictionary is None and col.data_type in ("STRING", "BYTES"):
                # raw var-byte column: the oracle keys it by each doc's value id (equal values, equal ids -- the
                # generators' first-seen order over values is the same over ids); decoded back from raw_values
                _, ids = np.unique(np.asarray(col.raw_values, dtype=str), return_inverse=True)
                d = np.frombuffer(ids.astype(">i4").tobytes() or b"\0", dtype=np.uint8)
                self.keep.append(d)
                c.dict = d.ctypes.data
                c.fwd_kind = ORC_FWD_RAW
                c.data_type = abi.PG_INT
                c.num_docs = c.cardinality = c.num_values = col.num_docs
                c.entry_bytes = 4
                continue
            if col.dictionary is None:  # raw forward index: the decoded values stand in for the dictionary
                d = np.frombuffer(col.raw_values.astype(_NP_BE[col.data_type]).tobytes() or b"\0", dtype=np.uint8)
            else:
                d = np.frombuffer(col.dictionary.to_bytes() or b"\0", dtype=np.uint8)
            f = np.frombuffer(col.fwd or b"\0", dtype=np.uint8)
            self.keep += [d, f]
            c.dict = d.ctypes.data
            c.fwd = f.ctypes.data
            if col.inverted is not None:
                iv = np.frombuffer(col.inverted, dtype=np.uint8)
                self.keep.append(iv)
                c.inv = iv.ctypes.data
                c.inv_bytes = len(col.inverted)
            if col.range_index is not None:
                rg = np.frombuffer(col.range_index, dtype=np.uint8)
                self.keep.append(rg)
                c.range = rg.ctypes.data
                c.range_bytes = len(col.range_index)
            c.fwd_kind = {"sv": ORC_FWD_SV, "sorted": ORC_FWD_SORTED, "mv": ORC_FWD_MV, "raw": ORC_FWD_RAW}[col.fwd_kind]
            c.data_type = abi.DTYPE_CODES[col.data_type]
            c.num_docs = col.num_docs
            c.cardinality = col.cardinality if col.dictionary is not None else col.num_docs
            c.bits = col.bits_per_element
            c.num_values = col.num_values
            c.entry_bytes = col.dictionary.entry_bytes if col.dictionary is not None else \
                np.dtype(_NP_BE[col.data_type]).itemsize


class OracleEngine:
    """Runs plans on the CPU restatement.  `threads` parallelises over segments (ctypes drops the GIL)."""

    def __init__(self, threads: int = 1):
        self.lib = load()
        self.threads = threads
        self._cols = {}

    @staticmethod
    def _array_threshold(plan: CPlan) -> int:
        """DictionaryBasedGroupKeyGenerator's array-based holder bound: the instance's maxInitialResultHolderCapacity
        (<= its numGroupsLimit, InstancePlanMakerImplV2.java:138-140)."""
        return min(plan.config.max_init_group_holder_capacity, plan.config.num_groups_limit)

    def columns(self, seg, table):
        k = (id(seg), id(table))
        if k not in self._cols:
            self._cols[k] = (seg, table, _SegmentColumns(seg, table))  # refs keep the ids valid
        return self._cols[k][2]

    def run_segment(self, plan: CPlan, si: int, seg: ImmutableSegment):
        cols = self.columns(seg, plan.table)
        out = C.POINTER(orc_segment_result)()
        rc = self.lib.orc_execute_segment(C.byref(plan.plan), si, cols.arr, self._array_threshold(plan), C.byref(out))
        if rc:
            raise RuntimeError(f"oracle failed rc={rc}")
        try:
            return self._to_value_rows(plan, seg, out.contents)
        finally:
            self.lib.orc_result_free(out)

    def distinct_pairs(self, plan: CPlan, si: int, seg: ImmutableSegment):
        """(group key value, distinct value) pairs of one segment for a one-key, one-DISTINCTCOUNT plan: the
        segment's per-group value sets (DistinctCountAggregationFunction's Set intermediate) as two int64 arrays, so a
        caller can merge many segments by value without a Python object per group."""
        cols = self.columns(seg, plan.table)
        out = C.POINTER(orc_segment_result)()
        if self.lib.orc_execute_segment(C.byref(plan.plan), si, cols.arr, self._array_threshold(plan), C.byref(out)):
            raise RuntimeError("oracle failed")
        try:
            r = out.contents
            A, G, nd = r.num_aggs, r.num_groups, r.num_distinct
            kd = np.ctypeslib.as_array(r.key_dict_ids, shape=(max(G, 1),))[:G].astype(np.int64)
            ga = np.ctypeslib.as_array(r.distinct_group_agg, shape=(max(nd, 1),))[:nd].astype(np.int64)
            di = np.ctypeslib.as_array(r.distinct_dict_ids, shape=(max(nd, 1),))[:nd].astype(np.int64)
            kcol = seg.columns[plan.query.group_by[0]].dictionary.values
            vcol = seg.columns[plan.aggs[0].arg.cols[0]].dictionary.values
            return np.asarray(kcol, dtype=np.int64)[kd[ga // A]], np.asarray(vcol, dtype=np.int64)[di]
        finally:
            self.lib.orc_result_free(out)

    def time_segments(self, plan: CPlan, segments: Sequence[ImmutableSegment], threads: int, seconds: float):
        """Throughput of the per-segment operators alone (filter -> projection -> aggregation / group-by of every
        segment, C, `threads` segments in flight as Pinot's combine worker tasks run them; the value-keyed merge is
        excluded).  Runs the whole segment list repeatedly for at least `seconds`; returns (rows/s, runs)."""
        cols = [self.columns(s, plan.table) for s in segments]
        threshold = self._array_threshold(plan)

        def one(i):
            out = C.POINTER(orc_segment_result)()
            rc = self.lib.orc_execute_segment(C.byref(plan.plan), i, cols[i].arr, threshold, C.byref(out))
            if rc:
                raise RuntimeError(f"oracle failed rc={rc}")
            self.lib.orc_result_free(out)

        import time
        rows = sum(s.num_docs for s in segments)
        with ThreadPoolExecutor(threads) as ex:
            list(ex.map(one, range(len(segments))))  # warm-up
            runs, t0 = 0, time.perf_counter()
            while True:
                list(ex.map(one, range(len(segments))))
                runs += 1
                el = time.perf_counter() - t0
                if el >= seconds:
                    break
        return runs * rows / el, runs

    def _to_value_rows(self, plan: CPlan, seg: ImmutableSegment, r: orc_segment_result):
        A, K, G = r.num_aggs, r.num_keys, r.num_groups
        aggs = plan.aggs
        vals = np.ctypeslib.as_array(r.values, shape=(G * A,)).reshape(G, A).copy() if G and A else np.zeros((G, A))
        cnts = np.ctypeslib.as_array(r.counts, shape=(G * A,)).reshape(G, A).copy() if G and A else \
            np.zeros((G, A), dtype=np.int64)
        keys = np.ctypeslib.as_array(r.key_dict_ids, shape=(G * K,)).reshape(G, K).copy() if G and K else \
            np.zeros((G, K), dtype=np.int32)
        distinct = {}
        if r.num_distinct:
            ga = np.ctypeslib.as_array(r.distinct_group_agg, shape=(r.num_distinct,))
            di = np.ctypeslib.as_array(r.distinct_dict_ids, shape=(r.num_distinct,))
            for g_a, d in zip(ga.tolist(), di.tolist()):
                distinct.setdefault(g_a, []).append(d)
        # a raw key column's "dictId" is a doc holding the value (orc_execute_segment's no-dictionary generator)
        key_vals = [seg.columns[c].dictionary.values if seg.columns[c].dictionary is not None
                    else seg.columns[c].raw_values for c in plan.query.group_by]
        rows = {}
        for g in range(G):
            key = tuple(_py(key_vals[k][int(keys[g, k])]) for k in range(K))
            row = []
            for a, ag in enumerate(aggs):
                f = ag.function
                v = float(vals[g, a])
                if f in ("COUNT", "COUNTMV"):
                    row.append(int(v))
                elif f == "AVG":
                    row.append((v, int(cnts[g, a])))
                elif f == "DISTINCTCOUNT":
                    col = seg.columns[ag.arg.cols[0]]
                    dv = col.dictionary.values if col.dictionary is not None else col.raw_values  # raw: doc ids
                    row.append({_py(dv[i]) for i in distinct.get(g * A + a, [])})
                else:
                    row.append(v)
            rows[key] = row
        s = r.stats
        st = ExecutionStats(s.num_docs_scanned, s.num_entries_scanned_in_filter, s.num_entries_scanned_post_filter,
                            s.num_total_docs, s.num_segments_processed, s.num_segments_matched)
        return rows, st

    def execute(self, table: Table, query, segments: Optional[Sequence[ImmutableSegment]] = None,
                server: bool = False, config=None) -> IntermediateResult:
        """config: the server instance's settings (InstanceConfig: numGroupsLimit, maxInitialResultHolderCapacity, trim
        sizes / threshold).  server=True: the reference server's combined result -- the per-segment trim when
        minSegmentGroupTrimSize is on, the IndexedTable's result size (group_trim) -- instead of every merged group."""
        if isinstance(query, str):
            query = parse(query)
        if has_filtered_aggregations(query):  # FilteredAggregationOperator.java:70-98: one plan per filter
            return execute_filtered(lambda q: self.execute(table, q, segments, config=config), query)
        segments = list(table.segments if segments is None else segments)
        plan = CPlan(table, query, segments, list(range(1, len(segments) + 1)), config=config)
        trim = group_trim(query, config) if server and query.group_by else None
        return self.run_plan(plan, segments, trim)

    def run_plan(self, plan: CPlan, segments: Sequence[ImmutableSegment], trim=None) -> IntermediateResult:
        if self.threads > 1:
            with ThreadPoolExecutor(self.threads) as ex:
                parts = list(ex.map(lambda i: self.run_segment(plan, i, segments[i]), range(len(segments))))
        else:
            parts = [self.run_segment(plan, i, s) for i, s in enumerate(segments)]
        q = plan.query
        merged = {}
        stats = ExecutionStats()
        limit = plan.config.num_groups_limit
        # AggregationGroupByOrderByOperator.java:112-113: numGroupsLimitReached when a segment's generator holds >= limit
        limit_reached = bool(q.group_by) and any(len(rows) >= limit for rows, _ in parts)
        closed = False  # IndexedTable without ORDER BY: no new keys once it holds resultSize (ConcurrentIndexedTable:76-86)
        for rows, st in parts:
            if trim is not None and trim.segment_size is not None and len(rows) > trim.segment_size:
                rows = resizer_top(q, plan.aggs, rows, trim.segment_size)  # AggregationGroupByOrderByOperator:118-132
            for k, v in rows.items():
                if k in merged:
                    merged[k] = merge_intermediate(plan.aggs, merged[k], v)
                elif not closed:
                    merged[k] = v
                    closed = trim is not None and not trim.ordered and trim.server_size is not None and \
                        len(merged) >= trim.server_size
            for f in stats.__dataclass_fields__:
                setattr(stats, f, getattr(stats, f) + getattr(st, f))
        n_merged = len(merged)
        # ConcurrentIndexedTable.upsertWithOrderBy (:61-65) resizes whenever the map holds >= trimThreshold records;
        # until its first resize the map holds every merged key, so it resizes iff the merged keys reach the threshold
        # (the resize itself is lossy and depends on thread scheduling: it is reported, not reproduced)
        resized = trim is not None and trim.ordered and trim.server_size is not None and \
            trim.threshold < MAX_TRIM_THRESHOLD and n_merged >= trim.threshold
        if trim is not None and trim.ordered and trim.server_size is not None and len(merged) > trim.server_size:
            merged = resizer_top(q, plan.aggs, merged, trim.server_size)  # IndexedTable.finish
        if not q.group_by and () not in merged:
            merged[()] = default_row(plan.aggs)
        return IntermediateResult(plan.aggs, list(q.group_by), merged, stats, limit_reached, resized,
                                  n_merged if q.group_by else None)


class _Rec:
    """An IntermediateRecord under TableResizer's comparator REVERSED (TableResizer.java:100-115, :164-175): the
    heap root is the kept record that ranks last."""
    __slots__ = ("key", "row", "vals", "asc")

    def __init__(self, key, row, vals, asc):
        self.key, self.row, self.vals, self.asc = key, row, vals, asc

    def cmp(self, other) -> int:  # the ORDER BY comparator: < 0 when self ranks before other
        for x, y, a in zip(self.vals, other.vals, self.asc):
            if x != y:
                return (-1 if x < y else 1) if a else (1 if x < y else -1)
        return 0

    def __lt__(self, other):  # reversed: the record ranking later is "smaller" (sits at the heap root)
        return self.cmp(other) > 0


def resizer_top(query: QueryContext, aggs, rows: dict, size: int) -> dict:
    """TableResizer.getTopRecords / trimInSegmentResults (data/table/TableResizer.java:160-310) restated: a heap of
    `size` records whose root is the worst kept one; each further record replaces the root when it ranks before it.
    Records the ORDER BY ties at the boundary are kept in arrival order (the reference's choice is arbitrary).  The
    order-by values are the group-by values and extractFinalResult of the aggregations (:121-150)."""
    import heapq
    if len(rows) <= size:
        return rows
    asc = [o.asc for o in query.order_by]

    def rec(k, v):
        vals = [final_value(aggs[aggs.index(o.agg)], v[aggs.index(o.agg)]) if o.kind == "AGG"
                else k[query.group_by.index(o.column)] for o in query.order_by]
        return _Rec(k, v, vals, asc)
    it = iter(rows.items())
    heap = [rec(k, v) for k, v in (next(it) for _ in range(size))]
    heapq.heapify(heap)
    for k, v in it:
        r = rec(k, v)
        if r.cmp(heap[0]) < 0:
            heapq.heapreplace(heap, r)
    return {r.key: r.row for r in heap}


def _py(v):
    if isinstance(v, (np.integer,)):
        return int(v)
    if isinstance(v, (np.floating,)):
        return float(v)
    return v
