"""GPU engine: loads libpinot_gpu.so (in-tree, gfx950) and drives it through the C ABI.

There is deliberately NO fallback here: if the HIP library is missing or the device is absent the
engine raises.  Falling back to the CPU is the caller's (Pinot's) decision on PG_E_UNSUPPORTED.
"""
from __future__ import annotations

import collections
import ctypes as C
import dataclasses
import importlib.util
import itertools
import os
import threading
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import abi
from .plan import (MAX_TRIM_THRESHOLD, CPlan, ExecutionStats, InstanceConfig, IntermediateResult, Table,
                   UnsupportedQuery, execute_filtered, group_trim, has_filtered_aggregations, merge_intermediate,
                   query_shape, top_groups)
from .query import QueryContext, parse
from .segment import Column, Dictionary, ImmutableSegment, num_bits_per_value, pack_bits

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PINOT_GPU_LIB", os.path.join(_HERE, "libpinot_gpu.so"))
_lib = None
_lib_lock = threading.Lock()


class PinotGpuError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{abi.STATUS_NAMES.get(code, code)}: {msg}")
        self.code = code


def load_library(path: str = LIB_PATH):
    """Load libpinot_gpu.so; raises if it has not been built (python __graft_entry__.py build)."""
    global _lib
    with _lib_lock:
        if _lib is None:
            if not os.path.exists(path):
                raise FileNotFoundError(f"{path} missing: build it with `make -C pinot_amd/csrc`")
            # one HIP runtime per process: torch's bundled libamdhip64 carries the same SONAME (libamdhip64.so.7) as
            # the /opt/rocm one the library is linked against, so with torch loaded first the dynamic linker binds the
            # library to torch's runtime instead of mapping a second one beside it (torch loaded after the library
            # would map its own); the Python host uses torch for device memory and streams, so load it first
            if importlib.util.find_spec("torch") is not None:
                import torch  # noqa: F401
            _lib = abi.declare(C.CDLL(path))
            if _lib.pg_abi_version() != abi.PG_ABI_VERSION:
                raise RuntimeError("libpinot_gpu ABI version mismatch")
        return _lib


def check(rc: int):
    if rc != abi.PG_OK:
        lib = load_library()
        buf = C.create_string_buffer(2048)
        lib.pg_last_error(buf, 2048)
        err = PinotGpuError(rc, buf.value.decode(errors="replace"))
        if rc == abi.PG_E_UNSUPPORTED:
            raise UnsupportedQuery(str(err))
        raise err


_seg_counter = itertools.count(1)


def fwd_desc(col: Column) -> abi.pg_col_desc:
    d = abi.pg_col_desc()
    d.kind = {"sv": abi.PG_IDX_FWD_SV_BITPACKED, "sorted": abi.PG_IDX_FWD_SV_SORTED,
              "mv": abi.PG_IDX_FWD_MV_BITPACKED, "raw": abi.PG_IDX_FWD_SV_RAW}[col.fwd_kind]
    d.data_type = abi.DTYPE_CODES[col.data_type]
    d.num_docs = col.num_docs
    d.cardinality = col.cardinality
    d.bits_per_element = col.bits_per_element
    d.num_values = col.num_values
    d.entry_bytes = col.dictionary.entry_bytes if col.dictionary is not None else \
        {"INT": 4, "LONG": 8, "FLOAT": 4, "DOUBLE": 8}[col.data_type]
    return d


class GpuEngine:
    """One engine per process: bound to one GPU (one process per GPU; the ranks merge over RCCL, pinot_amd.combine),
    or with `devices` to several logical devices of this process (pg_init_devices: segments placed on them
    round-robin or by `place`, every query merged across them inside the library)."""

    def __init__(self, device: int = 0, devices: Optional[Sequence[int]] = None):
        self.lib = load_library()
        if devices is not None:
            arr = (C.c_int * len(devices))(*devices)
            check(self.lib.pg_init_devices(arr, len(devices)))
            device = devices[0]
        else:
            check(self.lib.pg_init(device))
        self.device = device
        self.devices = list(devices) if devices is not None else [device]
        self._seg_keys: Dict[int, tuple] = {}    # id(segment) -> (segment, seg_key); holds the segment alive
        self._keymaps_uploaded = set()
        self._plans: "collections.OrderedDict[tuple, tuple]" = collections.OrderedDict()  # compiled-plan cache
        self._plan_lock = threading.Lock()
        self.plan_cache_hits = 0
        self.plan_cache_misses = 0
        self.plan_shape_hits = 0   # a cached plan of the same shape re-lowered for new filter literals

    # ---- residency (IndexingOverrides reader-provider hook)
    def upload_segment(self, seg: ImmutableSegment, table: Table, ldev: Optional[int] = None) -> int:
        """Make a segment resident (once); ldev: its logical device (pg_segment_place), else the library's
        round-robin placement."""
        hit = self._seg_keys.get(id(seg))
        if hit is not None:
            return hit[1]
        key = next(_seg_counter)
        if ldev is not None:
            check(self.lib.pg_segment_place(key, ldev))
        for name, col in seg.columns.items():
            cid = table.column_ids[name]
            if col.dictionary is None and col.data_type in ("STRING", "BYTES"):
                continue  # raw STRING / BYTES: resident only as its derived key encoding (upload_keymaps)
            d = fwd_desc(col)
            if col.dictionary is not None:  # raw columns: the chunked forward index alone
                dd = abi.pg_col_desc.from_buffer_copy(d)
                dd.kind = abi.PG_IDX_DICT
                self._upload(key, cid, dd, col.dictionary.to_bytes())
            self._upload(key, cid, d, col.fwd)
            if col.inverted is not None:
                di = abi.pg_col_desc.from_buffer_copy(d)
                di.kind = abi.PG_IDX_INV_BITMAP
                self._upload(key, cid, di, col.inverted)
            if col.range_index is not None:  # after the forward index: its device form derives from it
                dr = abi.pg_col_desc.from_buffer_copy(d)
                dr.kind = abi.PG_IDX_RANGE
                self._upload(key, cid, dr, col.range_index)
        self._seg_keys[id(seg)] = (seg, key)
        return key

    def register_device_segment(self, seg: ImmutableSegment, table: Table, dev_cols) -> int:
        """Make a segment resident from DEVICE buffers in the reference's byte layout (PG_SRC_DEVICE): used for
        synthetic segments generated on the GPU (pinot_amd.synth.DeviceColumn); `seg` carries the host metadata
        and dictionaries, as the reference keeps them on heap."""
        key = next(_seg_counter)
        for dc in dev_cols:
            col = seg.columns[dc.spec.name]
            cid = table.column_ids[dc.spec.name]
            d = fwd_desc(col)
            d.flags = abi.PG_SRC_DEVICE
            dd = abi.pg_col_desc.from_buffer_copy(d)
            dd.kind = abi.PG_IDX_DICT
            check(self.lib.pg_column_upload(key, cid, C.byref(dd), C.c_void_p(dc.dict_be.data_ptr()),
                                            dc.dict_be.numel()))
            check(self.lib.pg_column_upload(key, cid, C.byref(d), C.c_void_p(dc.fwd_be.data_ptr()),
                                            dc.fwd_be.numel()))
            if getattr(dc, "inv_be", None) is not None:
                di = abi.pg_col_desc.from_buffer_copy(d)
                di.kind = abi.PG_IDX_INV_BITMAP
                check(self.lib.pg_column_upload(key, cid, C.byref(di), C.c_void_p(dc.inv_be.data_ptr()),
                                                dc.inv_be.numel()))
        self._seg_keys[id(seg)] = (seg, key)
        return key

    def _upload(self, key, cid, desc, data: bytes):
        buf = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, dtype=np.uint8)
        check(self.lib.pg_column_upload(key, cid, C.byref(desc), buf.ctypes.data_as(C.c_void_p), len(data)))

    def upload_keymaps(self, table: Table, plan: CPlan, segments, seg_keys):
        spaces = list(plan.key_spaces)
        for ag in plan.aggs:
            if ag.function == "DISTINCTCOUNT":
                spaces.append(table.value_space(ag.arg.cols[0]))
        for p in plan.leaf_preds:  # filters on raw STRING / BYTES columns scan their derived encoding (col | DERIVED)
            if any(s.columns[p.column].dictionary is None and s.columns[p.column].data_type in ("STRING", "BYTES")
                   for s in segments):
                spaces.append(table.key_space(p.column))
        for ks in spaces:
            if ks.kind != abi.PG_KEY_KEYMAP:
                continue
            cid = table.column_ids[ks.column]
            if ks.derived is not None:
                cid |= abi.PG_COL_DERIVED
            for seg, key in zip(segments, seg_keys):
                if ks.derived is not None and (key, cid) not in self._keymaps_uploaded:
                    self._upload_derived(key, cid, seg.columns[ks.column], ks.derived[table.segments.index(seg)])
                if (key, cid) in self._keymaps_uploaded:
                    continue
                km = np.ascontiguousarray(ks.keymaps[table.segments.index(seg)], dtype=np.int32)
                d = abi.pg_col_desc()
                d.kind = abi.PG_IDX_KEYMAP
                d.cardinality = len(km)
                check(self.lib.pg_column_upload(key, cid, C.byref(d), km.ctypes.data_as(C.c_void_p), km.nbytes))
                self._keymaps_uploaded.add((key, cid))

    def _upload_derived(self, key, cid, col, derived):
        """The resident form of a derived key column (KeySpace.derived, col_id | PG_COL_DERIVED): a raw segment's
        host-built encoding as a LONG dictionary of order keys + a bit-packed SV forward index; a dictionary segment
        of the same table keeps its own dictionary and forward index (the keymap maps either to the global ids)."""
        if derived is not None:
            u, ids = derived
            b = num_bits_per_value(max(len(u) - 1, 0))
            col = Column(col.name, "LONG", True, Dictionary("LONG", u), len(ids), b, False, len(ids), 0,
                         fwd=pack_bits(ids, b), dict_ids=ids)
        d = fwd_desc(col)
        dd = abi.pg_col_desc.from_buffer_copy(d)
        dd.kind = abi.PG_IDX_DICT
        self._upload(key, cid, dd, col.dictionary.to_bytes())
        self._upload(key, cid, d, col.fwd)

    def dict_id_sets(self, col_id: int, data_type: str, literals: np.ndarray, seg_keys):
        """pg_dict_id_sets: the literals' dictIds in every segment's resident dictionary (one device launch)."""
        keys = np.ascontiguousarray(seg_keys, dtype=np.uint64)
        literals = np.ascontiguousarray(literals, dtype={"INT": np.int32, "LONG": np.int64, "FLOAT": np.float32,
                                                         "DOUBLE": np.float64}[data_type])
        S, n = len(keys), len(literals)
        ids = np.empty((S, max(n, 1)), dtype=np.int32)
        counts = np.empty(max(S, 1), dtype=np.uint32)
        check(self.lib.pg_dict_id_sets(keys.ctypes.data_as(C.POINTER(C.c_uint64)), S, col_id,
                                       abi.DTYPE_CODES[data_type], literals.ctypes.data_as(C.c_void_p), n,
                                       ids.ctypes.data_as(C.POINTER(C.c_int32)),
                                       counts.ctypes.data_as(C.POINTER(C.c_uint32))))
        return ids, counts

    def segment_device(self, seg: ImmutableSegment) -> int:
        """The logical device a resident segment lives on (pg_segment_device)."""
        out = C.c_uint32()
        check(self.lib.pg_segment_device(self._seg_keys[id(seg)][1], C.byref(out)))
        return out.value

    def release(self, seg: ImmutableSegment):
        hit = self._seg_keys.pop(id(seg), None)
        if hit is not None:
            check(self.lib.pg_segment_release(hit[1]))
            self._keymaps_uploaded = {k for k in self._keymaps_uploaded if k[0] != hit[1]}
            with self._plan_lock:  # plans over the released segment can never be hit again (keys are not reused)
                for ck in [ck for ck in self._plans if hit[1] in ck[3]]:
                    del self._plans[ck]

    # ---- execution
    def make_plan(self, table: Table, query: QueryContext, segments: Optional[Sequence[ImmutableSegment]] = None,
                  flags: int = abi.PG_PLAN_VALUE_SETS, trim=False, config: Optional[InstanceConfig] = None) -> CPlan:
        """flags: PG_PLAN_* (default: DISTINCTCOUNT value sets, the reference's Set intermediate).  trim: see CPlan
        (True: the query's ORDER BY / LIMIT with boundary ties, a final single-server answer; "server": the rows the
        reference server's combine keeps under `config` and the query options).  config: the server instance's
        settings (numGroupsLimit comes only from there, as in the reference)."""
        segments = list(table.segments if segments is None else segments)
        keys = [self.upload_segment(s, table) for s in segments]
        plan = CPlan(table, query, segments, keys, flags, trim, id_sets=self.dict_id_sets, config=config,
                     derived_ids=True)
        self.upload_keymaps(table, plan, segments, keys)
        return plan

    PLAN_CACHE_SIZE = 64

    def cached_plan(self, table: Table, sql: str, segments: Optional[Sequence[ImmutableSegment]] = None,
                    flags: int = abi.PG_PLAN_VALUE_SETS, trim=False, config: Optional[InstanceConfig] = None) -> CPlan:
        """make_plan through a compiled-plan cache (LRU, PLAN_CACHE_SIZE plans).  The reference plans every query from
        scratch (InstancePlanMakerImplV2.makeInstancePlan, ~microseconds of Java per segment); here a server answering
        the same query text again over the same resident segments reuses the lowered plan, and a query of the same
        SHAPE with other filter literals (query_shape: a parametrised query) reuses everything but the leaves, which
        CPlan.relower lowers for the new literals.  The key pins everything the plan depends on: the SQL text or the
        shape, the table object, the segments' residency keys (a released and re-uploaded segment gets a new key; keys
        are never reused), flags, trim and the instance config.  A plan is immutable once built (execution reads its
        image; each thread's copy of the image carries its own per-call scalars, CPlan.image), so reuse is exact."""
        segs = list(table.segments if segments is None else segments)
        keys = tuple(self.upload_segment(s, table) for s in segs)
        rest = (id(table), keys, flags, trim, None if config is None else dataclasses.astuple(config))
        ck = ("sql", sql) + rest
        with self._plan_lock:
            hit = self._plans.get(ck)
            if hit is not None and hit[0] is table:
                self._plans.move_to_end(ck)
                self.plan_cache_hits += 1
                return hit[1]
        q = parse(sql)
        sk = ("shape", query_shape(q)) + rest
        with self._plan_lock:
            shaped = self._plans.get(sk)
            if shaped is not None and shaped[0] is not table:
                shaped = None
        if shaped is not None:
            plan = shaped[1].relower(q, self.dict_id_sets)
            self.upload_keymaps(table, plan, segs, list(keys))
            with self._plan_lock:
                self.plan_shape_hits += 1
        else:
            plan = self.make_plan(table, q, segs, flags, trim, config)
            with self._plan_lock:
                self.plan_cache_misses += 1
                self._plans[sk] = (table, plan)
        with self._plan_lock:
            self._plans[ck] = (table, plan)
            while len(self._plans) > self.PLAN_CACHE_SIZE:
                self._plans.popitem(last=False)
        return plan

    def run_plan(self, plan: CPlan, image: bool = True) -> IntermediateResult:
        """pg_execute_image over the plan's relocatable image (the JNI form); image=False: pg_execute over the
        pointer-form pg_plan (the in-process form)."""
        res = C.POINTER(abi.pg_result)()
        if image:
            im, addr = plan.image()
            check(self.lib.pg_execute_image(addr, im.size, C.byref(res)))
        else:
            check(self.lib.pg_execute(C.byref(plan.plan), C.byref(res)))
        try:
            return self.decode(plan, res.contents)
        finally:
            self.lib.pg_result_free(res)

    def run_partial(self, plan: CPlan, image: bool = True):
        """pg_execute_partial(_image): this device's partial state (for the cross-GPU merge, pinot_amd.combine)."""
        p = C.POINTER(abi.pg_partials)()
        if image:
            im, addr = plan.image()
            check(self.lib.pg_execute_partial_image(addr, im.size, C.byref(p)))
        else:
            check(self.lib.pg_execute_partial(C.byref(plan.plan), C.byref(p)))
        return p

    def _finalize(self, plan: CPlan, p, res):
        im, addr = plan.image()
        check(self.lib.pg_partials_finalize_image(p, addr, im.size, C.byref(res)))

    def finalize_partial(self, plan: CPlan, p, free: bool = True) -> IntermediateResult:
        res = C.POINTER(abi.pg_result)()
        try:
            self._finalize(plan, p, res)
        finally:
            if free:
                self.lib.pg_partials_free(p)
        try:
            return self.decode(plan, res.contents)
        finally:
            self.lib.pg_result_free(res)

    def export_rows(self, p, num_parts: int, dst_ptr=None, dst_rows: int = 0, stream=None):
        """pg_partials_export: rows of the groups bucketed by owner part; returns the per-part row counts."""
        counts = (C.c_uint64 * num_parts)()
        check(self.lib.pg_partials_export(p, num_parts, dst_ptr, dst_rows, counts, stream))
        return list(counts)

    def create_like(self, p, capacity: int):
        out = C.POINTER(abi.pg_partials)()
        check(self.lib.pg_partials_create(p, capacity, C.byref(out)))
        return out

    def merge_rows(self, p, rows_ptr, n: int, stream=None):
        check(self.lib.pg_partials_merge(p, rows_ptr, n, stream))

    def execute(self, table: Table, query, segments=None, flags: int = abi.PG_PLAN_VALUE_SETS, trim=False,
                config: Optional[InstanceConfig] = None) -> IntermediateResult:
        sql = query if isinstance(query, str) else None
        if sql is not None:
            query = parse(query)
        if has_filtered_aggregations(query):  # FilteredAggregationOperator: one device plan per filter
            if query.group_by:  # the passes are aggregation-only (FilteredAggregationOperator); no group trim applies
                raise UnsupportedQuery("filtered aggregations with GROUP BY")
            return execute_filtered(lambda q: self.execute(table, q, segments, flags, config=config), query)
        if trim == "server" and query.group_by and group_trim(query, config).segment_size is not None:
            return self._execute_segment_trimmed(table, query, segments, flags, config)
        if sql is not None:  # SQL text: through the compiled-plan cache
            return self.run_plan(self.cached_plan(table, sql, segments, flags, trim, config))
        return self.run_plan(self.make_plan(table, query, segments, flags, trim, config))

    def _execute_segment_trimmed(self, table, query, segments, flags, config) -> IntermediateResult:
        """minSegmentGroupTrimSize > 0 with an ORDER BY: every segment's group-by result is trimmed to
        getTableCapacity(limit, minSegmentGroupTrimSize) under the ORDER BY before the combine
        (AggregationGroupByOrderByOperator.java:118-132, TableResizer.trimInSegmentResults), so each segment runs as its
        own device plan with an exact limit, the value-keyed rows merge as IndexedTable.upsert merges them, and the
        server keeps getTableCapacity(limit, minServerGroupTrimSize) rows (IndexedTable.finish)."""
        gt = group_trim(query, config)
        merged: dict = {}
        stats = ExecutionStats()
        aggs = None
        limit_reached = False
        for seg in (table.segments if segments is None else segments):
            r = self.run_plan(self.make_plan(table, query, [seg], flags, gt.segment_size, config))
            aggs = r.aggregations
            limit_reached |= r.groups_limit_reached
            for k, v in r.rows.items():
                merged[k] = merge_intermediate(aggs, merged[k], v) if k in merged else v
            for f in stats.__dataclass_fields__:
                setattr(stats, f, getattr(stats, f) + getattr(r.stats, f))
        n_merged = len(merged)
        if gt.server_size is not None:
            merged = top_groups(query, aggs, merged, gt.server_size)
        return IntermediateResult(aggs or query.aggregations, list(query.group_by), merged, stats, limit_reached,
                                  bool(gt.ordered and gt.server_size is not None and gt.threshold < MAX_TRIM_THRESHOLD
                                       and n_merged >= gt.threshold), n_merged)

    def last_trace(self) -> dict:
        """pg_last_trace: what the device did for this thread's last call -- the kernels that ran, the form each filter
        leaf took in how many segments, re-runs after a speculative overflow, docs matched (the trace scope the
        reference records per operator, BaseOperator.java:38, BitmapBasedFilterOperator.java:102-107)."""
        t = abi.pg_trace()
        check(self.lib.pg_last_trace(C.byref(t)))
        forms = []
        for li in range(min(t.num_leaves, abi.PG_TRACE_MAX_LEAVES)):
            forms.append({abi.LEAF_FORMS[f]: int(n) for f, n in enumerate(t.leaf_forms[li]) if n})
        return {"query_id": t.query_id, "path": [n for b, n in abi.PATH_NAMES.items() if t.path & b],
                "group_mode": ["none", "dense", "hash", "hash_per_segment", "partitioned"][t.group_mode]
                if t.group_mode < 5 else t.group_mode,
                "reruns": t.reruns, "rerun_reasons": t.rerun_reasons,
                "stream_leaf": None if t.stream_leaf == 0xFFFFFFFF else t.stream_leaf, "leaf_forms": forms,
                "num_segments": t.num_segments, "num_segments_nonscan": t.num_segments_nonscan,
                "num_docs_matched": t.num_docs_matched, "num_slots": t.num_slots, "device_ms": t.device_ms,
                "wall_ms": t.wall_ms}

    def last_timing(self) -> abi.pg_timing:
        t = abi.pg_timing()
        check(self.lib.pg_last_timing(C.byref(t)))
        return t

    def finalize_arrays(self, plan: CPlan, p) -> dict:
        """pg_partials_finalize -> the result as plain arrays (result_arrays); frees `p`."""
        res = C.POINTER(abi.pg_result)()
        try:
            self._finalize(plan, p, res)
        finally:
            self.lib.pg_partials_free(p)
        try:
            return self.result_arrays(res.contents)
        finally:
            self.lib.pg_result_free(res)

    @staticmethod
    def result_arrays(r: abi.pg_result) -> dict:
        """Copies of a pg_result's arrays: stats (int64[6]), keys uint32[G, K], values float64[G, A], counts
        int64[G, A] and, with value sets, distinct offsets uint64[G * A + 1] / ids uint32[num_distinct]."""
        A, K, G = r.num_aggs, r.num_keys, r.num_groups

        def copy(ptr, n, dt, size, shape):  # one bytes copy out of the library's buffer, viewed read-only (the
            return np.frombuffer(C.string_at(ptr, n * size), dtype=dt).reshape(shape)  # cheapest ctypes path)
        vals = copy(r.values, G * A, np.float64, 8, (G, A)) if G and A else np.zeros((G, A))
        cnts = copy(r.counts, G * A, np.int64, 8, (G, A)) if G and A else np.zeros((G, A), dtype=np.int64)
        keys = copy(r.keys, G * K, np.uint32, 4, (G, K)) if G and K else np.zeros((G, K), dtype=np.uint32)
        offs = ids = None
        if r.distinct_offsets:
            offs = copy(r.distinct_offsets, G * A + 1, np.uint64, 8, (G * A + 1,))
            nd = int(r.num_distinct)
            ids = copy(r.distinct_ids, nd, np.uint32, 4, (nd,)) if nd else np.zeros(0, dtype=np.uint32)
        s = r.stats
        stats = np.array([s.num_docs_scanned, s.num_entries_scanned_in_filter, s.num_entries_scanned_post_filter,
                          s.num_total_docs, s.num_segments_processed, s.num_segments_matched], dtype=np.int64)
        return {"G": G, "K": K, "A": A, "keys": keys, "values": vals, "counts": cnts, "offsets": offs, "ids": ids,
                "stats": stats, "flags": int(r.flags), "merged": int(r.num_groups_merged)}

    @staticmethod
    def decode(plan: CPlan, r) -> IntermediateResult:
        """pg_result (or its result_arrays) -> value-keyed IntermediateResult.  The arrays are copied out of the
        library's result here; the value-keyed rows (Python objects, the form the tests and the DataTable writer read)
        are built on first access to `.rows` (DeviceResult)."""
        ra = r if isinstance(r, dict) else GpuEngine.result_arrays(r)
        st = ExecutionStats(*ra["stats"].tolist())
        out = DeviceResult(plan.aggs, list(plan.query.group_by), lambda: GpuEngine._rows(plan, ra), st, ra)
        fl = ra.get("flags", 0)
        out.groups_limit_reached = bool(fl & abi.PG_RESULT_GROUPS_LIMIT_REACHED)
        out.trim_threshold_reached = bool(fl & abi.PG_RESULT_TRIM_THRESHOLD_REACHED)
        out.num_groups_merged = ra.get("merged")
        return out

    @staticmethod
    def _rows(plan: CPlan, ra: dict) -> dict:
        A, K, G = ra["A"], ra["K"], ra["G"]
        vals, cnts, keys = ra["values"], ra["counts"], ra["keys"]
        sets = None
        if ra["offsets"] is not None:
            sets = (ra["offsets"], ra["ids"].astype(np.int64))
        kinds = [0 if ag.function in ("COUNT", "COUNTMV") else 3 if ag.function == "DISTINCTCOUNT" else
                 1 if ag.function == "AVG" else 2 for ag in plan.aggs]
        dspaces = [plan.table.value_space(ag.arg.cols[0]) if k == 3 else None for ag, k in zip(plan.aggs, kinds)]
        # column-wise conversion (one numpy -> list conversion per key / aggregation column instead of a Python call
        # per element): 90 groups x 2 aggregations decode in ~40 us instead of ~200 us
        kcols = []
        for k in range(K):
            ks = plan.key_spaces[k]
            col = keys[:, k]
            if ks.kind == abi.PG_KEY_VALUE_OFFSET:
                kcols.append((col.astype(np.int64) + ks.base).tolist())
            else:
                vl = ks.values
                kcols.append([vl[i] for i in col.tolist()])
        keyt = list(zip(*kcols)) if K else [()] * G
        acols = []
        for a, kind in enumerate(kinds):
            v = vals[:, a]
            if kind == 0 or (kind == 3 and sets is None):  # counts; DISTINCTCOUNT size only (no PG_PLAN_VALUE_SETS)
                acols.append(np.rint(v).astype(np.int64).tolist())
            elif kind == 1:
                acols.append(list(zip(v.astype(np.float64).tolist(), cnts[:, a].astype(np.int64).tolist())))
            elif kind == 3:
                offs, ids = sets
                ds = dspaces[a]
                acols.append([ds.values_of(ids[offs[g * A + a]:offs[g * A + a + 1]]) for g in range(G)])
            else:
                acols.append(v.astype(np.float64).tolist())
        return dict(zip(keyt, map(list, zip(*acols)))) if A else {k: [] for k in keyt}


class DeviceResult(IntermediateResult):
    """An IntermediateResult whose value-keyed rows are materialised from the device result's arrays (`arrays`:
    GpuEngine.result_arrays) on first access."""

    def __init__(self, aggregations, group_by, make_rows, stats, arrays):
        self._make = make_rows
        self._rows = None
        self.arrays = arrays
        super().__init__(aggregations, group_by, None, stats)

    @property
    def rows(self):
        if self._make is not None:
            self._rows, self._make = self._make(), None
        return self._rows

    @rows.setter
    def rows(self, v):
        if v is not None:
            self._rows, self._make = v, None
