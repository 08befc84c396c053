"""ctypes mirror of include/pinot_gpu.h (the C ABI).  Shared by the GPU binding and the oracle."""
import ctypes as C

PG_ABI_VERSION = 9

PG_OK, PG_E_INVALID, PG_E_HIP, PG_E_NOMEM, PG_E_NOTFOUND, PG_E_UNSUPPORTED, PG_E_CANCELLED, PG_E_TIMEOUT, \
    PG_E_STATE = 0, -1, -2, -3, -4, -5, -6, -7, -8
STATUS_NAMES = {0: "PG_OK", -1: "PG_E_INVALID", -2: "PG_E_HIP", -3: "PG_E_NOMEM", -4: "PG_E_NOTFOUND",
                -5: "PG_E_UNSUPPORTED", -6: "PG_E_CANCELLED", -7: "PG_E_TIMEOUT", -8: "PG_E_STATE"}

PG_IDX_DICT, PG_IDX_FWD_SV_BITPACKED, PG_IDX_FWD_SV_SORTED, PG_IDX_FWD_MV_BITPACKED, PG_IDX_INV_BITMAP, \
    PG_IDX_KEYMAP, PG_IDX_FWD_SV_RAW, PG_IDX_RANGE = 1, 2, 3, 4, 5, 6, 7, 8
PG_INT, PG_LONG, PG_FLOAT, PG_DOUBLE, PG_STRING, PG_BYTES = 0, 1, 2, 3, 4, 5
DTYPE_CODES = {"INT": PG_INT, "LONG": PG_LONG, "FLOAT": PG_FLOAT, "DOUBLE": PG_DOUBLE, "STRING": PG_STRING,
               "BYTES": PG_BYTES}
PG_SRC_DEVICE = 1
PG_COL_DERIVED = 0x40000000

PG_LEAF_MATCH_ALL, PG_LEAF_EMPTY, PG_LEAF_SV_SCAN, PG_LEAF_SORTED, PG_LEAF_INVERTED, PG_LEAF_MV_SCAN, \
    PG_LEAF_RAW_SCAN, PG_LEAF_RANGE_INDEX = range(8)
PG_OP_NOT = -1


def PG_OP_AND(n):
    return -(0x100 | n)


def PG_OP_OR(n):
    return -(0x200 | n)


PG_AGG_COUNT, PG_AGG_SUM, PG_AGG_MIN, PG_AGG_MAX, PG_AGG_AVG, PG_AGG_DISTINCTCOUNT, PG_AGG_COUNTMV = range(7)
AGG_CODES = {"COUNT": PG_AGG_COUNT, "SUM": PG_AGG_SUM, "MIN": PG_AGG_MIN, "MAX": PG_AGG_MAX, "AVG": PG_AGG_AVG,
             "DISTINCTCOUNT": PG_AGG_DISTINCTCOUNT, "COUNTMV": PG_AGG_COUNTMV}
PG_EXPR_COL, PG_EXPR_MUL, PG_EXPR_ADD, PG_EXPR_SUB = range(4)
PG_KEY_VALUE_OFFSET, PG_KEY_KEYMAP = 0, 1
PG_ORDER_AGG, PG_ORDER_KEY = 0, 1
PG_PLAN_VALUE_SETS, PG_PLAN_HASH_GROUPS, PG_PLAN_F64_SUMS, PG_PLAN_NO_STREAM = 0x1, 0x2, 0x4, 0x8
PG_PLAN_EXACT_LIMIT = 0x10
PG_STATE_DENSE, PG_STATE_HASH, PG_STATE_TUPLES = 0, 1, 2
PG_RESULT_GROUPS_LIMIT_REACHED, PG_RESULT_TRIM_THRESHOLD_REACHED = 0x1, 0x2
PG_SUM_NONFINITE, PG_SUM_BOUNDS = 0x1, 0x2
PG_AGG_MV_VALUES = 0x1
PG_EMPTY_KEY = 0xFFFFFFFFFFFFFFFF


class pg_col_desc(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("data_type", C.c_uint32), ("num_docs", C.c_uint32),
                ("cardinality", C.c_uint32), ("bits_per_element", C.c_uint32), ("num_values", C.c_uint32),
                ("entry_bytes", C.c_uint32), ("flags", C.c_uint32)]


class pg_leaf(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("col_id", C.c_uint32), ("exclusive", C.c_uint32), ("num_ids", C.c_uint32),
                ("lo", C.c_int32), ("hi", C.c_int32), ("ids", C.POINTER(C.c_int32)),
                ("ilo", C.c_int64), ("ihi", C.c_int64), ("dlo", C.c_double), ("dhi", C.c_double),
                ("lo_inclusive", C.c_uint32), ("hi_inclusive", C.c_uint32), ("values", C.c_void_p),
                ("num_values", C.c_uint32), ("pad", C.c_uint32)]


class pg_agg(C.Structure):
    _fields_ = [("fn", C.c_uint32), ("op", C.c_uint32), ("col_a", C.c_uint32), ("col_b", C.c_uint32),
                ("key_kind", C.c_uint32), ("key_cardinality", C.c_uint32), ("key_base", C.c_int64),
                ("sum_exp", C.c_int32), ("sum_flags", C.c_uint32), ("sum_exp_lo", C.c_int32), ("flags", C.c_uint32)]


class pg_key(C.Structure):
    _fields_ = [("col_id", C.c_uint32), ("kind", C.c_uint32), ("cardinality", C.c_uint32), ("pad", C.c_uint32),
                ("base", C.c_int64)]


class pg_segment_ref(C.Structure):
    _fields_ = [("seg_key", C.c_uint64), ("num_docs", C.c_uint32), ("pad", C.c_uint32),
                ("leaves", C.POINTER(pg_leaf))]


class pg_order(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("index", C.c_uint32), ("desc", C.c_uint32), ("pad", C.c_uint32)]


class pg_plan(C.Structure):
    _fields_ = [("abi_version", C.c_uint32), ("num_segments", C.c_uint32), ("segments", C.POINTER(pg_segment_ref)),
                ("num_leaves", C.c_uint32), ("num_ops", C.c_uint32), ("ops", C.POINTER(C.c_int32)),
                ("num_aggs", C.c_uint32), ("num_keys", C.c_uint32), ("aggs", C.POINTER(pg_agg)),
                ("keys", C.POINTER(pg_key)), ("num_groups_limit", C.c_uint64), ("query_id", C.c_uint64),
                ("deadline_ms", C.c_int64), ("stream", C.c_void_p), ("flags", C.c_uint32),
                ("num_order", C.c_uint32), ("order", C.POINTER(pg_order)), ("limit", C.c_uint64),
                ("trim_threshold", C.c_uint64)]


PG_IMAGE_MAGIC = 0x49504750


class pg_image_header(C.Structure):
    _fields_ = [("magic", C.c_uint32), ("abi_version", C.c_uint32), ("image_bytes", C.c_uint64),
                ("num_segments", C.c_uint32), ("num_leaves", C.c_uint32), ("num_ops", C.c_uint32),
                ("num_aggs", C.c_uint32), ("num_keys", C.c_uint32), ("num_order", C.c_uint32), ("flags", C.c_uint32),
                ("trim_threshold", C.c_uint32), ("num_groups_limit", C.c_uint64), ("query_id", C.c_uint64),
                ("deadline_ms", C.c_int64), ("limit", C.c_uint64), ("segments_off", C.c_uint64),
                ("ops_off", C.c_uint64), ("aggs_off", C.c_uint64), ("keys_off", C.c_uint64), ("order_off", C.c_uint64)]


class pg_image_segment(C.Structure):
    _fields_ = [("seg_key", C.c_uint64), ("num_docs", C.c_uint32), ("pad", C.c_uint32), ("leaves_off", C.c_uint64)]


class pg_image_leaf(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("col_id", C.c_uint32), ("exclusive", C.c_uint32), ("num_ids", C.c_uint32),
                ("lo", C.c_int32), ("hi", C.c_int32), ("ids_off", C.c_uint64),
                ("ilo", C.c_int64), ("ihi", C.c_int64), ("dlo", C.c_double), ("dhi", C.c_double),
                ("lo_inclusive", C.c_uint32), ("hi_inclusive", C.c_uint32), ("values_off", C.c_uint64),
                ("num_values", C.c_uint32), ("pad", C.c_uint32)]


class pg_stats(C.Structure):
    _fields_ = [("num_docs_scanned", C.c_uint64), ("num_entries_scanned_in_filter", C.c_uint64),
                ("num_entries_scanned_post_filter", C.c_uint64), ("num_total_docs", C.c_uint64),
                ("num_segments_processed", C.c_uint64), ("num_segments_matched", C.c_uint64)]


class pg_result(C.Structure):
    _fields_ = [("stats", pg_stats), ("num_groups", C.c_uint64), ("num_keys", C.c_uint32), ("num_aggs", C.c_uint32),
                ("keys", C.POINTER(C.c_uint32)), ("values", C.POINTER(C.c_double)),
                ("counts", C.POINTER(C.c_int64)), ("num_distinct", C.c_uint64),
                ("distinct_offsets", C.POINTER(C.c_uint64)), ("distinct_ids", C.POINTER(C.c_uint32)),
                ("num_groups_merged", C.c_uint64), ("flags", C.c_uint32), ("pad", C.c_uint32)]


class pg_partials(C.Structure):
    _fields_ = [("stats", pg_stats), ("num_slots", C.c_uint64), ("mode", C.c_uint32), ("n_i64", C.c_uint32),
                ("n_fx", C.c_uint32), ("n_min", C.c_uint32), ("n_max", C.c_uint32), ("bitmap_words", C.c_uint32),
                ("layout", C.c_uint32), ("fx_sig", C.c_uint32), ("row_bytes", C.c_uint64), ("keys", C.c_void_p),
                ("i64", C.c_void_p), ("fx", C.c_void_p), ("mn", C.c_void_p), ("mx", C.c_void_p),
                ("bitmaps", C.c_void_p), ("impl", C.c_void_p), ("flags", C.c_uint32), ("pad", C.c_uint32)]


class pg_timing(C.Structure):
    _fields_ = [("prepass_ms", C.c_float), ("scan_ms", C.c_float), ("finalize_ms", C.c_float),
                ("scan_launches", C.c_uint32), ("host_compile_ms", C.c_float), ("execute_wall_ms", C.c_float),
                ("finalize_wall_ms", C.c_float), ("prefilter_ms", C.c_float)]


# pinot_trace.h
PG_TRACE_MAX_LEAVES = 16
LEAF_FORMS = ["MATCH_ALL", "EMPTY", "SCAN_RANGE", "SCAN_SET_LDS", "SCAN_SET_LUT", "SORTED_RANGE", "SORTED_BITMAP",
              "INVERTED", "MV_SCAN", "RAW_SCAN", "RANGE_INDEX"]
PG_PATH_FUSED_SCAN, PG_PATH_STREAM, PG_PATH_PARTITIONED, PG_PATH_WIDE_KEYS, PG_PATH_NONSCAN, PG_PATH_PREPASS = \
    0x1, 0x2, 0x4, 0x8, 0x10, 0x20
PG_PATH_INDEX_COUNT = 0x40
PATH_NAMES = {PG_PATH_FUSED_SCAN: "fused_scan", PG_PATH_STREAM: "stream", PG_PATH_PARTITIONED: "partitioned",
              PG_PATH_WIDE_KEYS: "wide_keys", PG_PATH_NONSCAN: "nonscan", PG_PATH_PREPASS: "prepass",
              PG_PATH_INDEX_COUNT: "index_count"}
PG_RERUN_STREAM, PG_RERUN_PARTITION, PG_RERUN_HASH = 0x1, 0x2, 0x4


class pg_trace(C.Structure):
    _fields_ = [("query_id", C.c_uint64), ("path", C.c_uint32), ("group_mode", C.c_uint32), ("reruns", C.c_uint32),
                ("rerun_reasons", C.c_uint32), ("num_leaves", C.c_uint32), ("stream_leaf", C.c_uint32),
                ("leaf_forms", (C.c_uint32 * len(LEAF_FORMS)) * PG_TRACE_MAX_LEAVES), ("pad", C.c_uint32),
                ("num_segments", C.c_uint64), ("num_segments_nonscan", C.c_uint64),
                ("num_docs_matched", C.c_uint64), ("num_slots", C.c_uint64), ("device_ms", C.c_float),
                ("wall_ms", C.c_float)]


# every symbol declared in include/*.h (checked by tests/test_abi.py)
EXPORTED = ["pg_init", "pg_last_error", "pg_resident_bytes", "pg_cancel", "pg_abi_version", "pg_column_upload",
            "pg_segment_release", "pg_execute", "pg_result_free", "pg_execute_partial", "pg_partials_finalize",
            "pg_partials_free", "pg_partials_copy", "pg_partials_export", "pg_partials_create", "pg_partials_merge",
            "pg_key_owner", "pg_last_timing", "pg_chunk_decompress", "pg_dict_id_sets", "pg_execute_image",
            "pg_execute_partial_image", "pg_partials_finalize_image", "pg_last_trace", "pg_init_devices",
            "pg_num_devices", "pg_segment_place", "pg_segment_device"]
PG_CODEC_PASS_THROUGH, PG_CODEC_SNAPPY, PG_CODEC_ZSTANDARD, PG_CODEC_LZ4, PG_CODEC_LZ4_LENGTH_PREFIXED = 0, 1, 2, 3, 4
PG_COPY_OUT, PG_COPY_IN = 0, 1


def declare(lib):
    """Attach argtypes / restypes to a loaded libpinot_gpu."""
    P = C.POINTER
    sigs = {
        "pg_init": ([C.c_int], C.c_int),
        "pg_init_devices": ([P(C.c_int), C.c_uint32], C.c_int),
        "pg_num_devices": ([P(C.c_uint32)], C.c_int),
        "pg_segment_place": ([C.c_uint64, C.c_uint32], C.c_int),
        "pg_segment_device": ([C.c_uint64, P(C.c_uint32)], C.c_int),
        "pg_last_error": ([C.c_char_p, C.c_size_t], C.c_int),
        "pg_resident_bytes": ([P(C.c_uint64)], C.c_int),
        "pg_cancel": ([C.c_uint64], C.c_int),
        "pg_abi_version": ([], C.c_int),
        "pg_column_upload": ([C.c_uint64, C.c_uint32, P(pg_col_desc), C.c_void_p, C.c_uint64], C.c_int),
        "pg_dict_id_sets": ([P(C.c_uint64), C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p, C.c_uint32, P(C.c_int32),
                             P(C.c_uint32)], C.c_int),
        "pg_segment_release": ([C.c_uint64], C.c_int),
        "pg_execute": ([P(pg_plan), P(P(pg_result))], C.c_int),
        "pg_result_free": ([P(pg_result)], C.c_int),
        "pg_execute_partial": ([P(pg_plan), P(P(pg_partials))], C.c_int),
        "pg_partials_finalize": ([P(pg_partials), P(pg_plan), P(P(pg_result))], C.c_int),
        "pg_partials_free": ([P(pg_partials)], C.c_int),
        "pg_last_timing": ([P(pg_timing)], C.c_int),
        "pg_partials_copy": ([P(pg_partials), C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p],
                             C.c_int),
        "pg_partials_export": ([P(pg_partials), C.c_uint32, C.c_void_p, C.c_uint64, P(C.c_uint64), C.c_void_p],
                               C.c_int),
        "pg_partials_create": ([P(pg_partials), C.c_uint64, P(P(pg_partials))], C.c_int),
        "pg_partials_merge": ([P(pg_partials), C.c_void_p, C.c_uint64, C.c_void_p], C.c_int),
        "pg_key_owner": ([C.c_uint64, C.c_uint32], C.c_uint32),
        "pg_chunk_decompress": ([C.c_uint32, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, P(C.c_uint64)], C.c_int),
        "pg_execute_image": ([C.c_void_p, C.c_uint64, P(P(pg_result))], C.c_int),
        "pg_last_trace": ([P(pg_trace)], C.c_int),
        "pg_execute_partial_image": ([C.c_void_p, C.c_uint64, P(P(pg_partials))], C.c_int),
        "pg_partials_finalize_image": ([P(pg_partials), C.c_void_p, C.c_uint64, P(P(pg_result))], C.c_int),
    }
    for name, (args, res) in sigs.items():
        f = getattr(lib, name)
        f.argtypes = args
        f.restype = res
    return lib


def build_image(plan: pg_plan, leaf_table=None, regions=()) -> "np.ndarray":
    """The relocatable image (include/pinot_gpu.h, pg_image_header) of a pointer-form pg_plan: every array the plan
    points to copied into one 8-byte-aligned buffer at a byte offset; an array several segments share (values-mode IN
    literals) is stored once.  Returns a uint8 view of length image_bytes.

    leaf_table: the plan's leaves as ONE [segment][leaf] array in pg_leaf's layout (CPlan), with `regions` = every
    numpy array its ids / values pointers point into: then the table is copied whole, each region once, and the
    pointers are turned into offsets with a few vectorized operations instead of a loop over the segments."""
    import numpy as np
    if leaf_table is not None and plan.num_segments:
        return _build_image_table(plan, leaf_table, regions)
    buf = bytearray(C.sizeof(pg_image_header))
    placed = {}
    keep = []  # temporaries stay alive while `placed` is keyed by their addresses

    def put(addr, nbytes, align=8):
        if not addr or not nbytes:
            return 0
        hit = placed.get((addr, nbytes))
        if hit is not None:
            return hit
        buf.extend(bytes(-len(buf) % align))
        off = len(buf)
        buf.extend(C.string_at(addr, nbytes))
        placed[(addr, nbytes)] = off
        return off

    def addr_of(ptr):
        return C.cast(ptr, C.c_void_p).value

    h = pg_image_header()
    h.magic, h.abi_version = PG_IMAGE_MAGIC, plan.abi_version
    for f in ("num_segments", "num_leaves", "num_ops", "num_aggs", "num_keys", "num_order", "flags",
              "num_groups_limit", "query_id", "deadline_ms", "limit"):
        setattr(h, f, getattr(plan, f))
    h.trim_threshold = min(plan.trim_threshold, 0xFFFFFFFF)
    h.ops_off = put(addr_of(plan.ops), 4 * plan.num_ops, 4)
    h.aggs_off = put(addr_of(plan.aggs), C.sizeof(pg_agg) * plan.num_aggs)
    h.keys_off = put(addr_of(plan.keys), C.sizeof(pg_key) * plan.num_keys)
    h.order_off = put(addr_of(plan.order), C.sizeof(pg_order) * plan.num_order, 4)
    segs = (pg_image_segment * max(plan.num_segments, 1))()
    L = plan.num_leaves
    for si in range(plan.num_segments):
        sr = plan.segments[si]
        leaves = (pg_image_leaf * max(L, 1))()
        keep.append(leaves)
        for li in range(L):
            x = sr.leaves[li]
            y = leaves[li]
            C.memmove(C.addressof(y), C.addressof(x), C.sizeof(pg_leaf))
            y.ids_off = put(addr_of(x.ids), 4 * x.num_ids, 4) if x.ids else 0
            y.values_off = put(x.values, 8 * (x.num_values or x.num_ids)) if x.values else 0
        segs[si].seg_key, segs[si].num_docs = sr.seg_key, sr.num_docs
        segs[si].leaves_off = put(C.addressof(leaves), C.sizeof(pg_image_leaf) * L) if L else 0
    h.segments_off = put(C.addressof(segs), C.sizeof(pg_image_segment) * plan.num_segments)
    buf.extend(bytes(-len(buf) % 8))
    h.image_bytes = len(buf)
    buf[:C.sizeof(h)] = bytes(h)
    out = np.empty(len(buf) // 8, dtype=np.uint64).view(np.uint8)
    out[:] = np.frombuffer(bytes(buf), dtype=np.uint8)
    return out


def _build_image_table(plan: pg_plan, tab, regions) -> "np.ndarray":
    import numpy as np
    S, L = plan.num_segments, plan.num_leaves
    parts = [bytes(C.sizeof(pg_image_header))]
    size = len(parts[0])

    def put(b: bytes, align=8) -> int:
        nonlocal size
        pad = -size % align
        if pad:
            parts.append(bytes(pad))
            size += pad
        off = size
        parts.append(b)
        size += len(b)
        return off

    def addr_of(ptr):
        return C.cast(ptr, C.c_void_p).value

    h = pg_image_header()
    h.magic, h.abi_version = PG_IMAGE_MAGIC, plan.abi_version
    for f in ("num_segments", "num_leaves", "num_ops", "num_aggs", "num_keys", "num_order", "flags",
              "num_groups_limit", "query_id", "deadline_ms", "limit"):
        setattr(h, f, getattr(plan, f))
    h.trim_threshold = min(plan.trim_threshold, 0xFFFFFFFF)
    h.ops_off = put(C.string_at(addr_of(plan.ops), 4 * plan.num_ops), 4) if plan.num_ops else 0
    h.aggs_off = put(C.string_at(addr_of(plan.aggs), C.sizeof(pg_agg) * plan.num_aggs)) if plan.num_aggs else 0
    h.keys_off = put(C.string_at(addr_of(plan.keys), C.sizeof(pg_key) * plan.num_keys)) if plan.num_keys else 0
    h.order_off = put(C.string_at(addr_of(plan.order), C.sizeof(pg_order) * plan.num_order), 4) if plan.num_order else 0
    # every region the leaves point into, once (8-byte aligned): regions sorted by address, each pointer's region
    # found by a search, only the regions some leaf points into copied, then the pointers rewritten as offsets
    regs = [a for _, a in sorted({int(a.ctypes.data): a for a in regions if a.nbytes}.items())]
    starts = np.array([a.ctypes.data for a in regs], dtype=np.uint64)
    ends = starts + np.array([a.nbytes for a in regs], dtype=np.uint64)
    lt = np.array(tab[:S, :max(L, 1)], copy=True)  # pg_image_leaf has pg_leaf's layout with offsets for pointers
    found = {}
    for f, nb in (("ids", 4), ("values", 8)):
        ptr = lt[f]
        nz = ptr != 0
        if not nz.any():
            continue
        i = np.searchsorted(starts, ptr[nz], side="right").astype(np.int64) - 1
        n = lt["num_ids"][nz].astype(np.uint64)
        if f == "values":
            nv = lt["num_values"][nz].astype(np.uint64)
            n = np.where(nv > 0, nv, n)
        if (i < 0).any() or (ptr[nz] + n * nb > ends[np.maximum(i, 0)]).any():
            raise ValueError(f"leaf {f} pointer outside the plan's arrays")
        found[f] = (nz, i)
    used = np.unique(np.concatenate([x[1] for x in found.values()])) if found else np.zeros(0, np.int64)
    offs = np.zeros(len(regs), dtype=np.uint64)
    for r in used:
        offs[r] = put(np.ascontiguousarray(regs[r]).tobytes())
    for f, (nz, i) in found.items():
        ptr = lt[f]
        ptr[nz] = offs[i] + (ptr[nz] - starts[i])
    leaves_off = put(lt.tobytes()) if L else 0
    segs = (pg_image_segment * S)()
    st = np.frombuffer(segs, dtype=[("seg_key", "<u8"), ("num_docs", "<u4"), ("pad", "<u4"), ("leaves_off", "<u8")])
    src = (pg_segment_ref * S).from_address(addr_of(plan.segments))
    sr = np.frombuffer(src, dtype=[("seg_key", "<u8"), ("num_docs", "<u4"), ("pad", "<u4"), ("leaves", "<u8")])
    st["seg_key"], st["num_docs"] = sr["seg_key"], sr["num_docs"]
    st["leaves_off"] = (leaves_off + np.arange(S, dtype=np.uint64) * (max(L, 1) * C.sizeof(pg_image_leaf))) if L else 0
    h.segments_off = put(bytes(segs))
    pad = -size % 8
    if pad:
        parts.append(bytes(pad))
        size += pad
    h.image_bytes = size
    parts[0] = bytes(h)
    out = np.empty(size // 8, dtype=np.uint64).view(np.uint8)
    out[:] = np.frombuffer(b"".join(parts), dtype=np.uint8)
    return out
