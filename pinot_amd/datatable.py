"""DataTable V3: the bytes a Pinot server returns to the broker for one query, built from the device path's
server-side result, and the broker side that decodes and reduces them.

Restated from the reference's Java, not copied:
  * layout        -- core/common/datatable/DataTableImplV3.java:37-69 (13-int header: version, rows, columns, then
                     (start, length) of the exceptions / dictionary map / data schema / fixed-size / variable-size
                     sections; after them the metadata length + metadata), toBytes :188-297
  * metadata      -- DataTableImplV3.serializeMetadata :311-338: entry count, then per entry the key id and a BE
                     int / BE long / (length, UTF-8) value by the key's type (common/utils/DataTable.java MetadataKey)
  * exceptions    -- :375-392 (count, then error code + (length, UTF-8) message)
  * dictionary map / schema -- BaseDataTable.serializeDictionaryMap :91-114, DataSchema.toBytes :153-178 (column
                     names, then column type NAMES, each (length, UTF-8))
  * rows          -- BaseDataTableBuilder :30-162 + DataTableBuilderV2V3 :49-98: fixed-size rows at the offsets of
                     DataTableUtils.computeColumnOffsets (INT 4, LONG 8, FLOAT 8 before V4, DOUBLE 8, STRING 4 =
                     per-column dictionary id, OBJECT / arrays 8 = (variable-section position, length)); an OBJECT
                     value is its ObjectSerDeUtils type id (BE int) followed by its serialized bytes
  * objects       -- ObjectSerDeUtils.java: Long (1) / Double (2) 8 B BE, AvgPair (4) = BE double sum + BE long
                     count (customobject/AvgPair.java:53-58), IntSet (9) / LongSet (15) / FloatSet (16) / DoubleSet
                     (17) = BE int size + BE values, StringSet (18) = size + (length, UTF-8) per value
  * result tables -- IntermediateResultsBlock.getAggregationResultDataTable :455-538 (one row, columns named
                     AggregationFunction.getColumnName() = "<type>_<expr>", intermediate column types), getResultDataTable
                     :351-399 (group-by: key columns then "<type>(<expr>)" columns, AggregationGroupByOrderByOperator
                     .java:70-94), attachMetadataToDataTable :544-569
  * broker reduce -- decode every server's table, merge intermediates by key (AggregationFunction.merge), final values,
                     ORDER BY / LIMIT (query/reduce/GroupByDataTableReducer.java:86-200, AggregationDataTableReducer)

Parity is unpinned for the bytes: the reference holds no serialized DataTable fixture (its DataTableSerDeTest
builds random tables in Java), so tests/test_datatable.py checks the layout field by field against this restatement,
round trips, and the broker reduce of split results against the whole-table oracle.  Java HashMap iteration orders
(metadata entries, dictionary map, set members) are not part of the contract; they are written here in a fixed order
(sets ascending).
"""
import struct
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

from .plan import ExecutionStats, IntermediateResult, merge_intermediate, reduce_to_rows
from .query import Aggregation, QueryContext

VERSION_3 = 3
HEADER_SIZE = 13 * 4

# MetadataKey (pinot-common/.../utils/DataTable.java): name -> (id, value type)
METADATA_KEYS = {
    "unknown": (0, "STRING"), "table": (1, "STRING"), "numDocsScanned": (2, "LONG"),
    "numEntriesScannedInFilter": (3, "LONG"), "numEntriesScannedPostFilter": (4, "LONG"),
    "numSegmentsQueried": (5, "INT"), "numSegmentsProcessed": (6, "INT"), "numSegmentsMatched": (7, "INT"),
    "numConsumingSegmentsQueried": (8, "INT"), "minConsumingFreshnessTimeMs": (9, "LONG"), "totalDocs": (10, "LONG"),
    "numGroupsLimitReached": (11, "STRING"), "timeUsedMs": (12, "LONG"), "traceInfo": (13, "STRING"),
    "requestId": (14, "LONG"), "numResizes": (15, "INT"), "resizeTimeMs": (16, "LONG"),
    "threadCpuTimeNs": (17, "LONG"), "systemActivitiesCpuTimeNs": (18, "LONG"),
    "responseSerializationCpuTimeNs": (19, "LONG"), "numSegmentsPrunedByServer": (20, "INT"),
    "numSegmentsPrunedByInvalid": (21, "INT"), "numSegmentsPrunedByLimit": (22, "INT"),
    "numSegmentsPrunedByValue": (23, "INT"), "explainPlanNumEmptyFilterSegments": (24, "INT"),
    "explainPlanNumMatchAllFilterSegments": (25, "INT"), "numConsumingSegmentsProcessed": (26, "INT"),
    "numConsumingSegmentsMatched": (27, "INT"),
}
METADATA_BY_ID = {v[0]: (k, v[1]) for k, v in METADATA_KEYS.items()}

# ObjectSerDeUtils.ObjectType ids of the intermediate types the device path produces
OBJ_STRING, OBJ_LONG, OBJ_DOUBLE, OBJ_AVG_PAIR, OBJ_INT_SET = 0, 1, 2, 4, 9
OBJ_LONG_SET, OBJ_FLOAT_SET, OBJ_DOUBLE_SET, OBJ_STRING_SET, OBJ_BYTES_SET, OBJ_NULL = 15, 16, 17, 18, 19, 100
SET_TYPE_OF_COLUMN = {"INT": OBJ_INT_SET, "LONG": OBJ_LONG_SET, "FLOAT": OBJ_FLOAT_SET, "DOUBLE": OBJ_DOUBLE_SET,
                      "STRING": OBJ_STRING_SET, "BYTES": OBJ_BYTES_SET}
_SET_FMT = {OBJ_INT_SET: ">i", OBJ_LONG_SET: ">q", OBJ_FLOAT_SET: ">f", OBJ_DOUBLE_SET: ">d"}

# AggregationFunctionType.getName() (pinot-segment-spi/.../AggregationFunctionType.java)
_TYPE_NAME = {"COUNT": "count", "SUM": "sum", "MIN": "min", "MAX": "max", "AVG": "avg",
              "DISTINCTCOUNT": "distinctCount", "COUNTMV": "countMV"}
# getIntermediateResultColumnType of each function (e.g. SumAggregationFunction.java:282)
_INTERMEDIATE_TYPE = {"COUNT": "LONG", "COUNTMV": "LONG", "SUM": "DOUBLE", "MIN": "DOUBLE", "MAX": "DOUBLE",
                      "AVG": "OBJECT", "DISTINCTCOUNT": "OBJECT"}


def column_name(ag: Aggregation) -> str:
    """AggregationFunction.getColumnName(): "<type>_<expression>" (aggregation-only tables); COUNT(*) is "count_star"
    (CountAggregationFunction.java:37,62: COLUMN_NAME = "count_star")."""
    if ag.function == "COUNT":
        return "count_star"
    return f"{_TYPE_NAME[ag.function]}{'MV' if ag.mv else ''}_{ag.arg}"


def result_column_name(ag: Aggregation) -> str:
    """AggregationFunction.getResultColumnName(): "<type lower-case>(<expression>)" (group-by tables)."""
    return f"{(_TYPE_NAME[ag.function] + ('MV' if ag.mv else '')).lower()}({ag.arg})"


@dataclass
class DataSchema:
    names: List[str]
    types: List[str]   # ColumnDataType names (INT, LONG, FLOAT, DOUBLE, STRING, OBJECT, ...)


@dataclass
class DataTable:
    schema: Optional[DataSchema]
    rows: List[list]   # python values; OBJECT cells as (object type id, value)
    metadata: Dict[str, str] = field(default_factory=dict)
    exceptions: Dict[int, str] = field(default_factory=dict)


# ------------------------------------------------------------------------------------------------ encode

def _s(b: bytearray, text: str):
    raw = text.encode("utf-8")
    b += struct.pack(">i", len(raw))
    b += raw


def _fixed_width(t: str) -> int:
    """DataTableUtils.computeColumnOffsets for V3."""
    return {"INT": 4, "LONG": 8, "FLOAT": 8, "DOUBLE": 8, "STRING": 4, "BYTES": 4}.get(t, 8)


def serialize_object(type_id: int, value) -> bytes:
    if type_id == OBJ_LONG:
        return struct.pack(">q", int(value))
    if type_id == OBJ_DOUBLE:
        return struct.pack(">d", float(value))
    if type_id == OBJ_STRING:
        return str(value).encode("utf-8")
    if type_id == OBJ_AVG_PAIR:
        s, c = value
        return struct.pack(">dq", float(s), int(c))
    if type_id in _SET_FMT:
        vals = sorted(value)
        return struct.pack(">i", len(vals)) + b"".join(struct.pack(_SET_FMT[type_id], v) for v in vals)
    if type_id == OBJ_STRING_SET:
        out = bytearray(struct.pack(">i", len(value)))
        for v in sorted(value):
            _s(out, v)
        return bytes(out)
    if type_id == OBJ_BYTES_SET:  # BYTES_SET_SER_DE (ObjectSerDeUtils.java:774-793): size, then (length, bytes) each
        out = bytearray(struct.pack(">i", len(value)))
        for v in sorted(value):
            raw = bytes.fromhex(v)
            out += struct.pack(">i", len(raw)) + raw
        return bytes(out)
    raise ValueError(f"object type {type_id}")


def deserialize_object(type_id: int, raw: bytes):
    if type_id == OBJ_NULL:
        return None
    if type_id == OBJ_LONG:
        return struct.unpack(">q", raw)[0]
    if type_id == OBJ_DOUBLE:
        return struct.unpack(">d", raw)[0]
    if type_id == OBJ_STRING:
        return raw.decode("utf-8")
    if type_id == OBJ_AVG_PAIR:
        return struct.unpack(">dq", raw)
    if type_id in _SET_FMT:
        n = struct.unpack_from(">i", raw)[0]
        w = struct.calcsize(_SET_FMT[type_id])
        return {struct.unpack_from(_SET_FMT[type_id], raw, 4 + i * w)[0] for i in range(n)}
    if type_id in (OBJ_STRING_SET, OBJ_BYTES_SET):
        n, pos, out = struct.unpack_from(">i", raw)[0], 4, set()
        for _ in range(n):
            ln = struct.unpack_from(">i", raw, pos)[0]
            b = raw[pos + 4:pos + 4 + ln]
            out.add(b.decode("utf-8") if type_id == OBJ_STRING_SET else b.hex())
            pos += 4 + ln
        return out
    raise ValueError(f"object type {type_id}")


def to_bytes(dt: DataTable) -> bytes:
    """DataTableImplV3.toBytes."""
    exc = bytearray(struct.pack(">i", len(dt.exceptions)))
    for code, msg in dt.exceptions.items():
        exc += struct.pack(">i", code)
        _s(exc, msg)
    fixed = bytearray()
    var = bytearray()
    dictionary: Dict[str, Dict[str, int]] = {}
    schema_b = b""
    if dt.schema is not None:
        sb = bytearray(struct.pack(">i", len(dt.schema.names)))
        for n in dt.schema.names:
            _s(sb, n)
        for t in dt.schema.types:
            _s(sb, t)
        schema_b = bytes(sb)
        widths = [_fixed_width(t) for t in dt.schema.types]
        for row in dt.rows:
            for name, t, w, v in zip(dt.schema.names, dt.schema.types, widths, row):
                if t == "INT":
                    cell = struct.pack(">i", int(v))
                elif t == "LONG":
                    cell = struct.pack(">q", int(v))
                elif t == "FLOAT":
                    cell = struct.pack(">f", float(v))
                elif t == "DOUBLE":
                    cell = struct.pack(">d", float(v))
                elif t in ("STRING", "BYTES"):  # BYTES: its hex string (DataTableBuilderV2V3.setColumn(ByteArray) :69-72)
                    d = dictionary.setdefault(name, {})
                    cell = struct.pack(">i", d.setdefault(str(v), len(d)))
                elif t == "OBJECT":
                    type_id, value = v
                    pos = len(var)
                    if type_id == OBJ_NULL:
                        var += struct.pack(">i", OBJ_NULL)
                        cell = struct.pack(">ii", pos, 0)
                    else:
                        raw = serialize_object(type_id, value)
                        var += struct.pack(">i", type_id)
                        var += raw
                        cell = struct.pack(">ii", pos, len(raw))
                else:
                    raise ValueError(f"column type {t}")
                fixed += cell.ljust(w, b"\0")
    dict_b = b""
    if dictionary:
        db = bytearray(struct.pack(">i", len(dictionary)))
        for col, d in dictionary.items():
            _s(db, col)
            db += struct.pack(">i", len(d))
            for value, i in d.items():
                db += struct.pack(">i", i)
                _s(db, value)
        dict_b = bytes(db)
    out = bytearray(struct.pack(">iii", VERSION_3, len(dt.rows), len(dt.schema.names) if dt.schema else 0))
    off = HEADER_SIZE
    for sec in (bytes(exc), dict_b, schema_b, bytes(fixed)):
        out += struct.pack(">ii", off, len(sec))
        off += len(sec)
    out += struct.pack(">ii", off, len(var))
    out += exc + dict_b + schema_b + fixed + var
    meta = bytearray(struct.pack(">i", 0))
    n = 0
    for name, value in dt.metadata.items():
        if name not in METADATA_KEYS:  # unknown keys are not written (serializeMetadata skips them)
            continue
        kid, kt = METADATA_KEYS[name]
        meta += struct.pack(">i", kid)
        if kt == "INT":
            meta += struct.pack(">i", int(value))
        elif kt == "LONG":
            meta += struct.pack(">q", int(value))
        else:
            _s(meta, str(value))
        n += 1
    struct.pack_into(">i", meta, 0, n)
    out += struct.pack(">i", len(meta)) + meta
    return bytes(out)


# ------------------------------------------------------------------------------------------------ decode

def _str_at(b: bytes, pos: int) -> Tuple[str, int]:
    ln = struct.unpack_from(">i", b, pos)[0]
    return b[pos + 4:pos + 4 + ln].decode("utf-8"), pos + 4 + ln


def from_bytes(b: bytes) -> DataTable:
    """DataTableImplV3(ByteBuffer) -- the broker side."""
    version, nrows, ncols = struct.unpack_from(">iii", b, 0)
    if version != VERSION_3:
        raise ValueError(f"DataTable version {version}")
    sec = [struct.unpack_from(">ii", b, 12 + 8 * i) for i in range(5)]
    (es, el), (ds, dl), (ss, sl), (fs, fl), (vs, vl) = sec
    exceptions = {}
    if el:
        n = struct.unpack_from(">i", b, es)[0]
        pos = es + 4
        for _ in range(n):
            code = struct.unpack_from(">i", b, pos)[0]
            msg, pos = _str_at(b, pos + 4)
            exceptions[code] = msg
    rev: Dict[str, Dict[int, str]] = {}
    if dl:
        n = struct.unpack_from(">i", b, ds)[0]
        pos = ds + 4
        for _ in range(n):
            col, pos = _str_at(b, pos)
            m = struct.unpack_from(">i", b, pos)[0]
            pos += 4
            d = {}
            for _ in range(m):
                i = struct.unpack_from(">i", b, pos)[0]
                v, pos = _str_at(b, pos + 4)
                d[i] = v
            rev[col] = d
    schema = None
    rows: List[list] = []
    if sl:
        n = struct.unpack_from(">i", b, ss)[0]
        pos = ss + 4
        names, types = [], []
        for _ in range(n):
            s, pos = _str_at(b, pos)
            names.append(s)
        for _ in range(n):
            s, pos = _str_at(b, pos)
            types.append(s)
        schema = DataSchema(names, types)
        widths = [_fixed_width(t) for t in types]
        row_size = sum(widths)
        var = b[vs:vs + vl]
        for r in range(nrows):
            at = fs + r * row_size
            row = []
            for name, t, w in zip(names, types, widths):
                if t == "INT":
                    row.append(struct.unpack_from(">i", b, at)[0])
                elif t == "LONG":
                    row.append(struct.unpack_from(">q", b, at)[0])
                elif t == "FLOAT":
                    row.append(struct.unpack_from(">f", b, at)[0])
                elif t == "DOUBLE":
                    row.append(struct.unpack_from(">d", b, at)[0])
                elif t in ("STRING", "BYTES"):
                    row.append(rev[name][struct.unpack_from(">i", b, at)[0]])
                else:
                    p, ln = struct.unpack_from(">ii", b, at)
                    tid = struct.unpack_from(">i", var, p)[0]
                    row.append((tid, deserialize_object(tid, var[p + 4:p + 4 + ln])))
                at += w
            rows.append(row)
    end = max(HEADER_SIZE, *(s + l for s, l in sec))
    meta_len = struct.unpack_from(">i", b, end)[0]
    metadata = {}
    if meta_len:
        n = struct.unpack_from(">i", b, end + 4)[0]
        pos = end + 8
        for _ in range(n):
            kid = struct.unpack_from(">i", b, pos)[0]
            pos += 4
            name, kt = METADATA_BY_ID[kid]
            if kt == "INT":
                metadata[name] = str(struct.unpack_from(">i", b, pos)[0])
                pos += 4
            elif kt == "LONG":
                metadata[name] = str(struct.unpack_from(">q", b, pos)[0])
                pos += 8
            else:
                metadata[name], pos = _str_at(b, pos)
    return DataTable(schema, rows, metadata, exceptions)


# ------------------------------------------------------------------------------------------------ results <-> tables

def _stats_metadata(st: ExecutionStats, groups_limit_reached: bool = False) -> Dict[str, str]:
    """IntermediateResultsBlock.attachMetadataToDataTable (consuming-segment counters are 0 on immutable segments)."""
    md = {"numDocsScanned": st.num_docs_scanned, "numEntriesScannedInFilter": st.num_entries_scanned_in_filter,
          "numEntriesScannedPostFilter": st.num_entries_scanned_post_filter,
          "numSegmentsProcessed": st.num_segments_processed, "numSegmentsMatched": st.num_segments_matched,
          "numConsumingSegmentsProcessed": 0, "numConsumingSegmentsMatched": 0, "numResizes": 0, "resizeTimeMs": 0,
          "totalDocs": st.num_total_docs}
    out = {k: str(int(v)) for k, v in md.items()}
    if groups_limit_reached:
        out["numGroupsLimitReached"] = "true"
    return out


def _cell(ag: Aggregation, v, column_type):
    f = ag.function
    if f in ("COUNT", "COUNTMV"):
        return int(round(v))
    if f in ("SUM", "MIN", "MAX"):
        return float(v)
    if f == "AVG":
        return (OBJ_AVG_PAIR, (float(v[0]), int(v[1])))
    if f == "DISTINCTCOUNT":
        if not isinstance(v, set):
            raise ValueError("DISTINCTCOUNT crosses the wire as a value set: run the device path with "
                             "PG_PLAN_VALUE_SETS")
        return (SET_TYPE_OF_COLUMN[column_type(ag.arg.cols[0])], v)
    raise ValueError(f)


def result_to_datatable(query: QueryContext, res: IntermediateResult, column_type,
                        groups_limit_reached: bool = False) -> DataTable:
    """The server's DataTable for an aggregation / group-by result (IntermediateResultsBlock.getDataTable).
    `column_type(name)` gives a column's stored data type (INT / LONG / FLOAT / DOUBLE / STRING / BYTES; BYTES values
    as hex strings, as the reference's DataTable V3 carries them)."""
    aggs = res.aggregations
    md = _stats_metadata(res.stats, groups_limit_reached)
    if not res.group_by:
        from .plan import default_row
        vals = res.rows.get((), None) or default_row(aggs)
        schema = DataSchema([column_name(a) for a in aggs], [_INTERMEDIATE_TYPE[a.function] for a in aggs])
        return DataTable(schema, [[_cell(a, v, column_type) for a, v in zip(aggs, vals)]], md)
    names = list(res.group_by) + [result_column_name(a) for a in aggs]
    types = [column_type(c) for c in res.group_by] + [_INTERMEDIATE_TYPE[a.function] for a in aggs]
    rows = [list(key) + [_cell(a, v, column_type) for a, v in zip(aggs, vals)] for key, vals in res.rows.items()]
    return DataTable(DataSchema(names, types), rows, md)


def _value(ag: Aggregation, cell):
    if ag.function in ("AVG", "DISTINCTCOUNT"):
        tid, v = cell
        return tuple(v) if ag.function == "AVG" else set(v)
    return cell


def datatable_to_result(query: QueryContext, dt: DataTable) -> IntermediateResult:
    """Back to value-keyed intermediates (what DataTableReducer implementations read)."""
    aggs = query.aggregations
    k = len(query.group_by)
    rows: Dict[tuple, list] = {}
    for r in dt.rows:
        key = tuple(r[:k])
        vals = [_value(a, c) for a, c in zip(aggs, r[k:])]
        rows[key] = merge_intermediate(aggs, rows[key], vals) if key in rows else vals
    md = dt.metadata
    st = ExecutionStats(int(md.get("numDocsScanned", 0)), int(md.get("numEntriesScannedInFilter", 0)),
                        int(md.get("numEntriesScannedPostFilter", 0)), int(md.get("totalDocs", 0)),
                        int(md.get("numSegmentsProcessed", 0)), int(md.get("numSegmentsMatched", 0)))
    return IntermediateResult(aggs, list(query.group_by), rows, st)


def broker_reduce(query: QueryContext, tables: Sequence[bytes]) -> Tuple[List[str], List[list], ExecutionStats]:
    """BrokerReduceService: decode every server's DataTable, merge by key, final values + ORDER BY / LIMIT; the
    execution statistics summed over servers."""
    merged: Optional[IntermediateResult] = None
    for raw in tables:
        dt = from_bytes(raw)
        if dt.exceptions:
            raise RuntimeError(f"server exceptions: {dt.exceptions}")
        r = datatable_to_result(query, dt)
        if merged is None:
            merged = r
            continue
        for key, vals in r.rows.items():
            merged.rows[key] = merge_intermediate(merged.aggregations, merged.rows[key], vals) \
                if key in merged.rows else vals
        for f in ("num_docs_scanned", "num_entries_scanned_in_filter", "num_entries_scanned_post_filter",
                  "num_total_docs", "num_segments_processed", "num_segments_matched"):
            setattr(merged.stats, f, getattr(merged.stats, f) + getattr(r.stats, f))
    if merged is None:
        merged = IntermediateResult(query.aggregations, list(query.group_by), {})
    names, rows = reduce_to_rows(query, merged)
    return names, rows, merged.stats

