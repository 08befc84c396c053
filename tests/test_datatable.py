"""DataTable V3 serialization of server results and the broker reduce (pinot_amd/datatable.py).

Parity unpinned for the bytes (the reference holds no serialized DataTable fixture): the layout is checked field by
field against DataTableImplV3.toBytes / BaseDataTableBuilder as restated in the module docstring, results round trip,
and DataTables of split segments reduce to the whole-table oracle answer."""
import struct

import pytest

from pinot_amd import datatable as dtm
from pinot_amd.plan import Table, reduce_to_rows
from pinot_amd.query import parse

QUERIES = [
    "SELECT COUNT(*), SUM(column1), MIN(column3), MAX(column6), AVG(column7) FROM t",
    "SELECT DISTINCTCOUNT(column1), DISTINCTCOUNT(column11) FROM t WHERE column3 > 1000000000",
    "SELECT COUNT(*) FROM t WHERE column5 = 'nope'",
    "SELECT column11, COUNT(*), SUM(column1), MIN(column3), MAX(column3), AVG(column9) FROM t GROUP BY column11",
    "SELECT column11, column12, SUM(column1) FROM t GROUP BY column11, column12 ORDER BY SUM(column1) DESC, "
    "column11, column12 LIMIT 7",
    "SELECT column12, DISTINCTCOUNT(column11), DISTINCTCOUNT(column7) FROM t GROUP BY column12",
    "SELECT daysSinceEpoch, column17, SUM(column18) FROM t WHERE column11 NOT IN ('t', 'P') "
    "GROUP BY daysSinceEpoch, column17",
]


def _i(b, off):
    return struct.unpack_from(">i", b, off)[0]


def test_layout_of_an_aggregation_table():
    """Header offsets, schema bytes, fixed-size row and variable-size objects exactly as DataTableImplV3 writes them."""
    schema = dtm.DataSchema(["count_star", "sum_x", "avg_y", "distinctCount_z"], ["LONG", "DOUBLE", "OBJECT", "OBJECT"])
    dt = dtm.DataTable(schema, [[7, 2.5, (dtm.OBJ_AVG_PAIR, (10.0, 4)), (dtm.OBJ_INT_SET, {3, -1})]],
                       {"numDocsScanned": "7", "totalDocs": "100", "numSegmentsProcessed": "2"})
    b = dtm.to_bytes(dt)
    assert (_i(b, 0), _i(b, 4), _i(b, 8)) == (3, 1, 4)
    sec = [(_i(b, 12 + 8 * k), _i(b, 16 + 8 * k)) for k in range(5)]
    assert sec[0] == (52, 4) and _i(b, 52) == 0               # no exceptions: just the count
    assert sec[1] == (56, 0)                                    # no STRING columns: no dictionary map
    exp_schema = struct.pack(">i", 4)
    for s in schema.names + schema.types:
        exp_schema += struct.pack(">i", len(s)) + s.encode()
    assert sec[2] == (56, len(exp_schema)) and b[56:56 + len(exp_schema)] == exp_schema
    fs, fl = sec[3]
    assert fl == 32  # LONG 8 + DOUBLE 8 + 2 x (position, length)
    avg = struct.pack(">dq", 10.0, 4)
    iset = struct.pack(">iii", 2, -1, 3)
    assert b[fs:fs + 32] == struct.pack(">qdiiii", 7, 2.5, 0, len(avg), 4 + len(avg), len(iset))
    vs, vl = sec[4]
    assert vs == fs + fl and b[vs:vs + vl] == struct.pack(">i", 4) + avg + struct.pack(">i", 9) + iset
    mlen = _i(b, vs + vl)
    assert vs + vl + 4 + mlen == len(b)
    meta = b[vs + vl + 4:]
    assert _i(meta, 0) == 3
    assert meta[4:] == (struct.pack(">iq", 2, 7) + struct.pack(">iq", 10, 100) + struct.pack(">ii", 6, 2))
    back = dtm.from_bytes(b)
    assert back.schema == schema and back.metadata == dt.metadata
    assert back.rows == [[7, 2.5, (4, (10.0, 4)), (9, {3, -1})]]


def test_string_keys_go_through_the_dictionary_map():
    schema = dtm.DataSchema(["column11", "count(*)"], ["STRING", "LONG"])
    rows = [["P", 3], ["o", 4], ["P", 5]]
    b = dtm.to_bytes(dtm.DataTable(schema, rows, {}, {200: "boom"}))
    (ds, dl) = (_i(b, 20), _i(b, 24))
    exp = struct.pack(">i", 1) + struct.pack(">i", 8) + b"column11" + struct.pack(">i", 2)
    exp += struct.pack(">i", 0) + struct.pack(">i", 1) + b"P" + struct.pack(">i", 1) + struct.pack(">i", 1) + b"o"
    assert b[ds:ds + dl] == exp
    fs = _i(b, 36)
    assert [_i(b, fs + 12 * r) for r in range(3)] == [0, 1, 0]
    back = dtm.from_bytes(b)
    assert back.rows == rows and back.exceptions == {200: "boom"}


@pytest.mark.parametrize("sql", QUERIES)
def test_results_round_trip_and_reduce_like_the_oracle(sql, oracle_engine, sv_segment):
    """Two servers of two segments each: each server's oracle result -> DataTable bytes -> broker reduce == the
    oracle over all four segments (the reference's inter-segment test setup, BaseQueriesTest.java:151-190)."""
    q = parse(sql)
    whole = Table("t", [sv_segment] * 4)
    ref = reduce_to_rows(q, oracle_engine.execute(whole, q))
    tables = []
    for _ in range(2):
        t = Table("t", [sv_segment] * 2)
        res = oracle_engine.execute(t, q)
        dt = dtm.result_to_datatable(q, res, t.data_type)
        raw = dtm.to_bytes(dt)
        back = dtm.from_bytes(raw)
        assert back.rows == dt.rows and back.metadata == dt.metadata
        tables.append(raw)
    names, rows, stats = dtm.broker_reduce(q, tables)
    assert (names, rows) == ref
    st = oracle_engine.execute(whole, q).stats
    assert (stats.num_docs_scanned, stats.num_total_docs) == (st.num_docs_scanned, st.num_total_docs)


def test_distinct_count_must_cross_as_a_set():
    q = parse("SELECT DISTINCTCOUNT(column1) FROM t")
    from pinot_amd.plan import IntermediateResult
    res = IntermediateResult(q.aggregations, [], {(): [17]})
    with pytest.raises(ValueError):
        dtm.result_to_datatable(q, res, lambda c: "INT")


@pytest.mark.gpu
@pytest.mark.parametrize("sql", QUERIES)
def test_device_results_serialize_and_reduce(sql, gpu_engine, oracle_engine, sv_segment):
    """The device path's server result (value sets for DISTINCTCOUNT) as DataTable bytes from two servers reduces to
    the oracle's whole-table answer."""
    q = parse(sql)
    ref = reduce_to_rows(q, oracle_engine.execute(Table("t", [sv_segment] * 4), q))
    tables = []
    for _ in range(2):
        t = Table("t", [sv_segment] * 2)
        tables.append(dtm.to_bytes(dtm.result_to_datatable(q, gpu_engine.execute(t, q), t.data_type)))
    assert dtm.broker_reduce(q, tables)[:2] == ref
