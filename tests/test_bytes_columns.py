"""BYTES columns: dictionaries in the reference's layout (SegmentDictionaryCreator.java:202-221 -- ByteArray values
sorted unsigned-lexicographically, stored as their raw bytes zero-padded to the longest entry; BytesDictionary reads
them back without the padding), values presented as lowercase hex strings (BytesUtils.toHexString, as query literals
and results carry them), group keys and DISTINCTCOUNT values through the keymap, the DataTable V3 forms (a BYTES cell
is its hex string through the dictionary map, DataTableBuilderV2V3.setColumn(ByteArray) :69-72; a DISTINCTCOUNT set is
BYTES_SET_SER_DE, ObjectSerDeUtils.java:774-793) and HAVING on a BYTES key (HavingFilterHandlerTest.java:91-97).
Parity is pinned by the reference's own layout rules and known answers; no serialized BYTES fixture exists in it."""
import struct

import numpy as np
import pytest

from pinot_amd import datatable as dtm
from pinot_amd.plan import Table, having_match, reduce_to_rows
from pinot_amd.query import parse
from pinot_amd.segment import Dictionary, ImmutableSegment, build_dictionary

VALUES = [b"\x80", b"\x7f\x01", b"\xff", b"\x01", b"\x01\x02\x03", b"\x7f", b"\x00\x11"]


def test_dictionary_layout_and_order():
    d, ids = build_dictionary("BYTES", VALUES + [v.hex() for v in VALUES])  # bytes and hex strings are one value
    want = sorted(VALUES)  # Python compares bytes unsigned-lexicographically, as ByteArray.compare does
    assert d.values == [v.hex() for v in want] and d.entry_bytes == 3
    assert d.to_bytes() == b"".join(v + b"\0" * (3 - len(v)) for v in want)
    assert list(ids[:len(VALUES)]) == list(ids[len(VALUES):]) == [want.index(v) for v in VALUES]
    back = Dictionary.from_bytes("BYTES", d.to_bytes(), len(want), 3)
    assert back.values == d.values
    assert d.index_of("7F01") == want.index(b"\x7f\x01") and d.index_of("0203") == -1


def _segments():
    rng = np.random.default_rng(5)
    segs = []
    for s in range(3):
        n = 4000 + 77 * s
        data = {"b": [VALUES[i] for i in rng.integers(0, len(VALUES), n)],
                "k": rng.integers(0, 6, n), "v": rng.integers(0, 1000, n)}
        segs.append(ImmutableSegment.create(f"b{s}", data, {"b": "BYTES", "k": "INT", "v": "INT"}))
    return segs


QUERIES = [
    "SELECT b, COUNT(*), SUM(v) FROM t GROUP BY b",
    "SELECT k, DISTINCTCOUNT(b), MAX(v) FROM t WHERE v < 500 GROUP BY k",
    "SELECT b, k, COUNT(*) FROM t WHERE b IN ('7f01', 'ff', '010203') GROUP BY b, k",
    "SELECT DISTINCTCOUNT(b), COUNT(*) FROM t WHERE b <> '80'",
]


@pytest.fixture(scope="module")
def bytes_table():
    return Table("t", _segments())


def _np_rows(table, sql):
    q = parse(sql)
    b = np.concatenate([np.asarray(s.columns["b"].dictionary.values, dtype=object)[s.columns["b"].dict_ids]
                        for s in table.segments])
    k = np.concatenate([np.asarray(s.columns["k"].dictionary.values)[s.columns["k"].dict_ids] for s in table.segments])
    v = np.concatenate([np.asarray(s.columns["v"].dictionary.values)[s.columns["v"].dict_ids] for s in table.segments])
    return q, b, k, v


def test_oracle_groups_bytes_keys_by_value(bytes_table, oracle_engine):
    q, b, k, v = _np_rows(bytes_table, QUERIES[0])
    res = oracle_engine.execute(bytes_table, q)
    want = {(x,): [int((b == x).sum()), float(v[b == x].sum())] for x in set(b)}
    assert {kk: [r[0], r[1]] for kk, r in res.rows.items()} == want
    q, b, k, v = _np_rows(bytes_table, QUERIES[1])
    res = oracle_engine.execute(bytes_table, q)
    for kk, row in res.rows.items():
        m = (k == kk[0]) & (v < 500)
        assert row[0] == set(b[m]) and row[1] == float(v[m].max())


@pytest.mark.parametrize("sql", QUERIES)
def test_bytes_results_cross_the_datatable(sql, bytes_table, oracle_engine):
    """Two servers' DataTables (BYTES keys as hex strings in the dictionary map, BYTES value sets as BytesSet) reduce to
    the whole table's answer."""
    q = parse(sql)
    ref = reduce_to_rows(q, oracle_engine.execute(bytes_table, q))
    tables = []
    for segs in (bytes_table.segments[:1], bytes_table.segments[1:]):
        t = Table("t", segs)
        dt = dtm.result_to_datatable(q, oracle_engine.execute(t, q), t.data_type)
        raw = dtm.to_bytes(dt)
        assert dtm.from_bytes(raw).rows == dt.rows
        tables.append(raw)
    assert dtm.broker_reduce(q, tables)[:2] == ref


def test_bytes_set_serde_layout():
    raw = dtm.serialize_object(dtm.OBJ_BYTES_SET, {"ff", "0102"})
    assert raw == struct.pack(">i", 2) + struct.pack(">i", 2) + b"\x01\x02" + struct.pack(">i", 1) + b"\xff"
    assert dtm.deserialize_object(dtm.OBJ_BYTES_SET, raw) == {"ff", "0102"}


def test_having_on_a_bytes_key():
    """HavingFilterHandlerTest.java:91-97's BYTES key d6 (byte[]{17} > 10 is true, byte[]{16} > 10 false): the key as
    its hex string, the literal read as hex."""
    sql = "SELECT COUNT(*) FROM testTable GROUP BY d6 HAVING d6 > 10"
    q = parse(sql)
    idx = {a: i for i, a in enumerate(q.aggregations)}
    assert having_match(q.having, q, idx, (bytes([17]).hex(),), [5])
    assert not having_match(q.having, q, idx, (bytes([16]).hex(),), [5])


def test_v1_v3_round_trip(tmp_path):
    seg = _segments()[0]
    for writer, sub in ((seg.write_v1, "v1"), (seg.write_v3, "v3")):
        writer(str(tmp_path / sub))
        back = ImmutableSegment.load(str(tmp_path / sub))
        c, o = back.columns["b"], seg.columns["b"]
        assert c.dictionary.values == o.dictionary.values and c.dictionary.entry_bytes == 3
        assert c.dictionary.to_bytes() == o.dictionary.to_bytes()


@pytest.mark.gpu
@pytest.mark.parametrize("sql", QUERIES)
def test_bytes_columns_on_device(sql, bytes_table, gpu_engine, oracle_engine):
    from helpers import assert_same_result
    q = parse(sql)
    assert_same_result(gpu_engine.execute(bytes_table, q), oracle_engine.execute(bytes_table, q), table=bytes_table)
