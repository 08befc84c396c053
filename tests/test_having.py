"""HAVING (QueryContext._havingFilter): parsed into post-aggregation predicates, its aggregations computed with the
query's (QueryContext.generateAggregationFunctions :514-560: select, HAVING, ORDER BY), the server trim sized as with
an ORDER BY (GroupByOrderByCombineOperator.java:82-84: getTableCapacity(limit, minServerGroupTrimSize)), and the filter
applied by the broker reduce to its sorted records until LIMIT rows passed (GroupByDataTableReducer.java:148-165,
HavingFilterHandler).

Pinned by the reference's own known answers: HavingFilterHandlerTest.java:33-104 (rows and isMatch results restated
below; its BYTES key case is in tests/test_bytes_columns.py)."""
import pytest

from helpers import assert_same_result
from pinot_amd import datatable as dtm
from pinot_amd.plan import Table, group_trim, having_match, reduce_to_rows
from pinot_amd.query import parse


def _match(sql, row):
    """isMatch of a row laid out as [group keys..., select values...] (the test's DataSchema order)."""
    q = parse(sql)
    aggs = q.aggregations
    idx = {a: i for i, a in enumerate(aggs)}
    K = len(q.group_by)
    finals = [None] * len(aggs)
    for s, v in zip(q.select, row[K:]):
        if s.kind == "AGG":
            finals[idx[s.agg]] = v
    return having_match(q.having, q, idx, tuple(row[:K]), finals)


@pytest.mark.parametrize("sql,rows", [
    ("SELECT COUNT(*) FROM testTable GROUP BY d1 HAVING COUNT(*) > 5",
     [((1, 5), False), ((2, 10), True), ((3, 3), False)]),
    ("SELECT MAX(m1), MIN(m1) FROM testTable GROUP BY d1 HAVING MAX(m1) IN (15, 20, 25) AND (MIN(m1) > 10 OR MIN(m1) <= 3)",
     [((1, 15.5, 13.0), False), ((2, 15.0, 3.0), True), ((3, 20.0, 7.5), False)]),
    ("SELECT MAX(m1), MIN(m2) FROM testTable GROUP BY d1 HAVING MAX(m1) > MIN(m2) * 2",
     [((1, 15.5, 13.0), False), ((2, 15.0, 3.0), True), ((3, 20.0, 10.0), False)]),
    ("SELECT COUNT(*) FROM testTable GROUP BY d1, d2, d3, d4, d5 HAVING d1 > 10 AND d2 > 10 AND d3 > 10 AND d4 > 10 "
     "AND d5 > '10'",
     [((11, 11, 10.5, 10.5, "11", 5), True), ((10, 11, 10.5, 10.5, "11", 5), False),
      ((11, 10, 10.5, 10.5, "11", 5), False), ((11, 11, 10.0, 10.5, "11", 5), False),
      ((11, 11, 10.5, 10.0, "11", 5), False), ((11, 11, 10.5, 10.5, "10", 5), False)]),
])
def test_having_filter_handler_known_answers(sql, rows):
    for row, want in rows:
        assert _match(sql, list(row)) == want, (row, want)


def test_having_parse_forms():
    q = parse("SELECT k, COUNT(*) AS c FROM t GROUP BY k HAVING c - 1 > 5 AND SUM(v) / (COUNT(*) + 2) < 3 "
              "AND NOT k BETWEEN 3 AND 9 ORDER BY c DESC LIMIT 3")
    assert [a.function for a in q.aggregations] == ["COUNT", "SUM"]   # HAVING-only SUM(v) is computed too
    with pytest.raises(ValueError):
        parse("SELECT COUNT(*) FROM t HAVING COUNT(*) > 1")              # HAVING needs a GROUP BY
    with pytest.raises(ValueError):
        parse("SELECT k, COUNT(*) FROM t GROUP BY k HAVING v > 1")       # v: neither a key nor an alias


def test_having_sizes_the_server_trim():
    gt = group_trim(parse("SELECT k, SUM(v) FROM t GROUP BY k HAVING SUM(v) > 0 LIMIT 100"))
    assert (gt.segment_size, gt.server_size, gt.ordered) == (None, 5000, False)   # capacity, not LIMIT
    gt = group_trim(parse("SELECT k, SUM(v) FROM t GROUP BY k HAVING SUM(v) > 0 LIMIT 7 OPTION(minServerGroupTrimSize=20)"))
    assert gt.server_size == 35


def _segments():
    from test_server_trim import _random_segments
    return _random_segments()


HAVING_QUERIES = [
    "SELECT k, SUM(v), COUNT(*) FROM t GROUP BY k HAVING COUNT(*) >= 14 ORDER BY SUM(v) DESC, k LIMIT 9",
    # ~12 000 (k, k2) groups: a server trim of getTableCapacity would make the merged values per-server approximations
    # (as in the reference), so the servers keep every group here
    "SELECT k, k2, MAX(v) FROM t GROUP BY k, k2 HAVING MAX(v) - MIN(v) < 50000 AND k2 <> 1 ORDER BY MAX(v), k, k2 "
    "LIMIT 20 OPTION(minServerGroupTrimSize=20000)",
    "SELECT k, DISTINCTCOUNT(i) AS d FROM t GROUP BY k HAVING d BETWEEN 8 AND 11 OR AVG(v) > 60000 ORDER BY d DESC, k "
    "LIMIT 15",
]


@pytest.mark.parametrize("sql", HAVING_QUERIES)
def test_oracle_having_two_servers_reduce_to_the_whole_table(sql, oracle_engine):
    """Two servers' trimmed results (each keeps all its groups) -> DataTables -> broker reduce with HAVING
    == the whole table's answer; every returned row passes HAVING and the ORDER BY is respected."""
    segs = _segments()
    q = parse(sql)
    want = reduce_to_rows(q, oracle_engine.execute(Table("t", segs), q))
    tables = []
    for part in (segs[:2], segs[2:]):
        t = Table("t", part)
        tables.append(dtm.to_bytes(dtm.result_to_datatable(q, oracle_engine.execute(t, q, server=True), t.data_type)))
    assert dtm.broker_reduce(q, tables)[:2] == want
    assert 0 < len(want[1]) <= q.limit


@pytest.mark.gpu
@pytest.mark.parametrize("sql", HAVING_QUERIES + [
    "SELECT k2, COUNT(*), SUM(v) FROM t GROUP BY k2 HAVING SUM(v) > 0 LIMIT 10",
])
def test_device_having(sql, gpu_engine, oracle_engine):
    """The device runs the HAVING query's aggregations (HAVING-only ones included) and server trim; the broker reduce
    of two device servers equals the oracle's whole-table answer."""
    segs = _segments()
    q = parse(sql)
    t_all = Table("t", segs)
    assert_same_result(gpu_engine.execute(t_all, q), oracle_engine.execute(t_all, q), table=t_all)
    want = reduce_to_rows(q, oracle_engine.execute(t_all, q))
    # trim=True (the final single-server answer): the device's ORDER BY cut keeps the broker's table capacity when
    # HAVING follows it, so groups failing HAVING never take LIMIT slots
    assert reduce_to_rows(q, gpu_engine.execute(t_all, q, trim=True))[:2] == want
    tables = []
    for part in (segs[:2], segs[2:]):
        t = Table("t", part)
        tables.append(dtm.to_bytes(dtm.result_to_datatable(q, gpu_engine.execute(t, q, trim="server"), t.data_type)))
    assert dtm.broker_reduce(q, tables)[:2] == want
