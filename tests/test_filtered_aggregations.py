"""Filtered aggregations: `AGG(x) FILTER (WHERE f)` -- AggregationPlanNode.buildFilteredAggOperator
(plan/AggregationPlanNode.java:87-146) + FilteredAggregationOperator (operator/query/FilteredAggregationOperator.java
:70-98): one pass per distinct aggregation filter over main AND f, the main pass for the rest; statistics summed.

Data and queries: the reference's FilteredAggregationsTest.java:111-123 (30 000 rows, INT_COL = NO_INDEX_COL = i with an
inverted index on INT_COL, STATIC_INT_COL = 10; two identical segments) and the cases of :164-300 that the SQL subset
expresses (no BOOLEAN / STARTSWITH / MOD / ABS / LN / CASE WHEN).  The reference checks each filtered query against an
equivalent non-filtered one; here every aggregation is also checked against a numpy evaluation of its combined filter."""
import numpy as np
import pytest

from pinot_amd.plan import Table, reduce_to_rows
from pinot_amd.query import parse
from pinot_amd.segment import ImmutableSegment

NUM_ROWS = 30000


@pytest.fixture(scope="module")
def filtered_table():
    i = np.arange(NUM_ROWS)
    data = {"INT_COL": i, "NO_INDEX_COL": i.copy(), "STATIC_INT_COL": np.full(NUM_ROWS, 10)}
    types = {"INT_COL": "INT", "NO_INDEX_COL": "INT", "STATIC_INT_COL": "INT"}
    segs = [ImmutableSegment.create(n, data, types, inverted=("INT_COL",))
            for n in ("firstTestSegment", "secondTestSegment")]
    return Table("MyTable", segs)


# (filtered query, equivalent non-filtered query or None): FilteredAggregationsTest.java:164-300
PAIRS = [
    ("SELECT SUM(INT_COL) FILTER(WHERE INT_COL > 9999) FROM MyTable WHERE INT_COL < 1000000",
     "SELECT SUM(INT_COL) FROM MyTable WHERE INT_COL > 9999 AND INT_COL < 1000000"),
    ("SELECT SUM(INT_COL) FILTER(WHERE INT_COL < 3) FROM MyTable WHERE INT_COL > 1",
     "SELECT SUM(INT_COL) FROM MyTable WHERE INT_COL > 1 AND INT_COL < 3"),
    ("SELECT COUNT(*) FILTER(WHERE INT_COL = 4) FROM MyTable", "SELECT COUNT(*) FROM MyTable WHERE INT_COL = 4"),
    ("SELECT SUM(INT_COL) FILTER(WHERE INT_COL > 8000) FROM MyTable ",
     "SELECT SUM(INT_COL) FROM MyTable WHERE INT_COL > 8000"),
    ("SELECT SUM(INT_COL) FILTER(WHERE NO_INDEX_COL <= 1) FROM MyTable WHERE INT_COL > 1",
     "SELECT SUM(INT_COL) FROM MyTable WHERE NO_INDEX_COL <= 1 AND INT_COL > 1"),
    ("SELECT AVG(INT_COL) FILTER(WHERE NO_INDEX_COL > -1) FROM MyTable", "SELECT AVG(INT_COL) FROM MyTable"),
    ("SELECT MIN(INT_COL) FILTER(WHERE NO_INDEX_COL > 29990), MAX(INT_COL) FILTER(WHERE INT_COL > 29990) FROM MyTable",
     "SELECT MIN(INT_COL), MAX(INT_COL) FROM MyTable WHERE INT_COL > 29990"),
    ("SELECT SUM(INT_COL) FILTER(WHERE INT_COL > 1234 AND INT_COL < 22000) AS total_sum FROM MyTable",
     "SELECT SUM(INT_COL) AS total_sum FROM MyTable WHERE INT_COL > 1234 AND INT_COL < 22000"),
    ("SELECT MAX(INT_COL) FILTER(WHERE INT_COL < 100) AS total_max FROM MyTable",
     "SELECT MAX(INT_COL) AS total_max FROM MyTable WHERE INT_COL < 100"),
    ("SELECT SUM(INT_COL) FILTER(WHERE INT_COL > 3) AS total_sum, SUM(INT_COL) FILTER(WHERE INT_COL < 4) AS total_sum2 "
     "FROM MyTable WHERE INT_COL > 2", None),
    ("SELECT SUM(INT_COL) FILTER(WHERE INT_COL > 12345) AS total_sum, SUM(INT_COL) FILTER(WHERE INT_COL < 59999) AS "
     "total_sum2, MIN(INT_COL) FILTER(WHERE INT_COL > 5000) AS total_min FROM MyTable WHERE INT_COL > 1000", None),
    ("SELECT SUM(INT_COL) FILTER(WHERE NO_INDEX_COL > 12345) AS total_sum, SUM(INT_COL) FILTER(WHERE NO_INDEX_COL < "
     "59999) AS total_sum2, MIN(INT_COL) FILTER(WHERE NO_INDEX_COL > 5000) AS total_min FROM MyTable WHERE INT_COL > "
     "1000", None),
    ("SELECT SUM(INT_COL) FILTER(WHERE INT_COL > 123 AND INT_COL < 25000) AS total_sum, MAX(INT_COL) FILTER(WHERE "
     "INT_COL > 123 AND INT_COL < 25000) AS total_max FROM MyTable", None),
    ("SELECT MIN(INT_COL) FILTER(WHERE NO_INDEX_COL > 29990) AS total_min, MAX(INT_COL) FILTER(WHERE INT_COL > 29990) "
     "AS total_max, SUM(INT_COL) FILTER(WHERE NO_INDEX_COL < 5000) AS total_sum, MAX(NO_INDEX_COL) FILTER(WHERE "
     "NO_INDEX_COL < 5000) AS total_max2 FROM MyTable", None),
    ("SELECT SUM(INT_COL), SUM(INT_COL) FILTER(WHERE INT_COL > 25000) AS total_sum FROM MyTable", None),
    ("SELECT SUM(INT_COL) FILTER(WHERE NO_INDEX_COL > 5), MAX(NO_INDEX_COL) FROM MyTable WHERE NO_INDEX_COL > 5", None),
    ("SELECT COUNT(*) FILTER(WHERE INT_COL IN (1, 2, 3)), COUNT(*), DISTINCTCOUNT(STATIC_INT_COL) FILTER(WHERE "
     "NOT INT_COL < 29000) FROM MyTable WHERE NO_INDEX_COL <> 2", None),
]


def _mask(f, vals):
    n = NUM_ROWS
    if f is None:
        return np.ones(n, dtype=bool)
    if f.type in ("AND", "OR"):
        ms = [_mask(c, vals) for c in f.children]
        return np.logical_and.reduce(ms) if f.type == "AND" else np.logical_or.reduce(ms)
    if f.type == "NOT":
        return ~_mask(f.children[0], vals)
    p = f.predicate
    v = vals[p.column]
    if p.type in ("EQ", "IN"):
        return np.isin(v, [int(x) for x in p.values])
    if p.type in ("NOT_EQ", "NOT_IN"):
        return ~np.isin(v, [int(x) for x in p.values])
    m = np.ones(n, dtype=bool)
    if p.lower != "*":
        m &= (v >= float(p.lower)) if p.lower_inclusive else (v > float(p.lower))
    if p.upper != "*":
        m &= (v <= float(p.upper)) if p.upper_inclusive else (v < float(p.upper))
    return m


def _expected(q):
    """Final values of each select item from numpy (two identical segments: counts and sums doubled)."""
    i = np.arange(NUM_ROWS)
    vals = {"INT_COL": i, "NO_INDEX_COL": i, "STATIC_INT_COL": np.full(NUM_ROWS, 10)}
    main = _mask(q.filter, vals)
    out = []
    for s in q.select:
        ag = s.agg
        m = main & _mask(ag.filter, vals)
        x = vals[ag.arg.cols[0]][m] if ag.arg.cols else None
        f = ag.function
        out.append(2 * int(m.sum()) if f == "COUNT" else 2.0 * x.sum() if f == "SUM" else
                   (float(x.min()) if x.size else float("inf")) if f == "MIN" else
                   (float(x.max()) if x.size else float("-inf")) if f == "MAX" else
                   (float(x.mean()) if x.size else float("-inf")) if f == "AVG" else len(set(x.tolist())))
    return out, main


def _check(engine, table, sql, equivalent):
    q = parse(sql)
    res = engine.execute(table, q)
    names, rows = reduce_to_rows(q, res)
    exp, main = _expected(q)
    assert rows[0] == exp, (rows[0], exp)
    if equivalent is not None:  # FilteredAggregationsTest.testQuery: same rows as the non-filtered form
        q2 = parse(equivalent)
        assert reduce_to_rows(q2, engine.execute(table, q2))[1] == rows
    # FilteredAggregationOperator statistics: docs of every pass (each = main AND its filter) + the main pass
    i = np.arange(NUM_ROWS)
    vals = {"INT_COL": i, "NO_INDEX_COL": i, "STATIC_INT_COL": np.full(NUM_ROWS, 10)}
    from pinot_amd.plan import filtered_aggregation_passes
    passes = filtered_aggregation_passes(q)
    docs = sum(2 * int(_mask(pq.filter, vals).sum()) for pq, _ in passes)
    if passes[-1][1]:  # non-filtered functions: a match-all pass over the main filter's docs besides the main pass
        docs += 2 * int(main.sum())
    cols = len({c for a in q.aggregations for c in a.arg.cols})
    st = res.stats
    assert (st.num_docs_scanned, st.num_entries_scanned_post_filter, st.num_total_docs) == (docs, docs * cols,
                                                                                            2 * NUM_ROWS)
    assert st.num_segments_matched == (2 if main.any() else 0)


@pytest.mark.parametrize("sql,equivalent", PAIRS)
def test_filtered_aggregations_oracle(sql, equivalent, oracle_engine, filtered_table):
    _check(oracle_engine, filtered_table, sql, equivalent)


def test_group_by_with_filter_is_rejected():
    with pytest.raises(ValueError, match="GROUP BY with FILTER"):
        parse("SELECT STATIC_INT_COL, SUM(INT_COL) FILTER(WHERE INT_COL > 3) FROM MyTable GROUP BY STATIC_INT_COL")


def test_same_filter_is_one_pass():
    q = parse("SELECT SUM(INT_COL) FILTER(WHERE INT_COL > 3), MAX(INT_COL) FILTER(WHERE INT_COL > 3), "
              "MIN(INT_COL) FILTER(WHERE INT_COL > 4), COUNT(*) FROM MyTable")
    from pinot_amd.plan import filtered_aggregation_passes
    passes = filtered_aggregation_passes(q)
    assert [idx for _, idx in passes] == [[0, 1], [2], [3]]


@pytest.mark.gpu
@pytest.mark.parametrize("sql,equivalent", PAIRS)
def test_filtered_aggregations_gpu(sql, equivalent, gpu_engine, oracle_engine, filtered_table):
    from helpers import assert_same_result
    _check(gpu_engine, filtered_table, sql, equivalent)
    q = parse(sql)
    assert_same_result(gpu_engine.execute(filtered_table, q), oracle_engine.execute(filtered_table, q),
                       table=filtered_table)
