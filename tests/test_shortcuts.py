"""The reference's O(index) / O(dictionary) operators, on the oracle and through the device path.

* FastFilteredCountOperator (operator/query/FastFilteredCountOperator.java:44-76): COUNT(*) over index-backed filters is
  the filter's matching-doc count; ExecutionStatistics(count, 0, 0, totalDocs).  Known answers: the non-TEXT/JSON cases
  of the reference's FastFilteredCountTest.java:153-306 on its own 1 000-row data (:103-115: class = i % 8 with an
  inverted index, sorted = i, intRangeCol = 1000 - i), two copies of the segment as in the test's inter-segment list.
* NonScanBasedAggregationOperator (operator/query/NonScanBasedAggregationOperator.java:80-150, chosen per segment by
  AggregationPlanNode.java:185-197): no group-by, a match-all filter in that segment, COUNT / MIN / MAX /
  DISTINCTCOUNT of dictionary columns -> answers from the dictionary with ExecutionStatistics(numTotalDocs, 0, 0,
  numTotalDocs).  The device path takes the same route per segment (no scan of those segments)."""
import numpy as np
import pytest

from pinot_amd.plan import Table, reduce_to_rows
from pinot_amd.query import parse
from pinot_amd.segment import ImmutableSegment

N, B = 1000, 8


def _fast_count_segment():
    i = np.arange(N)
    data = {"class": i % B, "sorted": i, "intRangeCol": N - i}
    return ImmutableSegment.create("testSegment", data, {"class": "INT", "sorted": "INT", "intRangeCol": "INT"},
                                   inverted=("class",))


def _cases():
    bc, bcc = N // B, N - N // B
    mn, mx = 20, N - 20
    all_b = "(" + ", ".join(str(x) for x in range(B)) + ")"
    two = "(0, 7)"
    t = "SELECT COUNT(*) FROM testTable"
    return [
        (t, N),
        (f"{t} WHERE class = 1", bc),
        (f"{t} WHERE sorted = 1", 1),
        (f"{t} WHERE sorted BETWEEN {mn} AND {mx}", mx - mn + 1),
        (f"{t} WHERE sorted NOT BETWEEN {mn} AND {mx}", N - (mx - mn + 1)),
        (f"{t} WHERE sorted IN {all_b}", B),
        (f"{t} WHERE sorted IN {all_b} AND class IN {all_b}", B),
        (f"{t} WHERE class <> 1", bcc),
        (f"{t} WHERE class IN {two}", 2 * bc),
        (f"{t} WHERE class NOT IN {two}", N - 2 * bc),
        (f"{t} WHERE class IN {two} AND sorted < {N // 2}", bc),
        (f"{t} WHERE sorted = 1 AND class = 1", 1),
        (f"{t} WHERE sorted = 1 AND class <> 1", 0),
        (f"{t} WHERE sorted = 1 AND class <> 0", 1),
        (f"{t} WHERE sorted <> 1 AND class = 1", bc - 1),
        (f"{t} WHERE sorted >= 0 AND class = 1", bc),
        (f"{t} WHERE sorted > 1 AND class = 1", bc - 1),
        (f"{t} WHERE sorted >= 0 AND class <> 1", bcc),
        (f"{t} WHERE sorted >= 0 OR class <> 0", N),
        (f"{t} WHERE sorted < {bc} AND class <> 0", bc - bc // B - 1),
        (f"{t} WHERE sorted >= {bc} AND class <> 0", bcc - bcc // B),
        (f"{t} WHERE sorted < {B - 1} AND class = {B - 1}", 0),
        (f"{t} WHERE sorted >= {B - 2} AND class = {B - 2}", bc),
        (f"{t} WHERE sorted >= {mn} AND sorted < {mx} AND class = 0", bc - (mn + N - mx) // B),
        (f"{t} WHERE intRangeCol >= {mn} AND intRangeCol < {mx}", mx - mn),
        (f"{t} WHERE intRangeCol < {mx}", mx - 1),
        (f"{t} WHERE intRangeCol NOT BETWEEN {mn} AND {mx}", N - mx + mn - 1),
        (f"{t} WHERE intRangeCol BETWEEN {mn} AND {mx} AND class = 0", bc - (mn + N - mx) // B),
        (f"{t} WHERE intRangeCol NOT BETWEEN {mn} AND {mx} AND class = 0", (mn + N - mx) // B),
    ]


CASES = _cases()


@pytest.fixture(scope="module")
def fast_count_table():
    seg = _fast_count_segment()
    return Table("testTable", [seg, seg])


def _check_count(res, q, expected, segments):
    assert reduce_to_rows(q, res)[1] == [[expected * segments]]
    st = res.stats
    assert (st.num_docs_scanned, st.num_entries_scanned_post_filter, st.num_total_docs) == \
        (expected * segments, 0, N * segments)


@pytest.mark.parametrize("sql,expected", CASES)
def test_fast_filtered_count_known_answers_oracle(sql, expected, oracle_engine, fast_count_table):
    q = parse(sql)
    _check_count(oracle_engine.execute(fast_count_table, q), q, expected, 2)


NON_SCAN = [
    ("SELECT COUNT(*), MIN(sorted), MAX(intRangeCol), DISTINCTCOUNT(class) FROM testTable", True),
    ("SELECT MAX(class), MIN(class) FROM testTable WHERE sorted >= 0", True),            # always-true predicate
    ("SELECT COUNT(*), MAX(sorted) FROM testTable WHERE class < 100 OR sorted = 3", True),  # OR with a match-all
    ("SELECT COUNT(*), MIN(sorted) FROM testTable WHERE NOT class > 100", True),          # NOT(empty)
    ("SELECT MIN(sorted) FROM testTable WHERE class = 3", False),                        # a real filter: scanned
    ("SELECT SUM(sorted), MIN(sorted) FROM testTable", False),                           # SUM needs the docs
]


@pytest.mark.parametrize("sql,non_scan", NON_SCAN)
def test_non_scan_aggregation_oracle(sql, non_scan, oracle_engine, fast_count_table):
    q = parse(sql)
    res = oracle_engine.execute(fast_count_table, q)
    seg = fast_count_table.segments[0]
    for ag, v in zip(res.aggregations, res.rows[()]):
        col = ag.arg.cols[0] if ag.arg.cols else None
        if non_scan and ag.function in ("MIN", "MAX"):
            vals = seg.columns[col].dictionary.values
            assert v == float(vals[0] if ag.function == "MIN" else vals[-1])
    if non_scan:
        assert (res.stats.num_docs_scanned, res.stats.num_entries_scanned_post_filter) == (2 * N, 0)
    else:
        assert res.stats.num_entries_scanned_post_filter == res.stats.num_docs_scanned * len(
            {c for a in q.aggregations for c in a.arg.cols})


@pytest.mark.gpu
@pytest.mark.parametrize("sql,expected", CASES)
def test_fast_filtered_count_known_answers_gpu(sql, expected, gpu_engine, fast_count_table):
    q = parse(sql)
    _check_count(gpu_engine.execute(fast_count_table, q), q, expected, 2)


@pytest.mark.gpu
@pytest.mark.parametrize("sql,non_scan", NON_SCAN)
def test_non_scan_aggregation_gpu(sql, non_scan, gpu_engine, oracle_engine, fast_count_table):
    from helpers import assert_same_result
    q = parse(sql)
    assert_same_result(gpu_engine.execute(fast_count_table, q), oracle_engine.execute(fast_count_table, q),
                       table=fast_count_table)


@pytest.mark.gpu
def test_non_scan_mixed_segments_gpu(gpu_engine, oracle_engine):
    """A predicate that is always true in one segment (its dictionary lies inside the range) and a real filter in the
    other: the first is answered from its dictionary, the second scanned; results and statistics as the oracle's."""
    from helpers import assert_same_result
    a = ImmutableSegment.create("a", {"x": np.arange(100, 200), "y": np.arange(100) % 7}, {"x": "INT", "y": "INT"})
    b = ImmutableSegment.create("b", {"x": np.arange(0, 300), "y": np.arange(300) % 5}, {"x": "INT", "y": "INT"})
    t = Table("t", [a, b])
    for sql in ["SELECT COUNT(*), MIN(y), MAX(x), DISTINCTCOUNT(y) FROM t WHERE x >= 100",
                "SELECT MIN(x), MAX(y) FROM t WHERE x BETWEEN 50 AND 250"]:
        q = parse(sql)
        assert_same_result(gpu_engine.execute(t, q), oracle_engine.execute(t, q), table=t)
