"""Helpers shared by the parity tests: turn expected.json cases into queries and compare results."""
import math

from pinot_amd.plan import final_value, reduce_to_rows
from pinot_amd.query import parse


def with_filter(query: str, filt: str) -> str:
    """Insert the shared FILTER where the case says `FILTER` (BaseSingleValueQueriesTest.java:73-77)."""
    return query.replace(" FILTER", filt) if " FILTER" in query else query


def inner_query(case, filt):
    q = case.get("query") or "SELECT COUNT(*), SUM(column1), MAX(column3), MIN(column6), AVG(column7) FROM testTable"
    if case.get("filtered"):
        q += filt
    if case.get("group_by"):
        q += " GROUP BY " + ", ".join(case["group_by"])
    return q


def check_inner_values(res, case):
    """QueriesTestUtils.testInnerSegmentAggregation(GroupBy)Result: longValue() of each result, AvgPair sum/count."""
    key = tuple(case.get("key", ()))
    assert key in res.rows, f"group key {key} missing; {len(res.rows)} groups, e.g. {sorted(res.rows.items())[:3]}"
    row = res.rows[key]
    exp = case["values"]
    for a, (ag, v, e) in enumerate(zip(res.aggregations, row, exp)):
        if ag.function == "AVG":
            assert int(v[0]) == e[0] and int(v[1]) == e[1], (a, v, e)
        else:
            assert int(v) == e, (a, ag, v, e)
    n_scanned, post, total = case["stats"]
    assert res.stats.num_docs_scanned == n_scanned
    assert res.stats.num_entries_scanned_post_filter == post
    assert res.stats.num_total_docs == total


def check_rows(got, exp, delta=None):
    assert len(got) == len(exp), (got, exp)
    for gr, er in zip(got, exp):
        assert len(gr) == len(er)
        for g, e in zip(gr, er):
            if isinstance(e, str):
                assert g == e, (gr, er)
            elif delta is not None:
                assert abs(float(g) - float(e)) <= delta * max(1.0, abs(float(e))), (gr, er)
            else:
                assert float(g) == float(e), (gr, er)


def run_rows(engine, table, sql):
    q = parse(sql)
    res = engine.execute(table, q)
    return q, res, reduce_to_rows(q, res)[1]


INTEGER_TYPES = ("INT", "LONG")


def _integer_input(ag, table):
    return table is not None and ag.arg.op in ("COL", "ADD", "SUB", "MUL") and \
        all(table.data_type(c) in INTEGER_TYPES for c in ag.arg.cols)


def _close(x, y, rel):
    """A double sum within `rel` of the oracle's; NaN matches NaN and an infinity the same infinity (IEEE sums of
    non-finite inputs are exact in any order)."""
    if math.isnan(y) or math.isinf(y):
        return (math.isnan(x) and math.isnan(y)) or x == y
    return math.isclose(x, y, rel_tol=rel, abs_tol=0)


def assert_same_result(a, b, rel=1e-9, table=None):
    """Device result vs oracle result, both IntermediateResult.  Bit-exact for counts / min / max / distinct value sets
    and keys, and for SUM / AVG sums of integer inputs (given `table`) while |sum| < 2^53 (the reference accumulates
    in double, exact below 2^53); `rel` relative tolerance for the other sums (north_star: 1e-9)."""
    assert set(a.rows) == set(b.rows), (sorted(a.rows)[:5], sorted(b.rows)[:5])
    for k in a.rows:
        for ag, x, y in zip(a.aggregations, a.rows[k], b.rows[k]):
            exact_sum = _integer_input(ag, table)
            if ag.function == "DISTINCTCOUNT":
                if isinstance(x, set) and isinstance(y, set):
                    assert x == y, (k, ag, len(x), len(y), sorted(x ^ y)[:5])
                else:
                    assert final_value(ag, x) == final_value(ag, y), (k, ag, x, y)
            elif ag.function == "AVG":
                assert x[1] == y[1], (k, ag, x, y)
                if exact_sum and abs(y[0]) < 2 ** 53:
                    assert x[0] == y[0], (k, ag, x, y)
                else:
                    assert _close(x[0], y[0], rel), (k, ag, x, y)
            elif ag.function in ("SUM",):
                if exact_sum and abs(y) < 2 ** 53:
                    assert x == y, (k, ag, x, y)
                else:
                    assert _close(x, y, rel), (k, ag, x, y)
            else:
                assert x == y, (k, ag, x, y)
    sa, sb = a.stats, b.stats
    assert sa.num_docs_scanned == sb.num_docs_scanned
    assert sa.num_entries_scanned_post_filter == sb.num_entries_scanned_post_filter
    assert sa.num_total_docs == sb.num_total_docs
