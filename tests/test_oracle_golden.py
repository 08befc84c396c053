"""Pin the CPU oracle (oracle/pinot_oracle.c) to the reference's own known answers (tests/golden/expected.json,
transcribed from pinot-core's query tests on the reference's test_data-sv.avro / simpleData200001.avro)."""
import os

import numpy as np
import pytest

from helpers import check_inner_values, check_rows, inner_query, run_rows, with_filter
from pinot_amd.plan import Table
from pinot_amd.query import parse
from pinot_amd.segment import ImmutableSegment


@pytest.mark.parametrize("i", range(2))
def test_inner_aggregation(i, expected, oracle_engine, sv_table_inner):
    case = expected["inner_aggregation"][i]
    res = oracle_engine.execute(sv_table_inner, inner_query(case, expected["filter"]))
    check_inner_values(res, case)


@pytest.mark.parametrize("i", range(8))
def test_inner_group_by(i, expected, oracle_engine, sv_table_inner):
    """ArrayBased / IntMap / LongMap / ArrayMap holders (cases 6-7: 9 keys whose cardinality product overflows a long)."""
    case = expected["inner_group_by"][i]
    res = oracle_engine.execute(sv_table_inner, inner_query(case, expected["filter"]))
    check_inner_values(res, case)


@pytest.mark.parametrize("i", range(3))
def test_inner_filtered_aggregation(i, expected, oracle_engine, sv_table_inner):
    """InnerSegmentAggregationSingleValueQueriesTest.testFilteredAggregations: FILTER clauses with IS NOT NULL
    (match-all without a null value vector) and the reference's pass statistics."""
    case = expected["inner_filtered_aggregation"][i]
    check_inner_values(oracle_engine.execute(sv_table_inner, case["query"]), case)


def test_inner_group_by_array_vs_map_holders(oracle_engine, sv_table_inner):
    """ArrayBased (card product <= 10 000) vs map-based holders give the same groups (DictionaryBasedGroupKeyGenerator)."""
    from oracle.oracle import OracleEngine
    q = "SELECT COUNT(*), SUM(column1) FROM testTable GROUP BY column11, column12"
    a = oracle_engine.execute(sv_table_inner, q)
    b = OracleEngine(array_based_threshold=1).execute(sv_table_inner, q)
    assert a.rows == b.rows


@pytest.mark.parametrize("i", range(24))
def test_inter_segment(i, expected, oracle_engine, sv_table_inter):
    cases = expected["inter"]
    if i >= len(cases):
        pytest.skip("no case")
    case = cases[i]
    q, res, rows = run_rows(oracle_engine, sv_table_inter, with_filter(case["query"], expected["filter"]))
    check_rows(rows, case["rows"], case.get("delta"))
    n_scanned, post, total = case["stats"]
    assert res.stats.num_docs_scanned == n_scanned
    assert res.stats.num_total_docs == total
    if post:  # 0 in the reference = answered from metadata / dictionary (no scan): the path still scans here
        assert res.stats.num_entries_scanned_post_filter == post


def test_query_executor_simple_data(expected, oracle_engine):
    """QueryExecutorTest.java:159-192: simpleData200001.avro as 2 segments."""
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "simple_data_200001.npz"))
    data = {k: z[k] for k in z.files}
    schema = {k: "INT" for k in z.files}
    seg = ImmutableSegment.create("simple", data, schema)
    t = Table("t", [seg, seg])
    e = expected["query_executor"]
    _, _, rows = run_rows(oracle_engine, t, "SELECT COUNT(*), SUM(met), MAX(met), MIN(met) FROM t")
    assert rows == [[e["count"], e["sum_met"], e["max_met"], e["min_met"]]]


def test_oracle_sees_filter_shortcuts(expected, sv_table_inner):
    """Predicate lowering on the reference's segment: column5 = 'gFuH' is always-true (card 1), daysSinceEpoch uses
    the sorted index, column11 NOT IN uses the inverted index (FilterOperatorUtils.getLeafFilterOperator :45-85)."""
    from pinot_amd import abi
    from pinot_amd.plan import CPlan
    q = parse("SELECT COUNT(*) FROM testTable" + expected["filter"])
    p = CPlan(sv_table_inner, q, sv_table_inner.segments, [1])
    kinds = {pred.column: lw.kind for pred, lw in zip(p.leaf_preds, p.lowered[0])}
    assert kinds["column5"] == abi.PG_LEAF_MATCH_ALL
    assert kinds["daysSinceEpoch"] == abi.PG_LEAF_SORTED
    assert kinds["column11"] == abi.PG_LEAF_INVERTED
    assert kinds["column1"] == abi.PG_LEAF_SV_SCAN
    assert kinds["column6"] == abi.PG_LEAF_SV_SCAN  # RANGE never uses the bitmap index


def test_ssb_synthetic_oracle_matches_numpy():
    """The oracle on a small config-3 (SSB Q1.1 shape) segment equals a direct numpy evaluation of the query."""
    import numpy as np
    from oracle.oracle import OracleEngine
    from pinot_amd import synth
    from pinot_amd.plan import Table
    from pinot_amd.query import parse
    n = 50_003
    seg = synth.make_segment_np(synth.SSB_LINEORDER, 0, n)
    v = {c.name: synth.values_np(c, 0, n) for c in synth.SSB_LINEORDER}
    m = ((v["lo_orderdate"] >= 8035) & (v["lo_orderdate"] <= 8399) & (v["lo_discount"] >= 1)
         & (v["lo_discount"] <= 3) & (v["lo_quantity"] < 25))
    want = float((v["lo_extendedprice"][m] * v["lo_discount"][m]).sum())
    r = OracleEngine(threads=1).execute(Table("lineorder", [seg]), parse(synth.ssb_q11_query()))
    assert r.stats.num_docs_scanned == int(m.sum())
    assert r.rows[()][0] == want


def test_baseball_oracle_matches_pandas():
    """Config 1 (synthetic baseballStats): the oracle's top-10 run scorers equal a pandas evaluation of the query."""
    import pandas as pd
    from oracle.oracle import OracleEngine
    from pinot_amd import synth
    from pinot_amd.plan import Table, reduce_to_rows
    seg = synth.baseball_segment(rows=20_011)
    df = pd.DataFrame({c: [seg.columns[c].dictionary.values[i] for i in seg.columns[c].dict_ids]
                       for c in ("playerName", "runs", "yearID")})
    for qi, sub in ((1, df), (3, df[df.yearID >= 2000])):
        q = parse(synth.BASEBALL_QUERIES[qi])
        rows = reduce_to_rows(q, OracleEngine().execute(Table("baseballStats", [seg]), q))[1]
        s = sub.groupby("playerName")["runs"].sum().reset_index()
        s = s.sort_values(["runs", "playerName"], ascending=[False, True]).head(10)
        assert rows == [[n, float(r)] for n, r in zip(s.playerName, s.runs)]
