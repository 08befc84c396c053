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
    from pinot_amd.plan import InstanceConfig
    q = "SELECT COUNT(*), SUM(column1) FROM testTable GROUP BY column11, column12"
    a = oracle_engine.execute(sv_table_inner, q)
    # max.init.group.holder.capacity = 1: every card product exceeds it, so the map-based holders run
    b = oracle_engine.execute(sv_table_inner, q, config=InstanceConfig(max_init_group_holder_capacity=1))
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


def _adanalytics_values(segs_n):
    import numpy as np
    from pinot_amd import synth
    cols = {c.name: [] for c in synth.ADANALYTICS}
    for s, n in segs_n:
        for c in synth.ADANALYTICS:
            cols[c.name].append(synth.values_np(c, s * n, n))
    return {k: np.concatenate(v) for k, v in cols.items()}


def test_adanalytics_lowering_pinned_by_numpy():
    """Config 2's SQL evaluated directly in numpy over the generator's values == the oracle over the lowered plan:
    pins plan.py's lowering (IN over a ~1 M-entry dictionary -> per-segment dictId sets, BETWEEN -> [lo, hi) on the
    sorted dictionary, NOT IN -> exclusive sets) independently of the pg_plan the GPU and the oracle share."""
    import numpy as np
    from oracle.oracle import OracleEngine
    from pinot_amd import synth
    from pinot_amd.plan import Table
    from pinot_amd.query import parse
    segs_n = [(0, 150_001), (7, 120_007)]
    segs = [synth.make_segment_np(synth.ADANALYTICS, s, n) for s, n in segs_n]
    v = _adanalytics_values(segs_n)
    t = Table("adAnalytics", segs)
    orc = OracleEngine()
    for num_ids in (1000, 20_000):
        ids = np.asarray([(i * 7919 + 13) % 1_000_000 for i in range(num_ids)])
        sql = synth.adanalytics_query(num_ids)
        for neg in (False, True):
            q = parse(sql.replace("accountId IN", "accountId NOT IN") if neg else sql)
            m = (v["daysSinceEpoch"] >= 18000) & (v["daysSinceEpoch"] <= 18089) & (np.isin(v["accountId"], ids) ^ neg)
            r = orc.execute(t, q)
            assert r.stats.num_docs_scanned == int(m.sum())
            days = np.unique(v["daysSinceEpoch"][m])
            want = {(int(d),): [float(v["clicks"][m & (v["daysSinceEpoch"] == d)].sum()),
                                float(v["impressions"][m & (v["daysSinceEpoch"] == d)].sum())] for d in days}
            assert r.rows == want, (num_ids, neg)
    # BETWEEN bounds that fall between dictionary values, and outside the value range
    for lo, hi in ((17899, 17905), (18263, 19000), (18000, 18000), (17000, 17800)):
        q = parse(f"SELECT COUNT(*), SUM(clicks) FROM adAnalytics WHERE daysSinceEpoch BETWEEN {lo} AND {hi}")
        m = (v["daysSinceEpoch"] >= lo) & (v["daysSinceEpoch"] <= hi)
        r = orc.execute(t, q)
        assert r.rows[()] == [int(m.sum()), float(v["clicks"][m].sum())], (lo, hi)


def test_index_path_lowering_pinned_by_numpy():
    """Config 5's SQL (sorted-index range, an OR of an inverted EQ and IN, an inverted NOT_EQ, an inverted IN of 2 000
    ids, COUNTMV) and variants with NOT IN / NOT BETWEEN / OR at the root, evaluated directly in numpy == the oracle
    over the lowered plan (sorted ranges, inverted dictId sets and the NOT_EQ flip pinned independently)."""
    import numpy as np
    from oracle.oracle import OracleEngine
    from pinot_amd import abi, synth
    from pinot_amd.plan import Table
    from pinot_amd.query import parse
    segs_n = [(0, 60_001), (5, 70_003)]
    segs = [synth.make_index_segment_np(s, n) for s, n in segs_n]
    vals = [synth.index_values_np(s, n) for s, n in segs_n]
    v = {k: np.concatenate([x[k] for x in vals]) for k in ("sortedCol", "inv1", "inv2", "inv3", "inv4")}
    nvals = np.concatenate([np.asarray([len(t) for t in x["mvTags"]]) for x in vals])
    t = Table("idx", segs)
    inv4 = np.asarray([i * 5 + 1 for i in range(2000)])
    inv2 = np.asarray([i * 5 for i in range(20)])
    rest = ((v["sortedCol"] >= 20000) & (v["sortedCol"] <= 59999) & ((v["inv1"] == 3) | np.isin(v["inv2"], inv2))
            & (v["inv3"] != 7))
    base = rest & np.isin(v["inv4"], inv4)
    ids = ", ".join(str(x) for x in inv4)
    cases = [(synth.index_query(), base),
             (synth.index_query().replace("inv4 IN", "inv4 NOT IN"), rest & ~np.isin(v["inv4"], inv4)),
             ("SELECT COUNT(*), COUNTMV(mvTags) FROM idx WHERE NOT sortedCol BETWEEN 1000 AND 98999 OR inv3 = 999",
              ~((v["sortedCol"] >= 1000) & (v["sortedCol"] <= 98999)) | (v["inv3"] == 999)),
             (f"SELECT COUNT(*), COUNTMV(mvTags) FROM idx WHERE sortedCol <> 50000 AND inv2 NOT IN (0, 1, 2) "
              f"AND inv4 IN ({ids})",
              (v["sortedCol"] != 50000) & ~np.isin(v["inv2"], [0, 1, 2]) & np.isin(v["inv4"], inv4))]
    orc = OracleEngine()
    for sql, m in cases:
        q = parse(sql)
        r = orc.execute(t, q)
        assert r.rows[()] == [int(m.sum()), int(nvals[m].sum())], sql[:120]
    # and the leaf operators the lowering chose (FilterOperatorUtils.getLeafFilterOperator)
    from pinot_amd.plan import CPlan
    p = CPlan(t, parse(synth.index_query()), segs, [1, 2])
    kinds = {pred.column: lw.kind for pred, lw in zip(p.leaf_preds, p.lowered[0])}
    assert kinds == {"sortedCol": abi.PG_LEAF_SORTED, "inv1": abi.PG_LEAF_INVERTED, "inv2": abi.PG_LEAF_INVERTED,
                     "inv3": abi.PG_LEAF_INVERTED, "inv4": abi.PG_LEAF_INVERTED}
