"""GROUP BY a multi-value column (DictionaryBasedGroupKeyGenerator.generateKeysForBlock(TransformBlock, int[][])
:188-200, getIntRawKeys :472-: a single MV column's raw keys are the doc's dictIds in stored order, SV keys folded in;
DefaultGroupByExecutor then calls aggregateGroupByMV, e.g. SumAggregationFunction.java:239-249): every matched doc
joins the group of each value in its list -- duplicates included -- with its own aggregation inputs, and COUNT counts
(doc, value) pairs.  Pinned against a Python restatement of that rule over the decoded values; the device against the
oracle.  Several MV keys group each tuple of the cartesian product of the doc's lists (getIntRawKeys :472-540; the
reference's own InnerSegmentAggregationMultiValueQueriesTest groups by column3, column6, column7: one SV and two MV
keys).  Under numGroupsLimit a segment keeps the keys seen first in (doc, key tuple) order.  Shapes the reference rejects
raise UnsupportedQuery: SV functions over MV columns (getXxxValuesSV) and COUNTMV
over SV columns."""
import numpy as np
import pytest

from pinot_amd.plan import InstanceConfig, Table, UnsupportedQuery, reduce_to_rows
from pinot_amd.query import parse
from pinot_amd.segment import ImmutableSegment


def _segments(n_segs=3, seed=11):
    rng = np.random.default_rng(seed)
    segs = []
    for s in range(n_segs):
        n = 3000 + 211 * s
        tags = [list(rng.integers(0, 25 + 3 * s, rng.integers(1, 6))) for _ in range(n)]
        tags[0] = [4, 4, 4]  # duplicates in one doc's list: three rows of group 4
        words = [[f"w{x}" for x in rng.integers(0, 9, rng.integers(1, 4))] for _ in range(n)]
        fm = [list(np.round(rng.normal(size=rng.integers(1, 4)) * 10, 3)) for _ in range(n)]
        data = {"tags": tags, "words": words, "k": rng.integers(0, 5, n), "v": rng.integers(-500, 500, n),
                "d": np.round(rng.normal(size=n) * 100, 2), "fm": fm}
        segs.append(ImmutableSegment.create(f"mv{s}", data, {"tags": "INT", "words": "STRING", "k": "INT", "v": "INT",
                                                            "d": "DOUBLE", "fm": "DOUBLE"}))
    return segs


@pytest.fixture(scope="module")
def mv_table():
    return Table("t", _segments())


QUERIES = [
    "SELECT tags, COUNT(*), SUM(v), MIN(d), MAX(v), AVG(d) FROM t GROUP BY tags",
    "SELECT k, tags, COUNT(*), SUM(d) FROM t WHERE v > -100 GROUP BY k, tags",
    "SELECT tags, k, DISTINCTCOUNT(v), COUNTMV(words) FROM t WHERE tags IN (3, 7) GROUP BY tags, k",
    "SELECT words, COUNT(*), SUM(v) FROM t WHERE d < 50 AND k <> 2 GROUP BY words",
    "SELECT tags, COUNTMV(tags), COUNT(*) FROM t WHERE words = 'w3' GROUP BY tags",
    "SELECT tags, SUM(v) FROM t GROUP BY tags ORDER BY SUM(v) DESC, tags LIMIT 5",
    # SUMMV / MINMV / MAXMV / AVGMV / DISTINCTCOUNTMV (*MVAggregationFunction: every value of the doc's list; AVGMV
    # counts values), aggregation-only, grouped, over the MV key's own column, ordered by an MV aggregation
    "SELECT SUMMV(tags), MINMV(tags), MAXMV(tags), AVGMV(tags), DISTINCTCOUNTMV(tags), COUNTMV(tags), COUNT(*) FROM t "
    "WHERE k < 3",
    "SELECT k, SUMMV(tags), AVGMV(fm), MAXMV(fm), MINMV(tags), SUMMV(fm) FROM t GROUP BY k",
    "SELECT tags, SUMMV(tags), AVGMV(tags), COUNT(*) FROM t WHERE v > 0 GROUP BY tags",
    "SELECT k, DISTINCTCOUNTMV(words), DISTINCTCOUNTMV(tags) FROM t WHERE d > -50 GROUP BY k",
    "SELECT MINMV(fm), MAXMV(tags), DISTINCTCOUNTMV(tags), AVGMV(fm) FROM t",
    "SELECT k, AVGMV(tags) FROM t GROUP BY k ORDER BY AVGMV(tags) DESC LIMIT 3",
    # several MV keys: one group per tuple of the product of the doc's lists (duplicates in a list kept)
    "SELECT tags, words, COUNT(*), SUM(v) FROM t GROUP BY tags, words",
    "SELECT k, words, tags, COUNT(*), MAX(d), SUMMV(fm), DISTINCTCOUNT(v) FROM t WHERE v < 200 GROUP BY k, words, tags",
    "SELECT words, fm, COUNT(*), AVG(v) FROM t WHERE tags IN (1, 2, 3) GROUP BY words, fm",
    "SELECT tags, k, words, SUM(v) FROM t GROUP BY tags, k, words ORDER BY SUM(v) DESC, tags, k, words LIMIT 6",
]


def _expected(table, sql, limit=None):
    """Python restatement: one row per (matched doc, tuple of the MV keys' lists) in doc / stored order (the lowest MV
    key outermost).  limit: numGroupsLimit -- per segment, a key not among the first `limit` keys seen in that order
    gets INVALID_ID and its rows are dropped (DictionaryBasedGroupKeyGenerator's map-based holders)."""
    q = parse(sql)
    rows = {}
    for seg in table.segments:
        cols = seg.columns
        seen = set()

        def val(c, i):
            col = cols[c]
            if col.single_value:
                return col.dictionary.values[col.dict_ids[i]]
            o = col.mv_offsets
            return [col.dictionary.values[j] for j in col.dict_ids[o[i]:o[i + 1]]]

        for i in range(seg.num_docs):
            if not _match(q.filter, lambda c: val(c, i)):
                continue
            keys = [()]
            for c in q.group_by:
                x = val(c, i)
                keys = [kk + (y,) for kk in keys for y in (x if isinstance(x, list) else [x])]
            for key in keys:
                key = tuple(y.item() if hasattr(y, "item") else y for y in key)
                if limit is not None and key not in seen:
                    if len(seen) >= limit:
                        continue
                    seen.add(key)
                r = rows.setdefault(key, [[] for _ in q.aggregations])
                for a, ag in enumerate(q.aggregations):
                    if ag.function == "COUNT":
                        r[a].append(1)
                    elif ag.function == "COUNTMV":
                        r[a].append(len(val(ag.arg.cols[0], i)))
                    elif ag.mv:  # SUMMV / MINMV / MAXMV / AVGMV / DISTINCTCOUNTMV: every value of the doc's list
                        r[a].extend(val(ag.arg.cols[0], i))
                    else:
                        r[a].append(val(ag.arg.cols[0], i))
    out = {}
    for key, lists in rows.items():
        row = []
        for ag, xs in zip(q.aggregations, lists):
            f = ag.function
            row.append(len(xs) if f == "COUNT" else sum(xs) if f in ("COUNTMV",) else float(np.sum(xs)) if f == "SUM"
                       else float(min(xs)) if f == "MIN" else float(max(xs)) if f == "MAX"
                       else (float(np.sum(xs)), len(xs)) if f == "AVG" else {getattr(y, "item", lambda: y)() for y in xs})
        out[key] = row
    return out


def _match(f, val):
    if f is None:
        return True
    if f.type == "AND":
        return all(_match(c, val) for c in f.children)
    if f.type == "OR":
        return any(_match(c, val) for c in f.children)
    if f.type == "NOT":
        return not _match(f.children[0], val)
    p = f.predicate
    x = val(p.column)
    xs = x if isinstance(x, list) else [x]
    conv = (lambda s: s) if isinstance(xs[0], str) else (lambda s: float(s))
    if p.type in ("EQ", "IN"):
        return any(y in [conv(v) for v in p.values] for y in xs)
    if p.type in ("NOT_EQ", "NOT_IN"):  # MV: every value outside the set (applyMV of the exclusive evaluator)
        return all(y not in [conv(v) for v in p.values] for y in xs)
    ok = lambda y: ((p.lower == "*" or (y >= conv(p.lower) if p.lower_inclusive else y > conv(p.lower))) and
                    (p.upper == "*" or (y <= conv(p.upper) if p.upper_inclusive else y < conv(p.upper))))
    return any(ok(y) for y in xs)


@pytest.mark.parametrize("sql", QUERIES)
def test_oracle_mv_group_by_matches_the_restatement(sql, mv_table, oracle_engine):
    q = parse(sql)
    got = oracle_engine.execute(mv_table, q)
    want = _expected(mv_table, sql)
    assert set(got.rows) == set(want)
    for key, row in want.items():
        for ag, g, w in zip(q.aggregations, got.rows[key], row):
            if ag.function == "AVG":
                assert g[1] == w[1] and np.isclose(g[0], w[0], rtol=1e-12)
            elif isinstance(w, float):
                assert np.isclose(g, w, rtol=1e-12, atol=1e-9), (key, ag, g, w)
            else:
                assert g == w, (key, ag, g, w)
    assert got.stats.num_docs_scanned == sum(
        1 for s in mv_table.segments for i in range(s.num_docs)
        if _match(q.filter, lambda c, s=s, i=i: _col_val(s, c, i)))


def _col_val(seg, c, i):
    col = seg.columns[c]
    if col.single_value:
        return col.dictionary.values[col.dict_ids[i]]
    o = col.mv_offsets
    return [col.dictionary.values[j] for j in col.dict_ids[o[i]:o[i + 1]]]


def test_plan_keys_carry_the_key_spaces(mv_table):
    """The pg_key of every group-by column carries its table-global key space (kind, cardinality, base)."""
    from pinot_amd.plan import CPlan
    p = CPlan(mv_table, parse("SELECT k, tags, COUNT(*) FROM t GROUP BY k, tags"), mv_table.segments, [1, 2, 3])
    for i, c in enumerate(("k", "tags")):
        ks = mv_table.key_space(c)
        assert (p.plan.keys[i].kind, p.plan.keys[i].cardinality, p.plan.keys[i].base) == \
            (ks.kind, ks.cardinality, ks.base) and ks.cardinality > 0


def test_mv_function_names():
    """SumMV's names: getColumnName "sumMV_tags", getResultColumnName "summv(tags)" (the type name lower-cased)."""
    from pinot_amd import datatable as dtm
    ag = parse("SELECT SUMMV(tags), DISTINCTCOUNTMV(words) FROM t").aggregations
    assert (ag[0].function, ag[0].mv, ag[0].name) == ("SUM", True, "SUMMV")
    assert dtm.column_name(ag[0]) == "sumMV_tags" and dtm.result_column_name(ag[0]) == "summv(tags)"
    assert dtm.column_name(ag[1]) == "distinctCountMV_words" and ag[0] != parse("SELECT SUM(tags) FROM t").aggregations[0]


@pytest.mark.parametrize("sql", [
    "SELECT k, SUMMV(v) FROM t GROUP BY k",                        # an MV function over an SV column
    "SELECT k, SUM(tags) FROM t GROUP BY k",                       # an SV function over an MV column
    "SELECT COUNTMV(v) FROM t",                                     # COUNTMV over an SV column
    "SELECT DISTINCTCOUNT(tags) FROM t",
])
def test_unrestated_mv_shapes_are_unsupported(sql, mv_table, oracle_engine):
    with pytest.raises(UnsupportedQuery):
        oracle_engine.execute(mv_table, parse(sql))


@pytest.mark.gpu
@pytest.mark.parametrize("sql", QUERIES)
def test_mv_group_by_on_device(sql, mv_table, gpu_engine, oracle_engine):
    from helpers import assert_same_result
    q = parse(sql)
    g, o = gpu_engine.execute(mv_table, q), oracle_engine.execute(mv_table, q)
    assert_same_result(g, o, table=mv_table)
    if q.order_by:
        assert reduce_to_rows(q, g) == reduce_to_rows(q, o)


TRUNCATING = [
    ("SELECT tags, COUNT(*), SUM(v) FROM t GROUP BY tags", 10),
    ("SELECT k, tags, COUNT(*), MAX(d) FROM t WHERE v > -200 GROUP BY k, tags", 30),
    ("SELECT tags, words, COUNT(*), SUM(v) FROM t GROUP BY tags, words", 40),
    ("SELECT k, words, tags, COUNT(*) FROM t GROUP BY k, words, tags", 100),
]


@pytest.mark.parametrize("sql,limit", TRUNCATING)
def test_oracle_mv_truncation_is_first_seen(sql, limit, mv_table, oracle_engine):
    """numGroupsLimit with multi-value keys: group ids go to keys in first-seen (doc, key tuple) order per segment."""
    q = parse(sql)
    got = oracle_engine.execute(mv_table, q, config=InstanceConfig.with_groups_limit(limit))
    want = _expected(mv_table, sql, limit=limit)
    assert set(got.rows) == set(want) and got.groups_limit_reached
    for key, row in want.items():
        for ag, g, w in zip(q.aggregations, got.rows[key], row):
            assert (np.isclose(g, w, rtol=1e-12, atol=1e-9) if isinstance(w, float) else g == w), (key, ag, g, w)


@pytest.mark.gpu
@pytest.mark.parametrize("sql,limit", TRUNCATING)
def test_mv_group_by_truncation_on_device(sql, limit, mv_table, gpu_engine, oracle_engine):
    """The device's per-segment table orders each (segment, key) by its first (doc, tuple position) sighting."""
    from helpers import assert_same_result
    cfg = InstanceConfig.with_groups_limit(limit)
    q = parse(sql)
    g, o = gpu_engine.execute(mv_table, q, config=cfg), oracle_engine.execute(mv_table, q, config=cfg)
    assert_same_result(g, o, table=mv_table)
    assert g.groups_limit_reached == o.groups_limit_reached
