"""Parity of the HIP path (libpinot_gpu.so through the C ABI) with the CPU oracle and the reference's known answers.

Bar (north_star): bit-exact for COUNT, MIN, MAX, integer SUM, DISTINCTCOUNT and group keys; 1e-9 relative for
double SUM / AVG sums.  Every test here runs on an MI355X (`-m gpu`)."""
import numpy as np
import pytest

from helpers import assert_same_result, check_inner_values, check_rows, inner_query, run_rows, with_filter
from pinot_amd.plan import MAX_TRIM_THRESHOLD, InstanceConfig, Table, UnsupportedQuery, reduce_to_rows
from pinot_amd.query import parse
from pinot_amd.segment import ImmutableSegment

pytestmark = pytest.mark.gpu


# ------------------------------------------------------------------ reference known answers (test_data-sv.avro)

@pytest.mark.parametrize("i", range(2))
def test_golden_inner_aggregation(i, expected, gpu_engine, sv_table_inner):
    case = expected["inner_aggregation"][i]
    res = gpu_engine.execute(sv_table_inner, inner_query(case, expected["filter"]))
    check_inner_values(res, case)


@pytest.mark.parametrize("i", range(8))
def test_golden_inner_group_by(i, expected, gpu_engine, sv_table_inner):
    """Cases 6-7 are the reference's ArrayMapBasedHolder answers (9 keys): the device tuple table of pg_wide.hip."""
    case = expected["inner_group_by"][i]
    res = gpu_engine.execute(sv_table_inner, inner_query(case, expected["filter"]))
    check_inner_values(res, case)


@pytest.mark.parametrize("i", range(3))
def test_golden_inner_filtered_aggregation(i, expected, gpu_engine, sv_table_inner):
    """testFilteredAggregations (IS NOT NULL filters) through one device plan per filter."""
    case = expected["inner_filtered_aggregation"][i]
    check_inner_values(gpu_engine.execute(sv_table_inner, case["query"]), case)


@pytest.mark.parametrize("i", range(24))
def test_golden_inter_segment(i, expected, gpu_engine, sv_table_inter):
    cases = expected["inter"]
    if i >= len(cases):
        pytest.skip("no case")
    case = cases[i]
    q, res, rows = run_rows(gpu_engine, sv_table_inter, with_filter(case["query"], expected["filter"]))
    check_rows(rows, case["rows"], case.get("delta"))
    n_scanned, post, total = case["stats"]
    assert res.stats.num_docs_scanned == n_scanned
    assert res.stats.num_total_docs == total


# ------------------------------------------------------------------ device vs oracle, same inputs

SV_QUERIES = [
    "SELECT COUNT(*) FROM t",
    "SELECT COUNT(*), SUM(column1), MIN(column3), MAX(column6), AVG(column7) FROM t",
    "SELECT SUM(column1), SUM(column3) FROM t WHERE column6 < 500000000",
    "SELECT COUNT(*) FROM t WHERE column11 IN ('P', 'o') AND column17 <> 5",
    "SELECT COUNT(*), MAX(column18) FROM t WHERE NOT column11 = 'P'",
    "SELECT COUNT(*) FROM t WHERE column7 IN (1, 2, 3, 4, 5, 6, 7, 8, 9, 10) OR column9 > 1000000000",
    "SELECT MIN(column1), MAX(column1) FROM t WHERE daysSinceEpoch = 126164076",
    "SELECT COUNT(*) FROM t WHERE daysSinceEpoch <> 126164076",
    "SELECT COUNT(*) FROM t WHERE column1 > 3000000000",
    "SELECT COUNT(*) FROM t WHERE column5 = 'nope'",
    "SELECT DISTINCTCOUNT(column1), DISTINCTCOUNT(column11), DISTINCTCOUNT(column12) FROM t WHERE column3 > 1000000000",
    "SELECT SUM(column1 * column3), SUM(column7 + column17), SUM(column7 - column18) FROM t",
    "SELECT MIN(column6 * column7), MAX(column17 - column18), AVG(column1 * column17) FROM t WHERE column6 > 10",
    "SELECT column11, COUNT(*), SUM(column1), MIN(column3), MAX(column3), AVG(column9) FROM t GROUP BY column11",
    "SELECT column11, column12, SUM(column1) FROM t GROUP BY column11, column12",
    "SELECT column9, COUNT(*) FROM t GROUP BY column9",
    "SELECT daysSinceEpoch, column17, SUM(column18) FROM t WHERE column11 NOT IN ('t', 'P') GROUP BY daysSinceEpoch, column17",
    "SELECT column12, DISTINCTCOUNT(column11), DISTINCTCOUNT(column7) FROM t GROUP BY column12",
    "SELECT column7, COUNT(*), SUM(column3) FROM t WHERE (column6 < 500000000 OR column11 NOT IN ('t', 'P')) AND "
    "NOT (column17 IN (1, 2) AND column18 > 100) GROUP BY column7",
]


@pytest.mark.parametrize("sql", SV_QUERIES)
def test_sv_queries_match_oracle(sql, gpu_engine, oracle_engine, sv_table_inter):
    q = parse(sql)
    g = gpu_engine.execute(sv_table_inter, q)
    o = oracle_engine.execute(sv_table_inter, q)
    assert_same_result(g, o, table=sv_table_inter)


@pytest.mark.parametrize("mode", ["0", "1"])
def test_streaming_prefilter_on_and_off(mode, monkeypatch, gpu_engine, oracle_engine, sv_table_inter):
    """The same filters with the root AND's leaves folded into the streaming pre-filter (pg_filter.hip, forced on)
    and evaluated by the fused scan alone (off): identical results and scan statistics."""
    monkeypatch.setenv("PG_PREFILTER", mode)
    for sql in [q for q in SV_QUERIES if "WHERE" in q] + [
            "SELECT column9, SUM(column1), COUNT(*) FROM t WHERE column7 IN (1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12) "
            "AND column3 > 1000000 AND column17 NOT IN (5, 7) GROUP BY column9",
            "SELECT COUNT(*), SUM(column3) FROM t WHERE daysSinceEpoch = 126164076 AND column6 < 900000000"]:
        q = parse(sql)
        assert_same_result(gpu_engine.execute(sv_table_inter, q), oracle_engine.execute(sv_table_inter, q),
                           table=sv_table_inter)


def test_unsupported_shape_is_reported_not_crashed(gpu_engine, sv_table_inner):
    """More aggregations than the device path takes -> PG_E_UNSUPPORTED (the caller falls back to the CPU plan)."""
    with pytest.raises(UnsupportedQuery):
        gpu_engine.execute(sv_table_inner, "SELECT COUNT(*), SUM(column1), SUM(column3), SUM(column6), SUM(column7), "
                                           "SUM(column9), SUM(column17), SUM(column18), MAX(column1) FROM t")


WIDE_KEYS = "column1, column3, column5, column6, column7, column9, column11, column12, column17"
WIDE_QUERIES = [
    f"SELECT COUNT(*), SUM(column18), MIN(column6), MAX(column3), AVG(column7) FROM t GROUP BY {WIDE_KEYS}",
    f"SELECT COUNT(*), SUM(column1) FROM t WHERE column3 > 1000000000 AND column11 <> 'P' GROUP BY {WIDE_KEYS}, "
    "column18, daysSinceEpoch",
    f"SELECT DISTINCTCOUNT(column11), COUNT(*) FROM t WHERE column6 < 900000000 GROUP BY column1, column3, column6, "
    "column7, column9",
]


@pytest.mark.parametrize("sql", WIDE_QUERIES)
def test_wide_group_keys_match_oracle(sql, gpu_engine, oracle_engine, sv_table_inter):
    """Group keys whose packed key exceeds 62 bits or that number more than 8 (ArrayMapBasedHolder,
    DictionaryBasedGroupKeyGenerator.java:777-): device tuple interning over 4 segments merged by value, dense and hash
    group states, the ORDER BY on the device (by an aggregation) and on the host (by a key)."""
    from pinot_amd import abi
    q = parse(sql)
    o = oracle_engine.execute(sv_table_inter, q)
    assert_same_result(gpu_engine.execute(sv_table_inter, q), o, table=sv_table_inter)
    assert_same_result(gpu_engine.execute(sv_table_inter, q, flags=abi.PG_PLAN_VALUE_SETS | abi.PG_PLAN_HASH_GROUPS), o,
                       table=sv_table_inter)
    for order in ("ORDER BY COUNT(*) DESC, column1, column3, column6 LIMIT 7", "ORDER BY column3 DESC, column1 LIMIT 9"):
        q2 = parse(sql.replace("SELECT ", "SELECT column1, column3, column6, ") + " " + order)
        assert reduce_to_rows(q2, gpu_engine.execute(sv_table_inter, q2, trim=True))[1] == \
            reduce_to_rows(q2, oracle_engine.execute(sv_table_inter, q2))[1]


@pytest.mark.parametrize("limit", [1, 500, 29000])
def test_wide_group_keys_num_groups_limit(limit, gpu_engine, oracle_engine, sv_table_inter):
    """The instance's numGroupsLimit with the ArrayMapBasedHolder: per segment the first `limit` tuples in doc order
    (getGroupId :812-819), then the value-keyed merge; numGroupsLimitReached as the oracle reports it."""
    q = parse(f"SELECT COUNT(*), SUM(column1) FROM t GROUP BY {WIDE_KEYS}")
    cfg = InstanceConfig.with_groups_limit(limit)
    g, o = gpu_engine.execute(sv_table_inter, q, config=cfg), oracle_engine.execute(sv_table_inter, q, config=cfg)
    assert_same_result(g, o, table=sv_table_inter)
    assert g.groups_limit_reached == o.groups_limit_reached


GROUP_QUERIES = [q for q in SV_QUERIES if "GROUP BY" in q] + [
    "SELECT column1, column6, column9, column11, column12, COUNT(*), SUM(column1), MAX(column3), MIN(column6), "
    "AVG(column7) FROM t GROUP BY column1, column6, column9, column11, column12",
    "SELECT column9, DISTINCTCOUNT(column1), SUM(column17) FROM t WHERE column3 > 1000000000 GROUP BY column9",
]


@pytest.mark.parametrize("sql", GROUP_QUERIES)
def test_group_by_hash_table_matches_oracle(sql, gpu_engine, oracle_engine, sv_table_inter):
    """The same group-bys through the device hash table (IntGroupIdMap / Long2IntOpenHashMap on the device) instead of
    direct addressing: identical results."""
    from pinot_amd import abi
    q = parse(sql)
    g = gpu_engine.execute(sv_table_inter, q, flags=abi.PG_PLAN_VALUE_SETS | abi.PG_PLAN_HASH_GROUPS)
    assert_same_result(g, oracle_engine.execute(sv_table_inter, q), table=sv_table_inter)


@pytest.mark.parametrize("limit", [1, 37, 500, 1736, 1737])
def test_num_groups_limit_truncation(limit, gpu_engine, oracle_engine):
    """The instance's numGroupsLimit below the segment's distinct keys: each segment keeps the keys it sees first (doc
    order) and drops the docs of later keys (IntGroupIdMap.getGroupId, DictionaryBasedGroupKeyGenerator.java:991-1016);
    the segments then merge by value.  Segments hold different data so their kept key sets differ.  The result
    reports numGroupsLimitReached exactly when a segment holds >= limit keys (AggregationGroupByOrderByOperator
    .java:112-113); an OPTION(numGroupsLimit=...) in the SQL is ignored, as Pinot 0.11 ignores it."""
    rng = np.random.default_rng(limit)
    segs = []
    for s_ in range(3):
        n = 20000 + 1111 * s_
        data = {"k": rng.integers(0, 2000, n), "k2": rng.integers(0, 3, n), "v": rng.integers(-10 ** 6, 10 ** 6, n),
                "d": rng.normal(size=n), "u": rng.integers(0, 300, n)}
        segs.append(_seg(f"t{s_}", data, {"k": "INT", "k2": "INT", "v": "LONG", "d": "DOUBLE", "u": "INT"}))
    t = Table("t", segs)
    for sql in ["SELECT k, COUNT(*), SUM(v), MIN(d), MAX(v), AVG(d), DISTINCTCOUNT(u) FROM t GROUP BY k",
                "SELECT k2, k, SUM(v) FROM t WHERE v > 0 GROUP BY k2, k"]:
        q = parse(sql)
        cfg = InstanceConfig.with_groups_limit(limit)
        g, o = gpu_engine.execute(t, q, config=cfg), oracle_engine.execute(t, q, config=cfg)
        assert_same_result(g, o, table=t)
        assert len(g.rows) <= 3 * limit
        assert g.groups_limit_reached == o.groups_limit_reached
        q_opt = parse(sql + " OPTION(numGroupsLimit=10000000)")   # not an instance setting: no effect
        assert_same_result(gpu_engine.execute(t, q_opt, config=cfg), o, table=t)


@pytest.mark.parametrize("select", ["0", "1"])
def test_order_by_trim_on_device(select, monkeypatch, gpu_engine, oracle_engine, sv_table_inter):
    """ORDER BY ... LIMIT applied on the device (TableResizer.getTopRecords): the kept candidates (boundary ties
    included) give the reference's top rows -- by a sort of every group's order key (PG_TRIM_SELECT=0) and by the
    radix select of the limit-th key (=1; by default from 65 536 groups)."""
    monkeypatch.setenv("PG_TRIM_SELECT", select)
    for sql in ["SELECT column9, SUM(column1) FROM t GROUP BY column9 ORDER BY SUM(column1) DESC, column9 LIMIT 7",
                "SELECT column11, column12, AVG(column3), COUNT(*) FROM t GROUP BY column11, column12 "
                "ORDER BY AVG(column3), column12 DESC, column11 LIMIT 5",
                "SELECT column12, DISTINCTCOUNT(column7) FROM t GROUP BY column12 ORDER BY DISTINCTCOUNT(column7) DESC, "
                "column12 LIMIT 3",
                "SELECT column1, column6, COUNT(*) FROM t GROUP BY column1, column6 ORDER BY COUNT(*) DESC, column1, "
                "column6 LIMIT 10"]:
        q = parse(sql)
        g = gpu_engine.execute(sv_table_inter, q, trim=True)
        o = oracle_engine.execute(sv_table_inter, q)
        assert reduce_to_rows(q, g)[1] == reduce_to_rows(q, o)[1], sql
        assert len(g.rows) <= len(o.rows)


def test_config4_shape_high_cardinality_distinctcount(gpu_engine, oracle_engine):
    """Config 4 in miniature: userId of high cardinality x itemId 1 000, DISTINCTCOUNT per user, ORDER BY DISTINCTCOUNT
    DESC, userId LIMIT 100, with an instance numGroupsLimit above the distinct users (as the reference must be run);
    plus the same under a 40 000 limit, which truncates per segment."""
    from pinot_amd import synth
    segs = [synth.make_segment_np(synth.highcard_specs(users=150_000), s, 200_003) for s in range(3)]
    t = Table("events", segs)
    for sql, cfg in [(synth.highcard_query(), InstanceConfig(num_groups_limit=10_000_000)),
                     (synth.highcard_query().replace("LIMIT 100", "LIMIT 20"), InstanceConfig(num_groups_limit=40_000))]:
        q = parse(sql)
        g = gpu_engine.execute(t, q, trim=True, config=cfg)
        o = oracle_engine.execute(t, q, config=cfg)
        assert reduce_to_rows(q, g)[1] == reduce_to_rows(q, o)[1]
        full = gpu_engine.execute(t, q, config=cfg)
        assert_same_result(full, o, table=t)
        assert full.groups_limit_reached == o.groups_limit_reached == (cfg.num_groups_limit == 40_000)


@pytest.mark.parametrize("mode", ["0", "1"])
def test_radix_partitioned_group_by(mode, monkeypatch, gpu_engine, oracle_engine):
    """Dense group-by through the radix-partitioned pipeline (pg_part.hip: count pass, scatter pass, level 2, LDS
    buckets; PG_PART=1 forces it below its state-size threshold) and through per-doc state updates (PG_PART=0):
    identical to the oracle -- DISTINCTCOUNT value sets, COUNTs, the trimmed top rows, filters, ragged segments."""
    from pinot_amd import abi, synth
    monkeypatch.setenv("PG_PART", mode)
    segs = [synth.make_segment_np(synth.highcard_specs(users=150_000), s, 200_003 + 977 * s) for s in range(3)]
    t = Table("events", segs)
    cfg = InstanceConfig(num_groups_limit=10_000_000)
    for sql in [synth.highcard_query(),
                "SELECT userId, COUNT(*), DISTINCTCOUNT(itemId), COUNT(*) FROM events WHERE itemId < 700 "
                "GROUP BY userId",
                "SELECT itemId, COUNT(*) FROM events WHERE userId BETWEEN 1000 AND 90000 GROUP BY itemId",
                "SELECT userId, COUNT(*) FROM events GROUP BY userId ORDER BY COUNT(*) DESC, userId LIMIT 10"]:
        q = parse(sql)
        o = oracle_engine.execute(t, q, config=cfg)
        assert_same_result(gpu_engine.execute(t, q, flags=abi.PG_PLAN_VALUE_SETS, config=cfg), o, table=t)
        if q.order_by:
            assert reduce_to_rows(q, gpu_engine.execute(t, q, trim=True, config=cfg))[1] == reduce_to_rows(q, o)[1]
            # the trim of a DISTINCTCOUNT-ordered state from its set-size histogram (finalize_core step 0) and the
            # general order-image radix select give the same server rows
            srv = gpu_engine.execute(t, q, trim="server", config=cfg)
            monkeypatch.setenv("PG_TRIM_POP", "0")
            gen = gpu_engine.execute(t, q, trim="server", config=cfg)
            monkeypatch.delenv("PG_TRIM_POP")
            assert srv.rows == gen.rows


def _skewed_events(seed: int, n: int, users: int, hot: int, items_scale: int = 1):
    """Events whose userIds crowd into the first `hot` ids for 90 % of the docs (a level-1 partition far over its
    uniform share), itemIds spread over [0, 1000) * items_scale."""
    rng = np.random.default_rng(seed)
    u = np.where(rng.random(n) < 0.9, rng.integers(0, hot, n), rng.integers(0, users, n)).astype(np.int64)
    i = (rng.integers(0, 1000, n) * items_scale).astype(np.int64)
    return {"userId": u, "itemId": i}


@pytest.mark.parametrize("case", ["skewed", "keymap"])
def test_radix_partitioned_speculative_regions(case, monkeypatch, gpu_engine, oracle_engine):
    """The speculative level-1 / level-2 regions of the radix-partitioned group-by (part_direct + part_split2s): a
    skewed key distribution overflows a region and the query reruns with exact offsets; sparse userIds (a keymap key
    space) with non-identity itemIds (dictionary gathers) take the gather modes.  Both identical to the oracle."""
    from pinot_amd import abi
    from pinot_amd.segment import ImmutableSegment
    monkeypatch.setenv("PG_PART", "1")
    types = {"userId": "INT", "itemId": "INT"}
    segs = []
    for s in range(3):
        if case == "skewed":
            data = _skewed_events(s, 300_007 + 13 * s, users=150_000, hot=700)
        else:
            data = _skewed_events(s, 200_003, users=60_000, hot=60_000, items_scale=7)
            data["userId"] = data["userId"] * 97 + 11  # span far above 4x the cardinality: a keymap key space
        segs.append(ImmutableSegment.create(f"ev{s}", data, types))
    t = Table("events", segs)
    if case == "keymap":
        assert t.key_space("userId").kind == abi.PG_KEY_KEYMAP
    cfg = InstanceConfig(num_groups_limit=10_000_000)
    for sql in [synth_highcard(),
                "SELECT userId, COUNT(*) FROM events GROUP BY userId ORDER BY COUNT(*) DESC, userId LIMIT 10"]:
        q = parse(sql)
        o = oracle_engine.execute(t, q, config=cfg)
        assert_same_result(gpu_engine.execute(t, q, flags=abi.PG_PLAN_VALUE_SETS, config=cfg), o, table=t)
        assert reduce_to_rows(q, gpu_engine.execute(t, q, trim=True, config=cfg))[1] == reduce_to_rows(q, o)[1]
    monkeypatch.setenv("PG_PART_SPEC", "0")  # the exact-offset pipeline on the same data
    q = parse(synth_highcard())
    assert_same_result(gpu_engine.execute(t, q, flags=abi.PG_PLAN_VALUE_SETS, config=cfg),
                       oracle_engine.execute(t, q, config=cfg), table=t)


def synth_highcard():
    from pinot_amd import synth
    return synth.highcard_query()


def test_config4_full_segments_match_oracle(gpu_engine, oracle_engine):
    """Config 4 at its stated scale: 4 full 7 812 500-row segments of the 10 M-user key space (device-generated, as the
    bench), every group's DISTINCTCOUNT and COUNT-free result through the radix-partitioned pipeline against the
    oracle's per-segment value sets merged by value, and the device-trimmed top 100 (ORDER BY DISTINCTCOUNT DESC,
    userId) against the oracle's.  The instance is configured as SURVEY §8(d) states the reference must be run:
    num.groups.limit 10 M (above the ~5.4 M users of a segment) and groupby.trim.threshold at MAX_TRIM_THRESHOLD (no
    lossy resize during the merge); at the default threshold (1 M) the result reports that the reference server would
    have resized its table mid-merge."""
    import torch
    from pinot_amd import abi, synth
    from pinot_amd.plan import CPlan
    dev = torch.device("cuda", 0)
    rows = synth.ADANALYTICS_ROWS_PER_SEGMENT
    segs, host = [], []
    table = None
    for si in range(4):
        dcs = synth.make_columns_torch(synth.HIGHCARD, si, rows, dev)
        seg = ImmutableSegment(f"ev_{si}", rows, {dc.spec.name: dc.meta_column() for dc in dcs})
        host.append(ImmutableSegment(f"ev_{si}", rows, {dc.spec.name: dc.host_column() for dc in dcs}))
        if table is None:
            table = Table("events", [seg])
        gpu_engine.register_device_segment(seg, table, dcs)
        segs.append(seg)
        del dcs
    t = Table("events", segs)
    q = parse(synth.highcard_query())
    cfg = InstanceConfig(num_groups_limit=10_000_000, groupby_trim_threshold=MAX_TRIM_THRESHOLD)
    # oracle: per-segment (user, item) value sets merged by value
    ht = Table("events", host)
    cp = CPlan(ht, q, host, list(range(1, len(host) + 1)), config=cfg)
    pk, pv = zip(*(oracle_engine.distinct_pairs(cp, i, sg) for i, sg in enumerate(host)))
    pair = np.unique(np.concatenate(pk) * (1 << 20) + np.concatenate(pv))
    users, counts = np.unique(pair >> 20, return_counts=True)
    # device: every group (keys, distinct counts) from the partial state
    plan = gpu_engine.make_plan(t, q, flags=0, config=cfg)
    ra = gpu_engine.finalize_arrays(plan, gpu_engine.run_partial(plan))
    ks = plan.key_spaces[0]
    assert ks.kind == abi.PG_KEY_VALUE_OFFSET
    gk = ra["keys"][:, 0].astype(np.int64) + ks.base
    order = np.argsort(gk)
    assert np.array_equal(gk[order], users)
    assert np.array_equal(ra["values"][order, 0].astype(np.int64), counts)
    assert ra["stats"][0] == 4 * rows
    # device-trimmed top rows (pg_execute: the bucket pass's set sizes feed the trim)
    top = np.lexsort((users, -counts))[:q.limit]
    want = [[int(users[i]), int(counts[i])] for i in top]
    assert reduce_to_rows(q, gpu_engine.execute(t, q, flags=0, trim=True, config=cfg))[1] == want
    # the server's result (GroupByOrderByCombineOperator: getTableCapacity(100, minServerGroupTrimSize = 5 000) rows
    # under the ORDER BY; the ORDER BY ends in the key, so the kept set is determined; no mid-merge resize under this
    # instance config): exactly the oracle's top 5 000
    srv = gpu_engine.execute(t, q, flags=0, trim="server", config=cfg)
    top = np.lexsort((users, -counts))[:5000]
    assert len(srv.rows) == 5000
    assert not srv.trim_threshold_reached and not srv.groups_limit_reached
    assert srv.num_groups_merged == len(users)
    # two segments under the default groupby.trim.threshold (1 M): the ~8 M merged users would have made the reference's
    # ConcurrentIndexedTable resize mid-merge (lossy); the device merges exactly and reports it.  Raised: no resize.
    two_users = np.unique(np.concatenate(pk[:2])).size
    for c2, hit in ((InstanceConfig(num_groups_limit=10_000_000), True), (cfg, False)):
        r2 = gpu_engine.execute(t, q, segments=segs[:2], flags=0, trim="server", config=c2)
        assert r2.trim_threshold_reached == hit and r2.num_groups_merged == two_users > 1_000_000
        assert len(r2.rows) == 5000
    assert sorted(k[0] for k in srv.rows) == sorted(users[top].tolist())
    ku = np.asarray([k[0] for k in srv.rows], dtype=np.int64)
    assert np.array_equal(np.asarray([v[0] for v in srv.rows.values()]), counts[np.searchsorted(users, ku)])
    for seg in segs:
        gpu_engine.release(seg)


@pytest.mark.parametrize("dtype", ["INT", "LONG", "FLOAT", "DOUBLE"])
def test_dict_id_sets_on_device(dtype, gpu_engine, oracle_engine):
    """pg_dict_id_sets (IN / NOT_IN literals looked up in every segment's resident dictionary in one launch) gives
    PredicateUtils.getDictIdSet's per-segment dictIds (plan.dict_id_set on the host); the queries through it match
    the oracle."""
    from pinot_amd.plan import dict_id_set, _coerced_literals
    rng = np.random.default_rng(7)
    segs = []
    for s in range(5):  # different dictionaries per segment (absent literals, ragged sizes)
        n = 20_011 + 3_001 * s
        v = rng.integers(-5_000, 5_000, n) * (3 if dtype in ("INT", "LONG") else 1)
        data = {"k": v.astype(np.int64) if dtype in ("INT", "LONG") else v.astype(np.float64) / 4,
                "m": rng.integers(0, 100, n).astype(np.int64)}
        segs.append(ImmutableSegment.create(f"d{s}", data, {"k": dtype, "m": "INT"}))
    t = Table("t", segs)
    lits = [x * 3 for x in range(-300, 300, 7)] if dtype in ("INT", "LONG") else [x / 4 for x in range(-900, 900, 11)]
    keys = [gpu_engine.upload_segment(s, t) for s in segs]
    d0 = segs[0].columns["k"].dictionary
    ids, counts = gpu_engine.dict_id_sets(t.column_ids["k"], dtype, _coerced_literals(d0, lits), keys)
    for si, s in enumerate(segs):
        want = dict_id_set(s.columns["k"].dictionary, lits)
        assert np.array_equal(ids[si, :counts[si]], want), si
    in_list = ", ".join(str(x) for x in lits)
    for sql in [f"SELECT COUNT(*), SUM(m) FROM t WHERE k IN ({in_list})",
                f"SELECT m, COUNT(*) FROM t WHERE k NOT IN ({in_list}) GROUP BY m"]:
        q = parse(sql)
        assert_same_result(gpu_engine.execute(t, q), oracle_engine.execute(t, q), table=t)
    if dtype in ("FLOAT", "DOUBLE"):
        # NaN / +-inf literals and a dictionary with infinite bounds: the lookup's interpolation step stays defined
        # (finite span, 0 <= f <= 1) and the binary search finds exactly what the host finds
        odd = [float("nan"), float("inf"), float("-inf"), 0.25, -1250.0]
        inf_seg = ImmutableSegment.create("dinf", {"k": np.asarray([-np.inf, -3.5, 0.25, 7.0, np.inf] * 1000),
                                                  "m": np.arange(5000, dtype=np.int64) % 7}, {"k": dtype, "m": "INT"})
        t2 = Table("t", segs[:2] + [inf_seg])
        keys2 = [gpu_engine.upload_segment(s, t2) for s in t2.segments]
        lit = np.asarray(sorted(x for x in odd if x == x) + [float("nan")])
        ids2, counts2 = gpu_engine.dict_id_sets(t2.column_ids["k"], dtype, lit, keys2)
        for si, s in enumerate(t2.segments):
            assert np.array_equal(ids2[si, :counts2[si]], dict_id_set(s.columns["k"].dictionary, list(lit))), si


def test_dict_id_sets_concurrent_with_release(gpu_engine):
    """pg_dict_id_sets on one thread while another releases the segments it looks up (pg_segment_release): the
    lookup holds the segment lock through its device work, so each call either sees the segment (the host's dictIds)
    or reports it unknown -- never a read of freed dictionaries."""
    import threading
    from pinot_amd.gpu import PinotGpuError
    from pinot_amd.plan import dict_id_set
    rng = np.random.default_rng(19)
    for rnd in range(4):
        segs = [ImmutableSegment.create(f"r{rnd}_{s}", {"k": rng.integers(0, 200_000, 150_000).astype(np.int64)},
                                        {"k": "LONG"}) for s in range(4)]
        t = Table("t", segs)
        keys = [gpu_engine.upload_segment(s, t) for s in segs]
        lits = np.arange(0, 200_000, 7, dtype=np.int64)
        want = [dict_id_set(s.columns["k"].dictionary, lits.tolist()) for s in segs]
        outcomes, errors = [], []

        def lookup():
            for _ in range(20):
                try:
                    ids, counts = gpu_engine.dict_id_sets(t.column_ids["k"], "LONG", lits, keys)
                    for si in range(len(segs)):
                        if not np.array_equal(ids[si, :counts[si]], want[si]):
                            errors.append(si)
                    outcomes.append("ok")
                except PinotGpuError as e:  # a released segment: refused, not read
                    outcomes.append(str(e)[:40])

        th = threading.Thread(target=lookup)
        th.start()
        for s in segs:
            gpu_engine.release(s)
        th.join()
        assert not errors, errors
        assert len(outcomes) == 20


def test_in_literals_on_mv_scan_leaves(gpu_engine, oracle_engine):
    """IN / NOT_IN over an MV column without an inverted index, several segments: the leaves cross as their literals
    (values mode) and the device finds each segment's dictIds while it builds the MV scan's LUT."""
    rng = np.random.default_rng(11)
    segs = []
    for s in range(3):
        n = 20_000 + 1_000 * s
        data = {"tags": [list(rng.integers(0, 400 + 50 * s, rng.integers(1, 6))) for _ in range(n)],
                "m": rng.integers(0, 30, n)}
        segs.append(_seg(f"mv{s}", data, {"tags": "INT", "m": "INT"}))
    t = Table("t", segs)
    lits = ", ".join(str(x) for x in range(3, 420, 7))
    for sql in [f"SELECT COUNT(*), COUNTMV(tags) FROM t WHERE tags IN ({lits})",
                f"SELECT m, COUNT(*) FROM t WHERE tags NOT IN ({lits}) GROUP BY m",
                f"SELECT COUNT(*) FROM t WHERE tags IN ({lits}) AND m < 10"]:
        q = parse(sql)
        assert_same_result(gpu_engine.execute(t, q), oracle_engine.execute(t, q), table=t)


def test_partial_rows_export_merge_roundtrip(gpu_engine, oracle_engine, sv_table_inter):
    """pg_partials_export (rows bucketed by owner) -> pg_partials_create + pg_partials_merge of every bucket ->
    finalize == the direct result, for a dense and a hash state."""
    import ctypes as C
    import torch
    from pinot_amd import abi
    q = parse("SELECT column11, column12, COUNT(*), SUM(column1), MIN(column3), MAX(column6), AVG(column9), "
              "DISTINCTCOUNT(column7) FROM t GROUP BY column11, column12")
    o = oracle_engine.execute(sv_table_inter, q)
    for flags in (abi.PG_PLAN_VALUE_SETS, abi.PG_PLAN_VALUE_SETS | abi.PG_PLAN_HASH_GROUPS):
        plan = gpu_engine.make_plan(sv_table_inter, q, flags=flags)
        p = gpu_engine.run_partial(plan)
        counts = gpu_engine.export_rows(p, 3)
        rb = p.contents.row_bytes
        buf = torch.empty(sum(counts) * rb, dtype=torch.uint8, device="cuda")
        assert gpu_engine.export_rows(p, 3, C.c_void_p(buf.data_ptr()), sum(counts)) == counts
        keys = buf.view(-1, rb)[:, :8].contiguous().view(torch.int64).cpu().numpy().astype(np.uint64)
        owners = [gpu_engine.lib.pg_key_owner(int(k), 3) for k in keys.ravel()]
        assert owners == sorted(owners)
        qq = gpu_engine.create_like(p, sum(counts))
        qq.contents.stats = p.contents.stats
        at = 0
        for c in counts:  # bucket by bucket, as the owners would receive them
            gpu_engine.merge_rows(qq, C.c_void_p(buf.data_ptr() + at * rb), c)
            at += c
        gpu_engine.lib.pg_partials_free(p)
        assert_same_result(gpu_engine.finalize_partial(plan, qq), o, table=sv_table_inter)


# ------------------------------------------------------------------ synthetic segments (config 2 shape + edges)

def _seg(name, data, schema, **kw):
    return ImmutableSegment.create(name, data, schema, **kw)


def test_config2_shape_small(gpu_engine, oracle_engine):
    from pinot_amd import synth
    segs = [synth.make_segment_np(synth.ADANALYTICS, s, 150_001) for s in range(3)]
    t = Table("adAnalytics", segs)
    q = parse(synth.adanalytics_query(5000))
    assert_same_result(gpu_engine.execute(t, q), oracle_engine.execute(t, q), table=t)


def test_config3_ssb_shape_small(gpu_engine, oracle_engine):
    """Config 3 (SSB Q1.1 shape): three range filters + SUM(lo_extendedprice * lo_discount), integer-exact."""
    from pinot_amd import synth
    segs = [synth.make_segment_np(synth.SSB_LINEORDER, s, 120_007) for s in range(3)]
    t = Table("lineorder", segs)
    q = parse(synth.ssb_q11_query())
    g, o = gpu_engine.execute(t, q), oracle_engine.execute(t, q)
    assert g.stats.num_docs_scanned > 0
    assert_same_result(g, o, table=t)


def test_large_dictionary_dense_decode(gpu_engine, oracle_engine):
    """Dense aggregation over a large-dictionary column: triggers the XCD-grouped work-item order (items of one
    segment interleaved over one XCD's blocks); results must not depend on the order."""
    from pinot_amd import synth
    segs = [synth.make_segment_np(synth.SSB_LINEORDER, s, 300_000) for s in range(4)]
    t = Table("lineorder", segs)
    for sql in ["SELECT SUM(lo_extendedprice), MIN(lo_extendedprice), MAX(lo_extendedprice), COUNT(*) FROM t",
                "SELECT lo_discount, SUM(lo_extendedprice), AVG(lo_extendedprice) FROM t GROUP BY lo_discount",
                "SELECT DISTINCTCOUNT(lo_quantity), SUM(lo_extendedprice * lo_quantity) FROM t WHERE lo_quantity > 3"]:
        q = parse(sql)
        assert_same_result(gpu_engine.execute(t, q), oracle_engine.execute(t, q), table=t)


def test_device_generated_segments_match_host_bytes(gpu_engine, oracle_engine):
    """Segments generated on the GPU (bench path) give the same results as their host copies through the oracle."""
    import torch
    from pinot_amd import synth
    from pinot_amd.segment import ImmutableSegment as IS
    segs, host_segs = [], []
    n = 200_000
    t_cols = {}
    for s in range(2):
        dcs = synth.make_columns_torch(synth.ADANALYTICS, s, n, torch.device("cuda"))
        cols = {dc.spec.name: dc.host_column() for dc in dcs}
        seg = IS(f"d{s}", n, cols)
        segs.append((seg, dcs))
    table = Table("adAnalytics", [s for s, _ in segs])
    for seg, dcs in segs:
        gpu_engine.register_device_segment(seg, table, dcs)
    q = parse(synth.adanalytics_query(20000))
    g = gpu_engine.execute(table, q)
    o = oracle_engine.execute(table, q)
    assert_same_result(g, o, table=table)
    assert g.stats.num_docs_scanned > 0


@pytest.mark.parametrize("n", [1, 63, 64, 4095, 4096, 4097, 10001, 70000])
def test_ragged_sizes(n, gpu_engine, oracle_engine):
    rng = np.random.default_rng(n)
    data = {"a": rng.integers(0, 3, n), "b": rng.integers(-1000, 1000, n), "c": rng.integers(0, 2 ** 21, n),
            "d": rng.normal(size=n)}
    seg = _seg("r", data, {"a": "INT", "b": "LONG", "c": "INT", "d": "DOUBLE"})
    t = Table("t", [seg, seg])
    for sql in ["SELECT COUNT(*), SUM(b), MIN(c), MAX(d), AVG(d) FROM t WHERE c > 1000",
                "SELECT a, COUNT(*), SUM(d), SUM(b), MIN(b) FROM t WHERE b BETWEEN -10 AND 500 GROUP BY a",
                "SELECT DISTINCTCOUNT(b) FROM t WHERE a <> 1"]:
        q = parse(sql)
        assert_same_result(gpu_engine.execute(t, q), oracle_engine.execute(t, q), table=t)


def test_balanced_split_over_ragged_segments(gpu_engine, oracle_engine):
    """Unequal segments (13/31/22/4 tiles of 8 192 docs): the balanced work split cuts the concatenated tile sequence
    into equal per-block ranges that straddle segment boundaries; per-segment state (match counts, IN sets, dictIds
    per segment dictionary) must still land in the right segment."""
    rng = np.random.default_rng(7)
    segs = []
    for i, n in enumerate([100_000, 250_001, 180_000, 8193 * 3]):
        data = {"k": rng.integers(0, 40, n), "v": rng.integers(-5000, 5000, n), "w": rng.integers(0, 300_000, n)}
        segs.append(_seg(f"b{i}", data, {"k": "INT", "v": "LONG", "w": "INT"}))
    t = Table("t", segs)
    ids = ", ".join(str(x) for x in range(0, 300_000, 97))
    for sql in ["SELECT COUNT(*), SUM(v), MIN(w), MAX(v) FROM t",
                f"SELECT k, COUNT(*), SUM(v) FROM t WHERE w IN ({ids}) GROUP BY k",
                "SELECT k, AVG(v), DISTINCTCOUNT(w) FROM t WHERE v BETWEEN -100 AND 2500 GROUP BY k"]:
        q = parse(sql)
        g, o = gpu_engine.execute(t, q), oracle_engine.execute(t, q)
        assert_same_result(g, o, table=t)
        assert g.stats.num_segments_matched == o.stats.num_segments_matched


def test_empty_and_all_filtered(gpu_engine, oracle_engine):
    rng = np.random.default_rng(1)
    seg = _seg("e", {"a": rng.integers(0, 10, 5000), "b": rng.integers(0, 100, 5000)}, {"a": "INT", "b": "INT"})
    t = Table("t", [seg])
    for sql in ["SELECT COUNT(*), SUM(b), MIN(b), MAX(b) FROM t WHERE a > 100",
                "SELECT a, SUM(b) FROM t WHERE a = 77 GROUP BY a",
                "SELECT COUNT(*) FROM t WHERE a IN (11, 12) OR b = 1000"]:
        q = parse(sql)
        g, o = gpu_engine.execute(t, q), oracle_engine.execute(t, q)
        assert_same_result(g, o, table=t)
        assert g.stats.num_docs_scanned == 0


def test_no_segments(gpu_engine, oracle_engine):
    """A query over an empty segment list (a server whose segments were all pruned): the readback of the match
    counts / error word and the small final state still runs (one launch into mapped host memory), stats all zero."""
    rng = np.random.default_rng(3)
    seg = _seg("z", {"a": rng.integers(0, 10, 3000), "b": rng.integers(0, 100, 3000)}, {"a": "INT", "b": "INT"})
    t = Table("t", [seg])
    for sql in ["SELECT COUNT(*), SUM(b), MIN(b), MAX(b) FROM t WHERE a > 3",
                "SELECT a, SUM(b) FROM t WHERE b < 50 GROUP BY a"]:
        q = parse(sql)
        g, o = gpu_engine.execute(t, q, segments=[]), oracle_engine.execute(t, q, segments=[])
        assert_same_result(g, o, table=t)
        assert g.stats.num_docs_scanned == 0 and g.stats.num_segments_processed == 0


def test_per_segment_dictionaries_merge_by_value(gpu_engine, oracle_engine):
    """dictIds are segment-local: different value sets per segment still merge by VALUE (IndexedTable keys)."""
    rng = np.random.default_rng(2)
    segs = []
    for s in range(4):
        n = 30000 + s * 777
        data = {"k": rng.integers(s * 5, s * 5 + 20, n), "name": np.array(["x%d" % i for i in range(s, s + 7)],
                                                                           dtype=object)[rng.integers(0, 7, n)],
                "v": rng.integers(0, 10 ** 6, n), "f": rng.uniform(-5, 5, n).astype(np.float32)}
        segs.append(_seg(f"s{s}", data, {"k": "INT", "name": "STRING", "v": "LONG", "f": "FLOAT"}))
    t = Table("t", segs)
    for sql in ["SELECT k, name, COUNT(*), SUM(v), MAX(f) FROM t GROUP BY k, name",
                "SELECT name, DISTINCTCOUNT(k), AVG(f), MIN(f) FROM t WHERE v < 500000 GROUP BY name",
                "SELECT f, COUNT(*) FROM t WHERE k < 3 GROUP BY f"]:
        q = parse(sql)
        assert_same_result(gpu_engine.execute(t, q), oracle_engine.execute(t, q), table=t)


@pytest.mark.parametrize("fused", ["1", "0"])
def test_sorted_and_inverted_and_mv(fused, monkeypatch, gpu_engine, oracle_engine):
    """Config-5 shape in miniature: sorted column, inverted-index leaves (incl. exclusive), MV COUNTMV + MV filter --
    through the fused index count (pg_index.hip: per-key LDS decode of the containers, no doc bitmaps) where the shape
    allows it (fused=1, the default) and through the index pre-pass + fused scan (PG_INDEX_FUSED=0)."""
    monkeypatch.setenv("PG_INDEX_FUSED", fused)
    rng = np.random.default_rng(3)
    n = 50000
    data = {"sortedCol": np.sort(rng.integers(0, 1000, n)), "inv1": rng.integers(0, 10, n),
            "inv2": rng.integers(0, 100, n), "inv3": rng.integers(0, 1000, n), "inv4": rng.integers(0, 10000, n),
            "mvTags": [list(rng.integers(0, 1000, rng.integers(1, 8))) for _ in range(n)]}
    seg = _seg("idx", data, {k: "INT" for k in data}, inverted=["inv1", "inv2", "inv3", "inv4", "mvTags"])
    seg2 = _seg("scan", data, {k: "INT" for k in data})  # same data, scan-only leaves
    for segs in ([seg], [seg2], [seg, seg2]):
        t = Table("t", segs)
        for sql in [
            "SELECT COUNT(*), COUNTMV(mvTags) FROM t WHERE sortedCol BETWEEN 100 AND 600 AND (inv1 = 3 OR inv2 IN "
            "(1, 5, 9, 50)) AND inv3 <> 7 AND inv4 IN (1, 2, 3, 100, 200, 300, 4000, 5000)",
            "SELECT COUNT(*), COUNTMV(mvTags) FROM t WHERE mvTags IN (5, 6, 7) AND NOT sortedCol < 200",
            "SELECT COUNT(*) FROM t WHERE mvTags NOT IN (1, 2, 3, 4, 5, 6, 7, 8, 9, 10)",
            "SELECT inv1, COUNTMV(mvTags), SUM(inv4) FROM t WHERE sortedCol IN (5, 77, 800) OR inv2 > 90 GROUP BY inv1",
            "SELECT COUNT(*) FROM t WHERE sortedCol NOT IN (5, 6, 7) AND inv1 NOT IN (0, 1)",
            "SELECT COUNTMV(mvTags) FROM t",
            "SELECT COUNT(*), COUNTMV(mvTags) FROM t WHERE NOT (inv1 IN (1, 2) AND inv3 < 500) OR inv4 = 77",
            "SELECT COUNT(*) FROM t WHERE inv2 NOT IN (3, 4) AND NOT inv1 = 5 AND sortedCol >= 10",
        ]:
            q = parse(sql)
            assert_same_result(gpu_engine.execute(t, q), oracle_engine.execute(t, q), table=t)
    t = Table("t", [seg])
    gpu_engine.execute(t, "SELECT COUNT(*), COUNTMV(mvTags) FROM t WHERE sortedCol BETWEEN 100 AND 600 AND inv1 = 3")
    assert ("index_count" in gpu_engine.last_trace()["path"]) == (fused == "1")
    # a scan leaf (inv3 < 500 is a dictId range: no range index) anywhere in the filter rules the fused count out
    gpu_engine.execute(t, "SELECT COUNT(*), COUNTMV(mvTags) FROM t WHERE NOT (inv1 IN (1, 2) AND inv3 < 500)")
    assert "index_count" not in gpu_engine.last_trace()["path"]


def test_fused_index_count_wide_mv_rows(gpu_engine, oracle_engine):
    """COUNTMV through the fused index count when some doc holds more than 15 values (no 4-bit count column: the row
    offsets), with segments whose inverted leaf is a constant (a dictId absent from one segment)."""
    rng = np.random.default_rng(5)
    segs = []
    for s_ in range(3):
        n = 40_000 + 999 * s_
        data = {"inv": rng.integers(0, 50 + 10 * s_, n),
                "tags": [list(rng.integers(0, 300, rng.integers(1, 40 if s_ == 1 else 6))) for _ in range(n)]}
        segs.append(_seg(f"w{s_}", data, {"inv": "INT", "tags": "INT"}, inverted=["inv"]))
    t = Table("t", segs)
    for sql in ["SELECT COUNT(*), COUNTMV(tags) FROM t WHERE inv IN (1, 7, 55, 59)",
                "SELECT COUNTMV(tags) FROM t WHERE inv <> 3",
                "SELECT COUNT(*), COUNTMV(tags) FROM t WHERE inv = 58 OR inv = 2"]:
        q = parse(sql)
        assert_same_result(gpu_engine.execute(t, q), oracle_engine.execute(t, q), table=t)
        assert "index_count" in gpu_engine.last_trace()["path"]


@pytest.mark.parametrize("neg", [False, True])
def test_fused_index_count_leaf_referenced_twice(neg, gpu_engine, oracle_engine):
    """An op program that references one inverted leaf twice (the ABI allows it; a JNI caller may send it): the fused
    count lets the positive leaves of an OR share one LDS chunk only when each is referenced once, so `a AND (a OR c)`
    still ANDs a's own docs and `NOT a AND (a OR c)` is `NOT a AND c`.  Built from a plan whose second, identical
    predicate's leaf is replaced by the first in the ops."""
    rng = np.random.default_rng(11)
    n = 60000
    seg = _seg("twice", {"inv1": rng.integers(0, 10, n), "inv2": rng.integers(0, 100, n)}, {"inv1": "INT", "inv2": "INT"},
               inverted=["inv1", "inv2"])
    t = Table("t", [seg])
    sql = ("SELECT COUNT(*) FROM t WHERE " + ("NOT inv1 = 3" if neg else "inv1 = 3") +
           " AND (inv1 = 3 OR inv2 IN (1, 5, 9, 50))")
    want = oracle_engine.execute(t, parse(sql))
    plan = gpu_engine.make_plan(t, parse(sql))
    assert list(plan.ops).count(1) == 1 and list(plan.ops).count(0) == 1
    for i, op in enumerate(plan.ops):
        if op == 1:
            plan.plan.ops[i] = 0  # the OR's `inv1 = 3` now names the AND's leaf 0
    got = gpu_engine.run_plan(plan, image=False)
    assert "index_count" in gpu_engine.last_trace()["path"]
    assert got.rows == want.rows


def test_config5_full_segment_matches_oracle(gpu_engine, oracle_engine):
    """Config 5 at its stated scale: full 7 812 500-doc segments built on the device in the reference's byte layouts
    (sorted pairs, portable-roaring inverted indexes, FixedBitMVForwardIndexWriter MV column: pinot_amd.synth), the
    bench query and variants with NOT_IN / range / OR / NOT on the inverted and sorted indexes, GPU vs oracle."""
    import torch
    from pinot_amd import synth
    dev = torch.device("cuda", 0)
    segs, host = [], []
    table = None
    for si in range(2):
        dcs = synth.make_index_columns_torch(si, 7_812_500, dev)
        seg = ImmutableSegment(f"idx_{si}", 7_812_500, {dc.spec.name: dc.meta_column() for dc in dcs})
        hs = ImmutableSegment(f"idx_{si}", 7_812_500, {dc.spec.name: dc.host_column() for dc in dcs})
        if table is None:
            table = Table("idx", [seg])
        gpu_engine.register_device_segment(seg, table, dcs)
        segs.append(seg)
        host.append(hs)
        del dcs
    t, ht = Table("idx", segs), Table("idx", host)
    for sql in [synth.index_query(),
                "SELECT COUNT(*), COUNTMV(mvTags) FROM idx WHERE sortedCol NOT BETWEEN 1000 AND 90000 AND inv4 NOT IN "
                "(3, 4, 5, 6, 7, 8) AND (inv2 < 20 OR inv1 = 9)",
                "SELECT COUNT(*) FROM idx WHERE inv3 IN (10, 20, 30) OR NOT inv1 <> 4",
                "SELECT inv1, COUNT(*), COUNTMV(mvTags) FROM idx WHERE sortedCol < 50000 AND inv2 = 42 GROUP BY inv1"]:
        q = parse(sql)
        assert_same_result(gpu_engine.execute(t, q), oracle_engine.execute(ht, q), table=t)
    for seg in segs:
        gpu_engine.release(seg)


def test_partials_roundtrip_single_rank(gpu_engine, oracle_engine, sv_table_inter):
    """pg_execute_partial -> pg_partials_copy out/in -> pg_partials_finalize == pg_execute (1-rank dense merge)."""
    import ctypes as C
    import torch
    from pinot_amd import abi
    q = parse("SELECT column11, COUNT(*), SUM(column1), MIN(column3), MAX(column6), AVG(column7) FROM t "
              "GROUP BY column11")
    o = oracle_engine.execute(sv_table_inter, q)
    # integer-exact i64 sums, then every sum as an exact fixed-point sum (its 128-bit pairs travel as 4 limbs each)
    for flags in (0, abi.PG_PLAN_F64_SUMS):
        plan = gpu_engine.make_plan(sv_table_inter, q, flags=flags)
        p = gpu_engine.run_partial(plan)
        pc = p.contents
        assert pc.mode == abi.PG_STATE_DENSE and (pc.n_fx == 2) == bool(flags)
        bufs = [torch.empty(max(pc.num_slots * k, 1) * 8, dtype=torch.uint8, device="cuda")
                for k in (pc.n_i64, 4 * pc.n_fx, pc.n_min, pc.n_max)]
        ptrs = [C.c_void_p(b.data_ptr()) for b in bufs]
        assert gpu_engine.lib.pg_partials_copy(p, abi.PG_COPY_OUT, *ptrs, None) == 0
        if flags:  # the limbs are 32-bit values: a SUM of them over ranks cannot overflow
            limbs = bufs[1].view(torch.int64)
            assert int(limbs.min()) >= 0 and int(limbs.max()) < (1 << 32)
        assert gpu_engine.lib.pg_partials_copy(p, abi.PG_COPY_IN, *ptrs, None) == 0
        g = gpu_engine.finalize_partial(plan, p)
        assert_same_result(g, o, table=sv_table_inter)


# ------------------------------------------------------------------ config 1: QuickStart baseballStats

@pytest.fixture(scope="module")
def baseball_table():
    from pinot_amd import synth
    return Table("baseballStats", [synth.baseball_segment()])


@pytest.mark.parametrize("qi", range(6))
def test_config1_baseball_quickstart(qi, gpu_engine, oracle_engine, baseball_table):
    """BASELINE config 1: Quickstart.java:185-213's baseballStats queries (STRING playerName group key through a
    keymap, inverted-index leaves on playerID / teamID) -- device vs oracle, plain and with the device ORDER BY trim."""
    from pinot_amd import synth
    q = parse(synth.BASEBALL_QUERIES[qi])
    o = oracle_engine.execute(baseball_table, q)
    g = gpu_engine.execute(baseball_table, q)
    assert_same_result(g, o, table=baseball_table)
    t = gpu_engine.execute(baseball_table, q, trim=True)
    assert reduce_to_rows(q, t)[1] == reduce_to_rows(q, o)[1]


def test_v3_store_segments_on_device(tmp_path, gpu_engine, oracle_engine):
    """Segments loaded from the V3 single-file store (SingleFileIndexDirectory) feed pg_column_upload unchanged:
    a synthetic segment written as V3 and the reference's own paddingNull V1 bytes converted to V3."""
    import os
    rng = np.random.default_rng(11)
    n = 60_000
    data = {"k": rng.integers(0, 50, n), "v": rng.integers(-10 ** 6, 10 ** 6, n), "s": np.sort(rng.integers(0, 90, n)),
            "t": np.array(["a", "bb", "ccc", "dd"], dtype=object)[rng.integers(0, 4, n)]}
    seg = _seg("v3", data, {"k": "INT", "v": "LONG", "s": "INT", "t": "STRING"}, inverted=["t"])
    seg.write_v3(str(tmp_path / "syn"))
    back = ImmutableSegment.load(str(tmp_path / "syn"))
    t_orig, t_v3 = Table("t", [seg]), Table("t", [back])
    for sql in ["SELECT k, COUNT(*), SUM(v), MIN(v) FROM t WHERE t IN ('a', 'dd') AND s BETWEEN 10 AND 70 GROUP BY k",
                "SELECT t, DISTINCTCOUNT(k), MAX(v) FROM t WHERE v > 0 GROUP BY t"]:
        q = parse(sql)
        assert_same_result(gpu_engine.execute(t_v3, q), oracle_engine.execute(t_orig, q), table=t_orig)
    golden = os.path.join(os.path.dirname(__file__), "golden", "padding_null")
    ImmutableSegment.load_v1(golden).write_v3(str(tmp_path / "pad"))
    pad = Table("t", [ImmutableSegment.load(str(tmp_path / "pad"))])
    q = parse("SELECT COUNT(*), MIN(age), MAX(age), SUM(age) FROM t")
    g = gpu_engine.execute(pad, q)
    assert g.rows[()][:4] == [5, 617.0, 1228.0, 617.0 + 824 + 837 + 1209 + 1228]


def test_plan_image_and_pointer_plan_agree(gpu_engine, sv_table_inter):
    """pg_execute_image (the relocatable image a JNI caller passes) and pg_execute (the in-process pointer plan) give
    identical results for the same lowered plan: every SV query, a values-mode IN over several segments, a server
    trim; and the partial / finalize pair through images."""
    from pinot_amd import synth
    segs = [synth.make_segment_np(synth.ADANALYTICS, s, 100_003) for s in range(3)]
    ad = Table("adAnalytics", segs)
    cases = [(sv_table_inter, q) for q in SV_QUERIES] + [(ad, synth.adanalytics_query(20000))]
    for t, sql in cases:
        q = parse(sql)
        for trim in (False, "server"):
            plan = gpu_engine.make_plan(t, q, trim=trim)
            a, b = gpu_engine.run_plan(plan, image=True), gpu_engine.run_plan(plan, image=False)
            assert a.rows == b.rows and a.stats == b.stats, sql
            c = gpu_engine.finalize_partial(plan, gpu_engine.run_partial(plan, image=True))
            assert c.rows == a.rows, sql


def _full_device_segments(gpu_engine, specs, table_name, n_segs, seg0=0):
    """n_segs full 7 812 500-row segments generated on the device (as bench.py does) + their host copies."""
    import torch
    from pinot_amd import synth
    dev = torch.device("cuda", 0)
    rows = synth.ADANALYTICS_ROWS_PER_SEGMENT
    segs, host, bits = [], [], []
    table = None
    for si in range(seg0, seg0 + n_segs):
        dcs = synth.make_columns_torch(specs, si, rows, dev)
        seg = ImmutableSegment(f"{table_name}_{si}", rows, {dc.spec.name: dc.meta_column() for dc in dcs})
        host.append(ImmutableSegment(f"{table_name}_{si}", rows, {dc.spec.name: dc.host_column() for dc in dcs}))
        bits.append({dc.spec.name: (dc.bits, dc.cardinality) for dc in dcs})
        if table is None:
            table = Table(table_name, [seg])
        gpu_engine.register_device_segment(seg, table, dcs)
        segs.append(seg)
        del dcs
    return Table(table_name, segs), Table(table_name, host), bits


@pytest.mark.parametrize("config", ["adanalytics", "ssb"])
def test_full_size_segments_match_oracle(config, gpu_engine):
    """Configs 2 and 3 at their stated segment size: full 7 812 500-row device-generated segments (2 for config 2, 3 for
    config 3), through the selective stream (scan_launches == 2: stream_kernel + the list-mode scan) -- for config 2 the
    benchmark's own kernel instance, accountId at 20 bits with a <= 1 M-id exact LUT -- against the oracle over the
    same segments' host bytes."""
    from oracle.oracle import OracleEngine
    from pinot_amd import synth
    specs, name, n, sql = ((synth.ADANALYTICS, "adAnalytics", 2, synth.adanalytics_query(1000)) if config == "adanalytics"
                           else (synth.SSB_LINEORDER, "lineorder", 3, synth.ssb_q11_query()))
    t, ht, bits = _full_device_segments(gpu_engine, specs, name, n, seg0=5)
    try:
        if config == "adanalytics":
            assert all(b["accountId"][0] == 20 and b["accountId"][1] <= 1 << 20 for b in bits)
        q = parse(sql)
        for trim in (False, "server"):
            g = gpu_engine.execute(t, q, flags=0, trim=trim)
            assert gpu_engine.last_timing().scan_launches == 2, "the selective stream did not run"
            o = OracleEngine(threads=8).execute(ht, q)
            assert_same_result(g, o, table=ht)
            assert g.stats.num_docs_scanned > 0
    finally:
        for seg in t.segments:
            gpu_engine.release(seg)
