"""Host lowering (pinot_amd/plan.py) without a GPU: the batched IN / NOT_IN lookup path of CPlan (one id_sets call per
predicate over all segments, as GpuEngine does through pg_dict_id_sets) lowers every leaf exactly as the per-segment
PredicateUtils.getDictIdSet restatement does."""
import numpy as np
import pytest

from pinot_amd import abi
from pinot_amd.plan import CPlan, Table, dict_id_set
from pinot_amd.query import parse
from pinot_amd.segment import ImmutableSegment


def _host_id_sets(segments, calls):
    """A host stand-in for pg_dict_id_sets: the same contract (ids [S, n] rows holding counts[s] ascending dictIds)."""
    by_key = {}

    def id_sets(col_id, data_type, literals, seg_keys):
        calls.append((col_id, data_type, len(literals)))
        n = len(literals)
        ids = np.full((len(seg_keys), max(n, 1)), -7, dtype=np.int32)
        counts = np.zeros(len(seg_keys), dtype=np.uint32)
        for s, k in enumerate(seg_keys):
            d = by_key[k]
            found = dict_id_set(d, list(literals))
            ids[s, :len(found)] = found
            counts[s] = len(found)
        return ids, counts

    return id_sets, by_key


@pytest.mark.parametrize("dtype", ["INT", "LONG", "FLOAT", "DOUBLE"])
def test_batched_in_lowering_matches_per_segment(dtype):
    rng = np.random.default_rng(3)
    segs = []
    for s in range(4):
        n = 3_001 + 997 * s
        v = rng.integers(-400, 400, n)
        data = {"k": v.astype(np.int64) if dtype in ("INT", "LONG") else v.astype(np.float64) / 8,
                "m": rng.integers(0, 50, n).astype(np.int64)}
        segs.append(ImmutableSegment.create(f"s{s}", data, {"k": dtype, "m": "INT"}))
    t = Table("t", segs)
    lits = ", ".join(str(x) for x in (range(-500, 500, 13) if dtype in ("INT", "LONG") else
                                      [x / 8 for x in range(-3_000, 3_000, 37)]))
    calls = []
    for sql in [f"SELECT COUNT(*) FROM t WHERE k IN ({lits})",
                f"SELECT m, COUNT(*) FROM t WHERE k NOT IN ({lits}) AND m < 30 GROUP BY m",
                "SELECT COUNT(*) FROM t WHERE k IN (123456789)"]:
        q = parse(sql)
        keys = list(range(1, len(segs) + 1))
        id_sets, by_key = _host_id_sets(segs, calls)
        by_key.update({k: s.columns["k"].dictionary for k, s in zip(keys, segs)})
        batched = CPlan(t, q, segs, keys, id_sets=id_sets)
        plain = CPlan(t, q, segs, keys)
        for lb, lp in zip(batched.lowered, plain.lowered):
            for a, b in zip(lb, lp):
                assert (a.kind, a.col_id, a.exclusive, a.lo, a.hi) == (b.kind, b.col_id, b.exclusive, b.lo, b.hi)
                assert (a.ids is None) == (b.ids is None)
                if a.ids is not None:
                    assert np.array_equal(np.asarray(a.ids, dtype=np.int32), np.asarray(b.ids, dtype=np.int32))
        # values mode on the C side: a non-contiguous IN / NOT_IN set crosses as the literals (ids left to the device)
        for si in range(len(segs)):
            leaf = batched.plan.segments[si].leaves[0]
            if leaf.num_ids and leaf.kind in (abi.PG_LEAF_SV_SCAN, abi.PG_LEAF_MV_SCAN):
                ids = batched.lowered[si][0].ids
                contiguous = int(ids[-1]) - int(ids[0]) + 1 == len(ids)
                assert bool(leaf.ids) == contiguous and (leaf.num_values > 0) != contiguous
    assert calls and all(c[1] == dtype for c in calls)


def test_literal_absent_everywhere_is_empty_leaf():
    rng = np.random.default_rng(0)  # unsorted columns: scan leaves (a sorted one would lower to a sorted-index leaf)
    segs = [ImmutableSegment.create(f"s{s}", {"k": rng.permutation(np.arange(10 * s, 10 * s + 10, dtype=np.int64))},
                                    {"k": "INT"}) for s in range(3)]
    t = Table("t", segs)
    calls = []
    id_sets, by_key = _host_id_sets(segs, calls)
    by_key.update({k: s.columns["k"].dictionary for k, s in zip([1, 2, 3], segs)})
    p = CPlan(t, parse("SELECT COUNT(*) FROM t WHERE k IN (5, 15, 99)"), segs, [1, 2, 3], id_sets=id_sets)
    kinds = [lw[0].kind for lw in p.lowered]
    assert kinds == [abi.PG_LEAF_SV_SCAN, abi.PG_LEAF_SV_SCAN, abi.PG_LEAF_EMPTY]


# ------------------------------------------------------------------ the instance's group-by settings


def test_num_groups_limit_is_an_instance_setting(oracle_engine):
    """numGroupsLimit comes from the server instance only (InstancePlanMakerImplV2.java:223; QueryOptionsUtils has no
    such option): an OPTION(numGroupsLimit=...) changes neither the plan nor the result, and the instance's limit
    truncates each segment to the first `limit` keys in doc order (IntGroupIdMap.getGroupId,
    DictionaryBasedGroupKeyGenerator.java:991-1016) -- checked against numpy -- with numGroupsLimitReached set."""
    from pinot_amd.plan import DEFAULT_NUM_GROUPS_LIMIT, InstanceConfig
    rng = np.random.default_rng(11)
    segs, raw = [], []
    for s in range(3):
        n = 5_000 + 777 * s
        data = {"k": rng.integers(0, 400, n).astype(np.int64), "v": rng.integers(-1000, 1000, n).astype(np.int64)}
        raw.append(data)
        segs.append(ImmutableSegment.create(f"n{s}", data, {"k": "INT", "v": "LONG"}))
    t = Table("t", segs)
    sql = "SELECT k, COUNT(*), SUM(v) FROM t GROUP BY k"
    assert CPlan(t, parse(sql + " OPTION(numGroupsLimit=5)"), segs, [1, 2, 3]).plan.num_groups_limit == \
        DEFAULT_NUM_GROUPS_LIMIT
    cfg = InstanceConfig.with_groups_limit(37)
    assert CPlan(t, parse(sql), segs, [1, 2, 3], config=cfg).plan.num_groups_limit == 37
    want = {}
    for d in raw:   # numpy: each segment keeps its first 37 distinct keys (doc order), then the merge by value
        keys, first = np.unique(d["k"], return_index=True)
        kept = keys[np.argsort(first)][:37]
        for k in kept.tolist():
            m = d["k"] == k
            c, sm = want.get((k,), [0, 0.0])
            want[(k,)] = [c + int(m.sum()), sm + float(d["v"][m].sum())]
    for extra in ("", " OPTION(numGroupsLimit=1000000)", " OPTION(numGroupsLimit=2)"):
        r = oracle_engine.execute(t, sql + extra, config=cfg)
        assert r.rows == want and r.groups_limit_reached
    full = oracle_engine.execute(t, sql + " OPTION(numGroupsLimit=2)")   # default instance: every group, no limit hit
    assert len(full.rows) == 400 and not full.groups_limit_reached
    with pytest.raises(ValueError):   # the constructor's precondition (InstancePlanMakerImplV2.java:138-140)
        InstanceConfig(num_groups_limit=100)
    with pytest.raises(ValueError):
        InstanceConfig(groupby_trim_threshold=0)


def test_trim_threshold_flag_in_the_oracle(oracle_engine):
    """groupTrimThreshold: the reference server's table (ORDER BY, server trim on) resizes whenever it holds >=
    threshold records (ConcurrentIndexedTable.java:61-65); the oracle reports that instead of reproducing the lossy,
    schedule-dependent resize, and the plan carries the threshold to the device (pg_plan.trim_threshold)."""
    from pinot_amd.plan import MAX_TRIM_THRESHOLD, InstanceConfig
    rng = np.random.default_rng(12)
    segs = [ImmutableSegment.create(f"m{s}", {"k": rng.integers(0, 3000, 20_000).astype(np.int64)}, {"k": "INT"})
            for s in range(2)]
    t = Table("t", segs)
    sql = "SELECT k, COUNT(*) FROM t GROUP BY k ORDER BY COUNT(*) DESC, k LIMIT 10"
    for thr, hit in ((1000, True), (2999, True), (3001, False), (MAX_TRIM_THRESHOLD, False)):
        cfg = InstanceConfig(groupby_trim_threshold=thr)
        r = oracle_engine.execute(t, sql, server=True, config=cfg)
        assert r.trim_threshold_reached == hit and r.num_groups_merged == 3000 and len(r.rows) == 5000 - 2000
        assert CPlan(t, parse(sql), segs, [1, 2], trim="server", config=cfg).plan.trim_threshold == \
            (thr if thr < MAX_TRIM_THRESHOLD else 0)
    # no ORDER BY: no resize at all (the table stops taking keys at its result size instead)
    r = oracle_engine.execute(t, "SELECT k, COUNT(*) FROM t GROUP BY k LIMIT 10", server=True,
                              config=InstanceConfig(groupby_trim_threshold=1000))
    assert not r.trim_threshold_reached
