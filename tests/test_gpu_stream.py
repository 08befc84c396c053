"""The selective stream (pg_filter.hip stream_kernel + the fused scan in list mode) against the oracle and against the
same plan without it (PG_PLAN_NO_STREAM; double sums may differ in summation order, within 1e-9 relative).

The stream is used when the root AND's first child (or the whole filter) is a packed scan leaf the host expects to
pass at most 1/32 of the docs: a lean kernel evaluates that leaf over every segment and compacts the survivors, and
the fused scan evaluates the AND's other children and aggregates over them.  Bar: identical to the oracle (integer
SUM / COUNT / MIN / MAX / keys exact), and identical with and without the stream.  A skewed column whose actual pass
fraction is far above the estimate overflows the survivor regions: the library must rerun without the stream and
still return the oracle's answer."""
import numpy as np
import pytest

from helpers import assert_same_result
from pinot_amd import abi
from pinot_amd.plan import Table
from pinot_amd.query import parse
from pinot_amd.segment import ImmutableSegment

pytestmark = pytest.mark.gpu

SCHEMA = {"day": "INT", "acct": "INT", "clicks": "INT", "imps": "LONG", "price": "DOUBLE", "tag": "STRING"}


def _segment(name, n, seed):
    rng = np.random.default_rng(seed)
    data = {
        "day": rng.integers(18000, 18365, n),
        "acct": rng.integers(0, 200_000, n),
        "clicks": rng.integers(0, 1000, n),
        "imps": rng.integers(0, 100_000, n),
        "price": np.round(rng.random(n) * 1000, 2),
        "tag": np.array(["t%d" % x for x in rng.integers(0, 50, n)]),
    }
    return ImmutableSegment.create(name, data, SCHEMA)


@pytest.fixture(scope="module")
def table():
    # ragged segment sizes (the last 32-doc group of each is partial)
    return Table("t", [_segment("s0", 150_001, 1), _segment("s1", 77_777, 2), _segment("s2", 200_003, 3)])


def _in_list(k, seed=7, hi=200_000):
    ids = np.random.default_rng(seed).choice(hi, k, replace=False)
    return ", ".join(str(int(x)) for x in sorted(ids))


STREAM_QUERIES = [
    # config 2 shape: selective IN first, range second, group by a small key
    f"SELECT day, SUM(clicks), SUM(imps) FROM t WHERE day BETWEEN 18000 AND 18089 AND acct IN ({_in_list(1000)}) "
    "GROUP BY day ORDER BY day LIMIT 400",
    # the whole filter is the selective leaf
    f"SELECT COUNT(*) FROM t WHERE acct IN ({_in_list(300)})",
    f"SELECT COUNT(*), SUM(clicks), MIN(imps), MAX(price), AVG(clicks) FROM t WHERE acct IN ({_in_list(2000)})",
    # a narrow range as the driving leaf, an OR subtree after it
    "SELECT SUM(clicks * imps), SUM(price) FROM t WHERE acct BETWEEN 1000 AND 1999 AND (tag = 't3' OR day < 18100)",
    "SELECT tag, COUNT(*), SUM(imps) FROM t WHERE acct IN (4242, 99, 150000) GROUP BY tag ORDER BY tag LIMIT 100",
    f"SELECT acct, COUNT(*), MAX(clicks) FROM t WHERE acct IN ({_in_list(500)}) AND clicks > 100 "
    "GROUP BY acct ORDER BY COUNT(*) DESC, acct LIMIT 20",
    f"SELECT DISTINCTCOUNT(tag), SUM(imps) FROM t WHERE acct IN ({_in_list(1500)}) AND NOT tag = 't7'",
]


@pytest.mark.parametrize("sql", STREAM_QUERIES, ids=[f"q{i}" for i in range(len(STREAM_QUERIES))])
def test_stream_matches_oracle_and_no_stream(sql, table, gpu_engine, oracle_engine):
    q = parse(sql)
    g = gpu_engine.execute(table, q)
    assert gpu_engine.last_timing().scan_launches == 2, "the selective stream did not run"
    o = oracle_engine.execute(table, q)
    assert_same_result(g, o, table=table)
    n = gpu_engine.execute(table, q, flags=abi.PG_PLAN_VALUE_SETS | abi.PG_PLAN_NO_STREAM)
    assert gpu_engine.last_timing().scan_launches == 1
    assert_same_result(g, n, table=table)  # double sums: summation order differs (1e-9 relative)
    assert g.stats.num_docs_scanned == n.stats.num_docs_scanned == o.stats.num_docs_scanned


@pytest.mark.parametrize("qi", [0, 5, 6])
def test_stream_exact_mode_further_leaves(qi, table, monkeypatch, gpu_engine, oracle_engine):
    """PG_STREAM_EXACT_EXTRA=1: the exact-mode stream (stream_kernel<B, true, 1024>) also tests the AND's following
    LDS-free leaves on the driving leaf's survivors; same answers as the oracle and as the plan without the stream."""
    monkeypatch.setenv("PG_STREAM_EXACT_EXTRA", "1")
    q = parse(STREAM_QUERIES[qi])
    g = gpu_engine.execute(table, q)
    assert gpu_engine.last_timing().scan_launches == 2, "the selective stream did not run"
    assert_same_result(g, oracle_engine.execute(table, q), table=table)
    n = gpu_engine.execute(table, q, flags=abi.PG_PLAN_VALUE_SETS | abi.PG_PLAN_NO_STREAM)
    assert_same_result(g, n, table=table)


@pytest.mark.parametrize("qi", [0, 1, 5])
def test_stream_overlapped_list_scan(qi, table, monkeypatch, gpu_engine, oracle_engine):
    """The list scan split in two halves, the first on a second HIP stream beside the stream kernel's second launch
    (exact mode, >= 2 segments, <= 2 aggregations and <= 1 key; PG_LIST_OVERLAP=1, off by default): same answers as
    the oracle and as PG_LIST_OVERLAP=0."""
    q = parse(STREAM_QUERIES[qi])
    monkeypatch.setenv("PG_LIST_OVERLAP", "1")
    g = gpu_engine.execute(table, q)
    assert gpu_engine.last_timing().scan_launches == 2, "the selective stream did not run"
    o = oracle_engine.execute(table, q)
    assert_same_result(g, o, table=table)
    assert g.stats.num_docs_scanned == o.stats.num_docs_scanned
    monkeypatch.setenv("PG_LIST_OVERLAP", "0")
    n = gpu_engine.execute(table, q)
    assert_same_result(g, n, table=table)
    assert g.stats.num_docs_scanned == n.stats.num_docs_scanned


def test_stream_not_used_for_unselective_filters(table, gpu_engine, oracle_engine):
    q = parse("SELECT SUM(clicks) FROM t WHERE day BETWEEN 18000 AND 18200 AND acct < 150000")
    g = gpu_engine.execute(table, q)
    assert gpu_engine.last_timing().scan_launches == 1
    assert_same_result(g, oracle_engine.execute(table, q), table=table)


def test_stream_overflow_reruns_without_it(gpu_engine, oracle_engine):
    """The estimate (1 id of 20 000 -> pass 5e-5) is wrong: 90 % of the docs hold that id.  The survivor regions
    overflow; the library reruns the query without the stream and the answer is still the oracle's."""
    n = 120_000
    rng = np.random.default_rng(11)
    hot = rng.random(n) < 0.9
    acct = np.where(hot, 777, rng.integers(0, 20_000, n))
    acct[:20_000] = np.arange(20_000)  # every id present: cardinality 20 000
    data = {"acct": acct, "clicks": rng.integers(0, 1000, n)}
    seg = ImmutableSegment.create("skew", data, {"acct": "INT", "clicks": "INT"})
    t = Table("t", [seg])
    q = parse("SELECT COUNT(*), SUM(clicks) FROM t WHERE acct IN (777)")
    g = gpu_engine.execute(t, q)
    assert gpu_engine.last_timing().scan_launches == 1, "expected the rerun without the stream"
    tr = gpu_engine.last_trace()   # the recording names the re-run and its reason
    assert tr["reruns"] == 1 and tr["rerun_reasons"] == 1 and "stream" not in tr["path"] and tr["stream_leaf"] is None
    o = oracle_engine.execute(t, q)
    assert_same_result(g, o, table=t)
    assert g.stats.num_docs_scanned == o.stats.num_docs_scanned > 0.7 * n


def test_stream_multi_leaf_ssb_shape(gpu_engine, oracle_engine):
    """Config 3 shape: no single leaf is selective (14 % / 27 % / 48 %), the three together pass ~1.8 %: the first
    is streamed at its bit width, the other two are tested on its survivors inside the stream kernel."""
    from pinot_amd import synth
    segs = [synth.make_segment_np(synth.SSB_LINEORDER, s, n) for s, n in enumerate((120_007, 64_000, 99_999))]
    t = Table("lineorder", segs)
    q = parse(synth.ssb_q11_query())
    g = gpu_engine.execute(t, q)
    assert gpu_engine.last_timing().scan_launches == 2, "the selective stream did not run"
    o = oracle_engine.execute(t, q)
    assert g.stats.num_docs_scanned > 0
    assert_same_result(g, o, table=t)
    n = gpu_engine.execute(t, q, flags=abi.PG_PLAN_VALUE_SETS | abi.PG_PLAN_NO_STREAM)
    assert_same_result(g, n, table=t)


@pytest.fixture(scope="module")
def wide_table():
    """acct cardinality ~290 K per segment: an IN list's LDS filter bitmap must be coarse (dictId >> shift), its
    candidates resolved through the exact global LUT (an exact LDS hash table beside a coarser bitmap measured slower:
    config 2's stream 0.54 -> 0.71 ms)."""
    segs = []
    for s, n in enumerate((300_000, 250_007)):
        rng = np.random.default_rng(100 + s)
        data = {"acct": rng.integers(0, 4_000_000, n), "day": rng.integers(0, 365, n),
                "clicks": rng.integers(0, 1000, n)}
        segs.append(ImmutableSegment.create(f"w{s}", data, {"acct": "INT", "day": "INT", "clicks": "INT"}))
    return Table("t", segs)


@pytest.mark.parametrize("k", [10, 1000, 3000])
def test_stream_in_list_coarse_bitmap(k, wide_table, gpu_engine, oracle_engine):
    ids = _in_list(k, seed=k, hi=4_000_000)
    for sql in (f"SELECT COUNT(*), SUM(clicks) FROM t WHERE acct IN ({ids})",
                # the IN list as a further AND leaf tested on the survivors of a selective range
                f"SELECT day, COUNT(*) FROM t WHERE day < 10 AND acct IN ({ids}) GROUP BY day ORDER BY day LIMIT 20"):
        q = parse(sql)
        g = gpu_engine.execute(wide_table, q)
        assert gpu_engine.last_timing().scan_launches == 2, "the selective stream did not run"
        assert_same_result(g, oracle_engine.execute(wide_table, q), table=wide_table)
        n = gpu_engine.execute(wide_table, q, flags=abi.PG_PLAN_VALUE_SETS | abi.PG_PLAN_NO_STREAM)
        assert_same_result(g, n, table=wide_table)


@pytest.mark.parametrize("pre", ["0", "1"])
def test_stream_further_leaves_slice_prefetch(pre, table, monkeypatch, gpu_engine, oracle_engine):
    """Config 3's shape: a wide range drives the stream (28 % pass) and the AND's further packed leaves are tested on
    its survivors from per-wave LDS slices; PG_STREAM_STAGE_PRE=1 DMAs every further leaf's slice at the start of each
    group round instead of after the driving test (off by default).  Same answers as the oracle either way."""
    monkeypatch.setenv("PG_STREAM_STAGE_PRE", pre)
    for sql in ["SELECT SUM(clicks * imps), COUNT(*) FROM t WHERE day BETWEEN 18000 AND 18100 "
                "AND clicks BETWEEN 1 AND 30 AND acct < 100000",
                "SELECT tag, SUM(imps) FROM t WHERE day BETWEEN 18100 AND 18250 AND clicks < 20 AND NOT tag = 't3' "
                "GROUP BY tag ORDER BY tag LIMIT 100"]:
        q = parse(sql)
        g = gpu_engine.execute(table, q)
        assert gpu_engine.last_timing().scan_launches == 2, "the selective stream did not run"
        assert_same_result(g, oracle_engine.execute(table, q), table=table)
