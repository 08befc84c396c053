"""Range index: the `.bitmap.range` file (RangeIndexCreator v1 written here, v1 / v2 headers
read), RangeIndexBasedFilterOperator leaves on the oracle and the device.

* Format: RangeIndexCreatorTest.java:112-130,240-290 restated as properties over 1 000 random unique values per type
  (ranges of numValuesPerRange + 1 values, "the off by one bug in v1"; a query inside one range has no full matches and
  that range's docs as partial matches; a query spanning ranges 0-2 fully matches range 1; the edge cases).
* Queries: dictionary and raw (INT / LONG / FLOAT / DOUBLE) columns with a range index against numpy, oracle vs device;
  the reference's FastFilteredCountTest intRangeCol cases with intRangeCol carrying a range index (:130).
* The v2 (bit-sliced) payload is RoaringBitmap 0.9.28's RangeBitmap, which the reference does not vendor: parity
  unpinned for its bytes; a v2 header (version, min) is accepted and answered exactly from the forward index."""
import struct

import numpy as np
import pytest

from pinot_amd import abi
from pinot_amd.plan import Table, lower_predicate, reduce_to_rows
from pinot_amd.query import parse
from pinot_amd.segment import (ImmutableSegment, range_index_header, range_index_v1_bytes, range_index_v1_docs)

_NP = {"INT": np.int32, "LONG": np.int64, "FLOAT": np.float32, "DOUBLE": np.float64}


def _unique_values(dt, n, seed):
    rng = np.random.default_rng(seed)
    if dt in ("INT", "LONG"):
        hi = 2 ** 31 - 1 if dt == "INT" else 2 ** 62
        v = rng.choice(np.arange(-5 * n, 5 * n), n, replace=False) * (hi // (10 * n))
    else:
        v = rng.random(n * 2)
        v = np.unique(v.astype(_NP[dt]))[:n]
        rng.shuffle(v)
    return np.asarray(v, dtype=_NP[dt])


@pytest.mark.parametrize("dt", ["INT", "LONG", "FLOAT", "DOUBLE"])
def test_v1_ranges_like_reference_creator_test(dt):
    n = 1000
    v = _unique_values(dt, n, {"INT": 1, "LONG": 2, "FLOAT": 3, "DOUBLE": 4}[dt])
    b = range_index_v1_bytes(v, dt)
    h = range_index_header(b)
    assert h["version"] == 1 and h["value_type"] == dt
    per = (n + 19) // 20 + 1                       # getNumValuesPerRange() + 1
    s = np.sort(v)
    split = [(s[i * per], s[(i + 1) * per - 1]) for i in range(n // per)] + [(s[(n // per) * per], s[-1])]
    assert len(h["starts"]) == len(split)
    assert np.array_equal(h["starts"], [a for a, _ in split])
    for rid, (lo, hi) in enumerate(split):     # single bucket: no full match, partial = that bucket
        full, part = range_index_v1_docs(b, lo, hi)
        assert full.size == 0
        assert np.array_equal(np.sort(v[part]), s[rid * per:rid * per + part.size])
    full, part = range_index_v1_docs(b, split[0][0], split[2][1])
    assert np.array_equal(np.sort(v[full]), s[per:2 * per])
    _, p0 = range_index_v1_docs(b, *split[0])
    _, p2 = range_index_v1_docs(b, *split[2])
    assert np.array_equal(part, np.union1d(p0, p2))
    info = np.iinfo(np.int64) if dt in ("INT", "LONG") else None
    lo_inf, hi_inf = (info.min, info.max) if info else (-np.inf, np.inf)
    full, part = range_index_v1_docs(b, lo_inf, hi_inf)
    assert full.size == n and part.size == 0
    assert range_index_v1_docs(b, lo_inf, lo_inf)[0].size == 0
    assert range_index_v1_docs(b, hi_inf, hi_inf)[1].size == 0


def test_v1_equal_values_never_split():
    v = np.repeat(np.arange(7), [500, 3, 3, 400, 1, 90, 3])
    b = range_index_v1_bytes(v, "INT")
    h = range_index_header(b)
    assert len(np.unique(h["starts"])) == len(h["starts"])
    for x in range(7):
        full, part = range_index_v1_docs(b, x, x)
        assert np.array_equal(np.union1d(full, part[v[part] == x]), np.flatnonzero(v == x))


def test_v2_header_and_bad_versions():
    h = range_index_header(struct.pack(">iq", 2, -17) + b"\0" * 8)
    assert h == {"version": 2, "min": -17}
    with pytest.raises(ValueError):
        range_index_header(struct.pack(">iq", 3, 0))


def _range_segments(n_segs=3, rows=40_000, seed=11):
    rng = np.random.default_rng(seed)
    segs = []
    for s in range(n_segs):
        n = rows + 777 * s
        data = {"k": rng.integers(0, 30, n), "d_int": rng.integers(0, 5000, n), "r_int": rng.integers(-10**5, 10**5, n),
                "r_long": rng.integers(-2 ** 40, 2 ** 40, n), "r_wide": rng.integers(-2 ** 45, 2 ** 45, n),
                "r_float": rng.normal(size=n).astype(np.float32), "r_double": rng.normal(size=n) * 1e3,
                "m": rng.integers(0, 100, n)}
        types = {"k": "INT", "d_int": "INT", "r_int": "INT", "r_long": "LONG", "r_wide": "LONG", "r_float": "FLOAT",
                 "r_double": "DOUBLE", "m": "INT"}
        segs.append(ImmutableSegment.create(
            f"g{s}", data, types, no_dictionary=("r_int", "r_long", "r_wide", "r_float", "r_double"),
            range_index=("d_int", "r_int", "r_long", "r_wide", "r_float", "r_double")))
    return segs


RANGE_QUERIES = [
    "SELECT COUNT(*), SUM(m) FROM t WHERE d_int BETWEEN 100 AND 2500",
    "SELECT COUNT(*), MAX(r_int), MIN(r_int), SUM(r_int) FROM t WHERE r_int > -500 AND r_int <= 70000",
    "SELECT COUNT(*), SUM(r_long), AVG(r_int) FROM t WHERE r_long < 12345678 AND d_int >= 4000",
    "SELECT COUNT(*), MIN(r_wide) FROM t WHERE r_wide >= 0",
    "SELECT COUNT(*), MAX(r_double) FROM t WHERE r_float BETWEEN -0.5 AND 0.25 OR r_double > 1500",
    "SELECT COUNT(*) FROM t WHERE NOT r_int BETWEEN -1000 AND 1000",
    "SELECT k, COUNT(*), SUM(r_int), MAX(r_long) FROM t WHERE r_int > 0 AND d_int < 1000 GROUP BY k",
    "SELECT COUNT(*) FROM t WHERE r_int > 500000",
    "SELECT COUNT(*), DISTINCTCOUNT(r_int) FROM t WHERE r_int BETWEEN 10 AND 20",
]


@pytest.fixture(scope="module")
def range_table():
    return Table("t", _range_segments())


def test_range_leaves_are_chosen(range_table):
    seg = range_table.segments[0]
    q = parse("SELECT COUNT(*) FROM t WHERE d_int > 3 AND r_int < 5 AND r_float < 0 AND k > 3 AND d_int IN (1, 2)")
    kinds = [lower_predicate(p, seg.columns[p.column], 0).kind for p in q.filter.leaves()]
    assert kinds == [abi.PG_LEAF_RANGE_INDEX] * 3 + [abi.PG_LEAF_SV_SCAN] * 2


@pytest.mark.parametrize("sql", RANGE_QUERIES)
def test_range_index_queries_oracle_vs_scan(sql, oracle_engine, range_table):
    """The range-index leaves (v1: full buckets + scanned edge buckets) answer what the scan answers."""
    q = parse(sql)
    res = oracle_engine.execute(range_table, q)
    no_idx = Table("t", [ImmutableSegment(s.name, s.num_docs, {c: _strip(col) for c, col in s.columns.items()})
                         for s in range_table.segments])
    ref = oracle_engine.execute(no_idx, q)
    assert reduce_to_rows(q, res) == reduce_to_rows(q, ref)
    assert res.stats.num_docs_scanned == ref.stats.num_docs_scanned
    assert res.stats.num_entries_scanned_in_filter <= ref.stats.num_entries_scanned_in_filter


def _strip(col):
    from dataclasses import replace
    return replace(col, range_index=None)


def test_store_round_trip(tmp_path):
    seg = _range_segments(1, 3000)[0]
    for writer, sub in ((seg.write_v1, "v1"), (seg.write_v3, "v3")):
        writer(str(tmp_path / sub))
        back = ImmutableSegment.load(str(tmp_path / sub))
        for c in ("d_int", "r_int", "r_double"):
            assert back.columns[c].range_index == seg.columns[c].range_index
        assert back.columns["k"].range_index is None
    assert (tmp_path / "v1" / "r_int.bitmap.range").exists()


def _fast_count_segment_with_range():
    n = 1000
    i = np.arange(n)
    data = {"class": i % 8, "sorted": i, "intRangeCol": n - i}
    return ImmutableSegment.create("testSegment", data, {"class": "INT", "sorted": "INT", "intRangeCol": "INT"},
                                   inverted=("class",), range_index=("intRangeCol",))


def test_fast_filtered_count_range_cases_oracle(oracle_engine):
    """FastFilteredCountTest.java:283-306 with intRangeCol's range index (:130): counts as the known answers, and the
    range leaves scan no entries beyond their v1 partial buckets."""
    from test_shortcuts import CASES, _check_count
    seg = _fast_count_segment_with_range()
    t = Table("testTable", [seg, seg])
    for sql, expected in CASES:
        if "intRangeCol" in sql:
            q = parse(sql)
            res = oracle_engine.execute(t, q)
            _check_count(res, q, expected, 2)


@pytest.mark.gpu
@pytest.mark.parametrize("sql", RANGE_QUERIES)
def test_range_index_queries_gpu(sql, gpu_engine, oracle_engine, range_table):
    from helpers import assert_same_result
    q = parse(sql)
    assert_same_result(gpu_engine.execute(range_table, q), oracle_engine.execute(range_table, q), table=range_table)


@pytest.mark.gpu
def test_fast_filtered_count_range_cases_gpu(gpu_engine):
    from test_shortcuts import CASES, _check_count
    seg = _fast_count_segment_with_range()
    t = Table("testTable", [seg, seg])
    for sql, expected in CASES:
        if "intRangeCol" in sql:
            q = parse(sql)
            _check_count(gpu_engine.execute(t, q), q, expected, 2)


@pytest.mark.gpu
def test_v2_header_upload_gpu(gpu_engine, oracle_engine):
    """A v2 (bit-sliced) header: min must match the column (0 for dictIds), answers exact from the forward index."""
    rng = np.random.default_rng(5)
    n = 20000
    data = {"r": rng.integers(100, 9000, n), "d": rng.integers(0, 300, n)}
    seg = ImmutableSegment.create("v2", data, {"r": "INT", "d": "INT"}, no_dictionary=("r",))
    seg.columns["r"].range_index = struct.pack(">iq", 2, int(data["r"].min())) + b"\0" * 16
    seg.columns["d"].range_index = struct.pack(">iq", 2, 0) + b"\0" * 16
    t = Table("t", [seg])
    from helpers import assert_same_result
    for sql in ["SELECT COUNT(*), SUM(d) FROM t WHERE r BETWEEN 500 AND 4000",
                "SELECT MAX(r), COUNT(*) FROM t WHERE d < 150 AND r > 8000"]:
        q = parse(sql)
        assert_same_result(gpu_engine.execute(t, q), oracle_engine.execute(t, q), table=t)
