"""Raw (no-dictionary) fixed-width forward index: the reference's chunked format
(BaseChunkSVForwardIndexWriter / FixedByteChunkSVForwardIndexReader / FixedBytePower2ChunkSVForwardIndexReader),
raw-value predicates and aggregations over it, on the oracle and the device.

Pinned by the reference's own bytes: tests/golden/raw_fwd/ holds the three fixtures of
FixedByteChunkSVForwardIndexTest.java:255-291 (fixedByteSVRDoubles.v1: v1 SNAPPY, 10 009 doubles i;
fixedByteCompressed.v2: v2 SNAPPY, and fixedByteRaw.v2: v2 PASS_THROUGH, 2 000 doubles i + 100.2356).

The LZ4 / LZ4_LENGTH_PREFIXED / ZSTANDARD chunk decoders of libpinot_gpu (pg_codec.hip, pg_chunk_decompress) are pinned
against independent encoders: the system liblz4 / libzstd (the native libraries lz4-java 1.8.0 and zstd-jni 1.4.9-5 wrap)
compress the data, the library must return it unchanged.  The reference holds no LZ4 / ZSTD chunk bytes."""
import os

import numpy as np
import pytest

from pinot_amd import abi
from pinot_amd.plan import Table, reduce_to_rows
from pinot_amd.query import parse
from pinot_amd.segment import (CHUNK_CODECS, Column, ImmutableSegment, chunk_compress, chunk_decompress,
                               raw_forward_bytes, raw_forward_header, raw_forward_values)

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "raw_fwd")
FIXTURES = [("fixedByteSVRDoubles.v1", 10009, 0.0, 1), ("fixedByteCompressed.v2", 2000, 100.2356, 1),
            ("fixedByteRaw.v2", 2000, 100.2356, 0)]


def _fixture(name):
    with open(os.path.join(GOLDEN, name), "rb") as f:
        return f.read()


@pytest.mark.parametrize("name,n,start,compression", FIXTURES)
def test_reference_fixtures_decode(name, n, start, compression):
    b = _fixture(name)
    assert raw_forward_header(b)["compression"] == compression
    assert np.array_equal(raw_forward_values(b, "DOUBLE", n), np.arange(n) + start)


@pytest.mark.parametrize("version", [2, 3, 4])
@pytest.mark.parametrize("dtype", ["INT", "LONG", "FLOAT", "DOUBLE"])
def test_writer_round_trip(version, dtype):
    rng = np.random.default_rng(version)
    vals = rng.integers(-10 ** 6, 10 ** 6, 2345).astype({"INT": np.int32, "LONG": np.int64, "FLOAT": np.float32,
                                                          "DOUBLE": np.float64}[dtype])
    b = raw_forward_bytes(vals, dtype, version, 1024 if version == 4 else 1000)
    h = raw_forward_header(b)
    assert (h["version"], h["total"], h["compression"]) == (version, 2345, 0)
    assert np.array_equal(raw_forward_values(b, dtype), vals)


def _codec_cases():
    rng = np.random.default_rng(11)
    cases = [b"", b"a", b"abc" * 1000, bytes(70000), rng.integers(0, 256, 5000, dtype=np.uint8).tobytes(),
             np.arange(20000, dtype=">i4").tobytes(), rng.normal(size=9000).astype(">f8").tobytes(),
             np.sort(rng.integers(0, 10 ** 9, 8000)).astype(">i8").tobytes(), b"The quick brown fox. " * 3000]
    for _ in range(12):
        n, k = int(rng.integers(1, 60000)), int(rng.integers(1, 300))
        cases.append((rng.integers(0, k, n) * int(rng.integers(1, 1000))).astype(rng.choice([">i4", ">i8"])).tobytes())
    return cases


@pytest.mark.parametrize("codec", ["SNAPPY", "LZ4", "LZ4_LENGTH_PREFIXED", "ZSTANDARD"])
def test_chunk_codecs_round_trip_independent_encoders(codec):
    """ChunkDecompressor.decompress restated in C (pg_chunk_decompress) returns what an independent encoder packed:
    liblz4 for LZ4 (block; length-prefixed = LZ4CompressorWithLength), libzstd level 3 (zstd-jni's default) and
    further levels / strategies for ZSTANDARD."""
    code = CHUNK_CODECS[codec]
    for b in _codec_cases():
        assert chunk_decompress(code, chunk_compress(code, b), len(b)) == b
    if codec == "ZSTANDARD":  # other levels exercise other block / table modes (raw, RLE, repeat, 4-stream literals)
        import ctypes as C
        zs = C.CDLL("libzstd.so.1")
        zs.ZSTD_compressBound.restype = C.c_size_t
        zs.ZSTD_compress.restype = C.c_size_t
        zs.ZSTD_compress.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_int]
        for lvl in (-5, 1, 9, 19):
            for b in _codec_cases():
                cap = zs.ZSTD_compressBound(C.c_size_t(len(b)))
                buf = C.create_string_buffer(max(cap, 1))
                n = zs.ZSTD_compress(buf, cap, b, len(b), lvl)
                assert chunk_decompress(code, buf.raw[:n], len(b)) == b, (lvl, len(b))


def test_chunk_codec_rejects_corrupt_input():
    from pinot_amd.gpu import PinotGpuError
    from pinot_amd.plan import UnsupportedQuery as U
    data = np.arange(5000, dtype=">i8").tobytes()
    for codec in ("LZ4", "ZSTANDARD", "SNAPPY"):
        c = bytearray(chunk_compress(CHUNK_CODECS[codec], data))
        c[len(c) // 2] ^= 0xFF
        c = bytes(c[:len(c) - 3])
        with pytest.raises((PinotGpuError, U)):
            chunk_decompress(CHUNK_CODECS[codec], c, len(data))


@pytest.mark.parametrize("codec", ["SNAPPY", "LZ4", "LZ4_LENGTH_PREFIXED", "ZSTANDARD"])
@pytest.mark.parametrize("version", [2, 3, 4])
def test_compressed_writer_round_trip(codec, version):
    rng = np.random.default_rng(version)
    vals = rng.integers(-10 ** 4, 10 ** 4, 23456).astype(np.int64)
    b = raw_forward_bytes(vals, "LONG", version, 1000, compression=codec)
    h = raw_forward_header(b)
    assert (h["version"], h["total"], h["compression"]) == (version, 23456, CHUNK_CODECS[codec])
    assert np.array_equal(raw_forward_values(b, "LONG"), vals)


def test_v4_chunks_are_a_power_of_two():
    """FixedBytePower2ChunkSVForwardIndexReader finds doc d in chunk d >>> numberOfTrailingZeros(numDocsPerChunk): a v4
    file is written with a power-of-two chunk size, and that lookup finds every doc's value in its chunk."""
    vals = np.arange(10_000, dtype=np.int32) * 3 - 7
    b = raw_forward_bytes(vals, "INT", 4, 1000, compression="LZ4")
    h = raw_forward_header(b)
    dpc = h["docs_per_chunk"]
    assert dpc == 1024 and dpc & (dpc - 1) == 0
    shift = dpc.bit_length() - 1
    ends = list(h["offsets"][1:]) + [len(b)]
    for d in (0, 1, 1023, 1024, 5000, 9999):
        c = d >> shift
        chunk = chunk_decompress(h["compression"], b[h["offsets"][c]:ends[c]], dpc * 4)
        assert np.frombuffer(chunk, dtype=">i4")[d & (dpc - 1)] == vals[d]
    bad = bytearray(b)
    bad[8:12] = (1000).to_bytes(4, "big")
    with pytest.raises(ValueError):
        raw_forward_header(bytes(bad))


def test_default_raw_dimension_is_lz4(oracle_engine):
    """SegmentColumnarIndexCreator.getColumnCompressionType (:356-368): a raw DIMENSION column is LZ4 by default, a
    METRIC PASS_THROUGH; the LZ4 column loads (decoded by the library) and queries match numpy."""
    rng = np.random.default_rng(3)
    n = 30_011
    d = rng.integers(-1000, 1000, n)
    m = rng.integers(0, 50, n)
    seg = ImmutableSegment.create("lz", {"d": d, "m": m}, {"d": "INT", "m": "LONG"}, no_dictionary=("d", "m"),
                                  field_types={"d": "DIMENSION", "m": "METRIC"})
    assert raw_forward_header(seg.columns["d"].fwd)["compression"] == CHUNK_CODECS["LZ4"]
    assert raw_forward_header(seg.columns["m"].fwd)["compression"] == CHUNK_CODECS["PASS_THROUGH"]
    assert np.array_equal(raw_forward_values(seg.columns["d"].fwd, "INT"), d)
    r = oracle_engine.execute(Table("t", [seg]), "SELECT COUNT(*), SUM(m), MIN(d) FROM t WHERE d > 100")
    k = d > 100
    assert r.rows[()] == [int(k.sum()), float(m[k].sum()), float(d[k].min())]


def _raw_segments(n_segs=3, rows=50_000, seed=7, codecs=None):
    rng = np.random.default_rng(seed)
    segs = []
    for s in range(n_segs):
        n = rows + 1013 * s
        data = {"k": rng.integers(0, 40, n), "m_int": rng.integers(-5000, 5000, n),
                "m_long": rng.integers(-2 ** 40, 2 ** 40, n), "m_float": rng.normal(size=n).astype(np.float32),
                "m_double": rng.normal(size=n) * 1e3, "u": rng.integers(0, 300, n),
                # a raw LONG key of a timestamp-like range (~1e9 values: hashed device state)
                "ts": 1_600_000_000_000 + rng.integers(0, 10 ** 9, n) // 997 * 997,
                # raw FLOAT / DOUBLE keys and a LONG key wider than 2^32 (derived dictionary encodings on the device)
                "g_float": (rng.integers(0, 50, n) * 0.25 - 3.0).astype(np.float32),
                "g_double": rng.integers(-3000, 3000, n) * 0.125 + 1e-3,
                "wide": rng.integers(0, 300, n) * 2 ** 40 - 2 ** 45}
        segs.append(ImmutableSegment.create(
            f"r{s}", data, {"k": "INT", "m_int": "INT", "m_long": "LONG", "m_float": "FLOAT", "m_double": "DOUBLE",
                            "u": "INT", "ts": "LONG", "g_float": "FLOAT", "g_double": "DOUBLE", "wide": "LONG"},
            no_dictionary=("m_int", "m_long", "m_float", "m_double", "u", "ts", "g_float", "g_double", "wide"),
            raw_version=2 + s % 3,
            raw_compression=codecs))
    return segs


RAW_QUERIES = [
    "SELECT COUNT(*), SUM(m_int), MIN(m_long), MAX(m_double), AVG(m_float) FROM t",
    "SELECT SUM(m_long), COUNT(*) FROM t WHERE m_int > 100 AND m_int <= 4000",
    "SELECT MAX(m_int), MIN(m_double) FROM t WHERE m_double BETWEEN -200.5 AND 300.25",
    "SELECT COUNT(*), SUM(m_double) FROM t WHERE m_float < 0 OR m_int IN (1, 2, 3, 4, 5, 6, 7)",
    "SELECT COUNT(*) FROM t WHERE m_int NOT IN (0, 1, 2) AND NOT m_long < 0",
    "SELECT COUNT(*), SUM(m_int) FROM t WHERE m_int = 42 OR m_int <> -42",
    "SELECT k, SUM(m_int), MAX(m_double), COUNT(*) FROM t WHERE m_float >= 0.5 GROUP BY k",
    "SELECT k, AVG(m_long), MIN(m_float) FROM t WHERE k < 20 AND m_int NOT BETWEEN -100 AND 100 GROUP BY k",
    "SELECT SUM(m_int * m_double), SUM(m_int + k), MIN(m_long - m_int) FROM t WHERE m_double > 0",
    "SELECT DISTINCTCOUNT(u), COUNT(*) FROM t WHERE m_int < 0",
    "SELECT k, DISTINCTCOUNT(u) FROM t GROUP BY k",
    "SELECT MIN(m_int), MAX(m_long), COUNT(*) FROM t",                     # non-scan: column metadata min / max
    # raw (no-dictionary) group keys: NoDictionarySingleColumnGroupKeyGenerator / NoDictionaryMultiColumnGroupKeyGenerator
    "SELECT u, COUNT(*), SUM(m_int), MAX(m_double) FROM t GROUP BY u",
    "SELECT m_int, COUNT(*), MIN(m_long) FROM t WHERE k < 10 GROUP BY m_int",
    "SELECT k, u, COUNT(*), AVG(m_float) FROM t WHERE m_double > 0 GROUP BY k, u",
    "SELECT ts, COUNT(*), SUM(m_long) FROM t WHERE m_int > 3000 GROUP BY ts",
    "SELECT u, m_int, COUNT(*) FROM t WHERE m_int BETWEEN -50 AND 50 GROUP BY u, m_int",
    "SELECT u, DISTINCTCOUNT(k), COUNT(*) FROM t GROUP BY u",
    # raw FLOAT / DOUBLE / wide LONG keys (the generators' Float2Int / Double2Int / Long2Int maps): grouped through a
    # host-built dictionary encoding of the raw values (KeySpace.build, PG_COL_DERIVED)
    "SELECT g_float, COUNT(*), SUM(m_int), MAX(m_double) FROM t GROUP BY g_float",
    "SELECT g_double, k, COUNT(*), AVG(m_float) FROM t WHERE m_int > 0 GROUP BY g_double, k",
    "SELECT wide, COUNT(*), MIN(m_long), SUM(wide) FROM t WHERE g_float < 5 GROUP BY wide",
    "SELECT g_float, wide, COUNT(*) FROM t WHERE m_double > 100 GROUP BY g_float, wide",
    "SELECT k, DISTINCTCOUNT(g_double), DISTINCTCOUNT(wide) FROM t GROUP BY k",
    "SELECT DISTINCTCOUNT(g_float), DISTINCTCOUNT(g_double), COUNT(*) FROM t WHERE k < 30",
    "SELECT g_double, SUM(g_double), COUNT(*) FROM t WHERE g_double > 100 GROUP BY g_double",
    # a raw integer range too wide for a dense value bitmap (~1e9 values): DISTINCTCOUNT over the derived encoding
    "SELECT k, DISTINCTCOUNT(ts) FROM t WHERE m_int > 4000 GROUP BY k",
    "SELECT DISTINCTCOUNT(ts), DISTINCTCOUNT(m_int), COUNT(*) FROM t",
]




@pytest.fixture(scope="module")
def raw_table():
    return Table("t", _raw_segments())


@pytest.mark.parametrize("sql", RAW_QUERIES)
def test_raw_queries_oracle_vs_numpy(sql, oracle_engine, raw_table):
    """The oracle's raw path against a numpy evaluation of the same query over the decoded values."""
    q = parse(sql)
    res = oracle_engine.execute(raw_table, q)
    vals = {c: np.concatenate([s.columns[c].raw_values if s.columns[c].dictionary is None
                               else s.columns[c].dictionary.values[s.columns[c].dict_ids] for s in raw_table.segments])
            for c in raw_table.segments[0].columns}
    mask = _np_filter(q.filter, vals)
    if not q.group_by:
        row = res.rows.get((), None)
        for ag, v in zip(q.aggregations, row):
            x = _np_agg(ag, vals, mask)
            if ag.function == "AVG":
                assert v[1] == x[1] and np.isclose(v[0], x[0], rtol=1e-9)
            elif ag.function == "DISTINCTCOUNT":
                assert v == x
            else:
                assert np.isclose(v, x, rtol=1e-9, atol=0) or v == x, (ag, v, x)
    else:
        kv = np.stack([vals[c][mask] for c in q.group_by], axis=1)
        uniq, inv = np.unique(kv, axis=0, return_inverse=True)
        inv = inv.reshape(-1)
        order = np.argsort(inv, kind="stable")
        bounds = np.searchsorted(inv[order], np.arange(len(uniq) + 1))
        sel = np.flatnonzero(mask)
        for gi in range(len(uniq)):
            m2 = np.zeros_like(mask)
            m2[sel[order[bounds[gi]:bounds[gi + 1]]]] = True
            for ag, v in zip(q.aggregations, res.rows[tuple(x.item() for x in uniq[gi])]):
                x = _np_agg(ag, vals, m2)
                if ag.function == "AVG":
                    assert v[1] == x[1] and np.isclose(v[0], x[0], rtol=1e-9)
                elif ag.function == "DISTINCTCOUNT":
                    assert v == x
                else:
                    assert np.isclose(v, x, rtol=1e-9) or v == x, (ag, uniq[gi], v, x)
        assert len(res.rows) == len(uniq)


def _np_filter(f, vals):
    n = len(next(iter(vals.values())))
    if f is None:
        return np.ones(n, dtype=bool)
    if f.type == "AND":
        m = np.ones(n, dtype=bool)
        for c in f.children:
            m &= _np_filter(c, vals)
        return m
    if f.type == "OR":
        m = np.zeros(n, dtype=bool)
        for c in f.children:
            m |= _np_filter(c, vals)
        return m
    if f.type == "NOT":
        return ~_np_filter(f.children[0], vals)
    p = f.predicate
    v = vals[p.column]
    conv = (lambda x: np.float32(float(x))) if v.dtype == np.float32 else float
    if p.type in ("EQ", "IN"):
        return np.isin(v, [conv(x) for x in p.values])
    if p.type in ("NOT_EQ", "NOT_IN"):
        return ~np.isin(v, [conv(x) for x in p.values])
    m = np.ones(v.size, dtype=bool)
    if p.lower != "*":
        m &= (v >= conv(p.lower)) if p.lower_inclusive else (v > conv(p.lower))
    if p.upper != "*":
        m &= (v <= conv(p.upper)) if p.upper_inclusive else (v < conv(p.upper))
    return m


def _np_agg(ag, vals, mask):
    f = ag.function
    if f == "COUNT":
        return int(mask.sum())
    e = ag.arg
    x = vals[e.cols[0]][mask].astype(np.float64)
    if e.op == "MUL":
        x = x * vals[e.cols[1]][mask]
    elif e.op == "ADD":
        x = x + vals[e.cols[1]][mask]
    elif e.op == "SUB":
        x = x - vals[e.cols[1]][mask]
    if f == "SUM":
        return float(np.sum(x))
    if f == "MIN":
        return float(x.min()) if x.size else float("inf")
    if f == "MAX":
        return float(x.max()) if x.size else float("-inf")
    if f == "AVG":
        return (float(np.sum(x)), int(x.size))
    if f == "DISTINCTCOUNT":
        return set(vals[e.cols[0]][mask].tolist())
    raise ValueError(f)


def test_raw_store_round_trip(tmp_path):
    """V1 (`<col>.sv.raw.fwd`, hasDictionary = false) and V3 (`forward_index` in columns.psf) stores load the raw
    columns back unchanged."""
    seg = _raw_segments(1, 5000)[0]
    for writer, sub in ((seg.write_v1, "v1"), (seg.write_v3, "v3")):
        writer(str(tmp_path / sub))
        back = ImmutableSegment.load(str(tmp_path / sub))
        for c in ("m_int", "m_long", "m_float", "m_double"):
            assert back.columns[c].dictionary is None
            assert np.array_equal(back.columns[c].raw_values, seg.columns[c].raw_values)
        assert os.path.exists(tmp_path / "v1" / "m_int.sv.raw.fwd") if sub == "v1" else True


def _first_seen_groups(table, cols, where, limit):
    """NoDictionarySingleColumnGroupKeyGenerator.getKeyForValue (:416-424) / NoDictionaryMultiColumnGroupKeyGenerator
    .getGroupIdForKey (:318-328) restated in Python: per segment, the value tuples of the matching docs get group ids in
    first-seen doc order until numGroupsLimit exist; later new tuples are dropped (INVALID_ID).  -> {tuple: doc count}
    merged over the segments by value."""
    out = {}
    for s in table.segments:
        v = [s.columns[c].raw_values if s.columns[c].dictionary is None
             else np.asarray(s.columns[c].dictionary.values)[s.columns[c].dict_ids] for c in cols]
        m = where(s)
        seen = {}
        for row in zip(*(x[m].tolist() for x in v)):
            if row in seen:
                seen[row] += 1
            elif len(seen) < limit:
                seen[row] = 1
        for key, c in seen.items():
            out[key] = out.get(key, 0) + c
    return out


@pytest.mark.parametrize("cols,limit", [(("m_int",), 700), (("u", "k"), 1500), (("ts",), 2000), (("g_double",), 2000),
                                        (("g_float", "wide"), 3000)])
def test_raw_group_by_limit_is_first_seen(cols, limit, oracle_engine, raw_table):
    """A raw key's groups under an instance numGroupsLimit: the first `limit` distinct keys in doc order per segment
    (the reference's no-dictionary generators have no array-based holder, so a small key range truncates too), then
    merged by value; numGroupsLimitReached when a segment reached the limit."""
    from pinot_amd.plan import InstanceConfig
    cfg = InstanceConfig(num_groups_limit=limit, max_init_group_holder_capacity=min(limit, 10_000))
    q = parse(f"SELECT {', '.join(cols)}, COUNT(*) FROM t WHERE m_double > -500 GROUP BY {', '.join(cols)}")
    res = oracle_engine.execute(raw_table, q, config=cfg)
    want = _first_seen_groups(raw_table, cols, lambda s: s.columns["m_double"].raw_values > -500, limit)
    assert {k: v[0] for k, v in res.rows.items()} == want
    assert res.groups_limit_reached


def test_raw_key_spaces_order_by_value():
    """Derived key spaces: the table's distinct raw values in the reference's key order (Double.compare: -0.0 below
    0.0, one NaN above +inf), keymaps from every segment's sorted distinct values to the global ids."""
    from pinot_amd.plan import KeySpace, order_keys
    d = np.array([3.5, -0.0, 0.0, np.nan, -np.inf, np.inf, -2.25, 3.5, np.nan], dtype=np.float64)
    assert np.all(np.diff(order_keys(np.array([-np.inf, -2.25, -0.0, 0.0, 3.5, np.inf, np.nan]))) > 0)
    segs = [ImmutableSegment.create(f"s{i}", {"x": v}, {"x": "DOUBLE"}, no_dictionary=("x",))
            for i, v in enumerate((d[:5], d[4:]))]
    ks = KeySpace.build("x", [s.columns["x"] for s in segs])
    assert ks.kind == abi.PG_KEY_KEYMAP and ks.cardinality == 7
    vals = ks.values
    assert vals[:6] == [-np.inf, -2.25, 0.0, 0.0, 3.5, np.inf] and np.isnan(vals[6])
    assert np.signbit(vals[2]) and not np.signbit(vals[3])
    for s, (u, ids), km in zip(segs, ks.derived, ks.keymaps):
        raw = s.columns["x"].raw_values
        got = np.asarray(vals)[km[ids]]
        assert np.array_equal(got, raw, equal_nan=True) and np.array_equal(np.signbit(got), np.signbit(raw))
    # a LONG key wider than 2^32 values: derived too; a narrow one stays a value-offset space
    wide = ImmutableSegment.create("w", {"x": np.array([-2 ** 40, 5, 2 ** 40])}, {"x": "LONG"}, no_dictionary=("x",))
    assert KeySpace.build("x", [wide.columns["x"]]).values == [-2 ** 40, 5, 2 ** 40]
    narrow = ImmutableSegment.create("n", {"x": np.array([-7, 5, 9])}, {"x": "LONG"}, no_dictionary=("x",))
    assert KeySpace.build("x", [narrow.columns["x"]]).kind == abi.PG_KEY_VALUE_OFFSET


@pytest.mark.gpu
@pytest.mark.parametrize("cols,limit", [(("m_int",), 700), (("u", "k"), 1500), (("ts",), 2000), (("g_double",), 2000),
                                        (("g_float", "wide"), 3000)])
def test_raw_group_by_limit_gpu(cols, limit, gpu_engine, oracle_engine, raw_table):
    """The device's per-segment truncation of raw keys equals the oracle's first-seen groups (and the limit flag)."""
    from helpers import assert_same_result
    from pinot_amd.plan import InstanceConfig
    cfg = InstanceConfig(num_groups_limit=limit, max_init_group_holder_capacity=min(limit, 10_000))
    q = parse(f"SELECT {', '.join(cols)}, COUNT(*), SUM(m_int) FROM t WHERE m_double > -500 GROUP BY {', '.join(cols)}")
    g, o = gpu_engine.execute(raw_table, q, config=cfg), oracle_engine.execute(raw_table, q, config=cfg)
    assert_same_result(g, o, table=raw_table)
    assert g.groups_limit_reached == o.groups_limit_reached


def _fixture_segment(name, n):
    """A segment whose DOUBLE metric is the reference's fixture bytes as they are (its own chunks and codec)."""
    b = _fixture(name)
    vals = raw_forward_values(b, "DOUBLE", n)
    col = Column("v", "DOUBLE", True, None, n, 0, False, n, 0, b, None, "METRIC", raw_values=vals,
                 raw_cardinality=n)
    seg = ImmutableSegment.create("f", {"k": np.arange(n) % 3}, {"k": "INT"})
    seg.columns["v"] = col
    return seg


@pytest.mark.gpu
@pytest.mark.parametrize("sql", RAW_QUERIES)
def test_raw_queries_gpu(sql, gpu_engine, oracle_engine, raw_table):
    from helpers import assert_same_result
    q = parse(sql)
    assert_same_result(gpu_engine.execute(raw_table, q), oracle_engine.execute(raw_table, q), table=raw_table)


@pytest.mark.gpu
@pytest.mark.parametrize("name,n,start,compression", FIXTURES)
def test_reference_fixture_bytes_on_device(name, n, start, compression, gpu_engine):
    """The reference's fixture bytes uploaded as they are (SNAPPY chunks decoded by the library): known answers."""
    seg = _fixture_segment(name, n)
    t = Table("f", [seg])
    q = parse("SELECT COUNT(*), SUM(v), MIN(v), MAX(v) FROM f WHERE v >= 10")
    exp = np.arange(n) + start
    exp = exp[exp >= 10]
    row = gpu_engine.execute(t, q).rows[()]
    assert row[0] == exp.size and row[2] == exp.min() and row[3] == exp.max()
    assert np.isclose(row[1], exp.sum(), rtol=1e-12)


CODEC_MIX = {"m_int": "LZ4", "m_long": "ZSTANDARD", "m_float": "LZ4_LENGTH_PREFIXED", "m_double": "SNAPPY",
             "u": "ZSTANDARD"}


@pytest.mark.gpu
@pytest.mark.parametrize("sql", RAW_QUERIES)
def test_compressed_raw_columns_gpu(sql, gpu_engine, oracle_engine):
    """LZ4 / ZSTANDARD / LZ4_LENGTH_PREFIXED / SNAPPY chunks decoded by the library at upload: the device results equal
    the oracle's over the same segments."""
    from helpers import assert_same_result
    t = _compressed_table()
    q = parse(sql)
    assert_same_result(gpu_engine.execute(t, q), oracle_engine.execute(t, q), table=t)


_COMPRESSED = []


def _compressed_table():
    if not _COMPRESSED:
        _COMPRESSED.append(Table("t", _raw_segments(3, 40_000, seed=9, codecs=CODEC_MIX)))
    return _COMPRESSED[0]


def test_chunk_decoders_fuzzed_under_sanitizers(tmp_path):
    """Malformed chunks (truncated, bit-flipped, overwritten, short output buffers; a few hundred per codec and chunk)
    through the decoders built with -fsanitize=address,undefined: every one decodes or is rejected, none reads or
    writes out of bounds (tests/test_sanitizers.py, tests/sanitize/codec_fuzz.cpp)."""
    import subprocess
    from test_sanitizers import SAN, test_chunk_decoders_under_sanitizers
    subprocess.run(["make", "-s", "-C", SAN], check=True)
    test_chunk_decoders_under_sanitizers(os.path.join(SAN, "build"), tmp_path)
