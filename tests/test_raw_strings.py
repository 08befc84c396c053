"""Raw (no-dictionary) STRING / BYTES columns: the var-byte chunked forward index (VarByteChunkSVForwardIndexWriter
versions 2 / 3, io/writer/impl/VarByteChunkSVForwardIndexWriter.java:38-166, 1 000 docs per chunk as
SingleValueVarByteRawIndexCreator.java:36 writes it) round-tripped through every chunk codec and both segment stores,
and such columns as group keys and DISTINCTCOUNT values (NoDictionarySingleColumnGroupKeyGenerator.java:93-129 keys
STRING / BYTES values through its Object2Int map): the device groups them through a host-built dictionary encoding
(KeySpace.build, PG_COL_DERIVED); filters on one (raw-value Equals / In / Range evaluators, String.equals / compareTo,
RangePredicateEvaluatorFactory.java:526-580) scan that encoding's per-doc ranks (plan.lower_derived_predicate).  Pinned
against a Python restatement over the decoded values (first-seen truncation under numGroupsLimit included), the GPU
against the oracle.
Byte parity of the format is unpinned (the reference holds no var-byte fixture); the layout is checked field by field."""
import struct

import numpy as np
import pytest

from pinot_amd.plan import InstanceConfig, Table, reduce_to_rows
from pinot_amd.query import parse
from pinot_amd.segment import (CHUNK_CODECS, ImmutableSegment, chunk_decompress, raw_forward_header,
                               raw_var_forward_bytes, raw_var_forward_values)

WORDS = ["alpha", "beta", "", "gamma-delta", "ünïcode", "zeta", "eta" * 20, "theta", "iota", "kappa"]


def test_var_byte_layout():
    vals = ["ab", "", "xyz", "q"]
    b = raw_var_forward_bytes(vals, "STRING", 2, docs_per_chunk=3, compression="PASS_THROUGH")
    h = raw_forward_header(b)
    assert (h["version"], h["num_chunks"], h["docs_per_chunk"], h["entry"], h["total"]) == (2, 2, 3, 3, 4)
    c0 = b[h["offsets"][0]:h["offsets"][1]]
    assert c0 == struct.pack(">3i", 12, 14, 14) + b"abxyz"            # row offsets from the chunk start, then bytes
    c1 = b[h["offsets"][1]:]
    assert c1 == struct.pack(">3i", 12, 0, 0) + b"q"                  # a partial chunk: 0 for the missing rows
    assert raw_var_forward_values(b, "STRING").tolist() == vals


@pytest.mark.parametrize("codec", sorted(CHUNK_CODECS))
@pytest.mark.parametrize("version", [2, 3])
def test_var_byte_round_trip(codec, version):
    rng = np.random.default_rng(version)
    vals = [WORDS[i] for i in rng.integers(0, len(WORDS), 2500)]
    b = raw_var_forward_bytes(vals, "STRING", version, compression=codec)
    assert raw_var_forward_values(b, "STRING").tolist() == vals
    by = [bytes([i % 256, 7]).hex() for i in rng.integers(0, 300, 1200)]
    assert raw_var_forward_values(raw_var_forward_bytes(by, "BYTES", version, compression=codec), "BYTES").tolist() == by
    if codec != "PASS_THROUGH":  # every chunk decodes on its own to its row offsets + bytes
        h = raw_forward_header(b)
        first = chunk_decompress(h["compression"], b[h["offsets"][0]:h["offsets"][1]], 1000 * (4 + h["entry"]))
        assert struct.unpack_from(">i", first, 0)[0] == 4000


def _segments(n_segs=3, seed=17):
    rng = np.random.default_rng(seed)
    segs = []
    for s in range(n_segs):
        n = 4000 + 313 * s
        data = {"w": [WORDS[i] for i in rng.integers(0, len(WORDS) - s, n)],
                "b": [bytes([int(x), 0x5a]) for x in rng.integers(0, 40, n)],
                "u": [f"user{x:05d}" for x in rng.integers(0, 3000, n)],
                "k": rng.integers(0, 6, n), "v": rng.integers(-1000, 1000, n)}
        segs.append(ImmutableSegment.create(f"rs{s}", data, {"w": "STRING", "b": "BYTES", "u": "STRING", "k": "INT",
                                                            "v": "INT"},
                                            no_dictionary=("w", "b", "u"), raw_version=2 + s % 2))
    return segs


@pytest.fixture(scope="module")
def rs_table():
    return Table("t", _segments())


QUERIES = [
    "SELECT w, COUNT(*), SUM(v), MAX(v) FROM t GROUP BY w",
    "SELECT b, k, COUNT(*), AVG(v) FROM t WHERE v > 0 GROUP BY b, k",
    "SELECT k, DISTINCTCOUNT(w), DISTINCTCOUNT(b), DISTINCTCOUNT(u) FROM t WHERE v < 500 GROUP BY k",
    "SELECT u, COUNT(*) FROM t WHERE k = 3 GROUP BY u",
    "SELECT w, SUM(v) FROM t GROUP BY w ORDER BY w DESC LIMIT 4",
]


def _vals(seg, c):
    col = seg.columns[c]
    return np.asarray(col.raw_values, dtype=object) if col.dictionary is None else \
        np.asarray(col.dictionary.values)[col.dict_ids]


def test_v1_v3_round_trip(tmp_path):
    seg = _segments(1)[0]
    for writer, sub in ((seg.write_v1, "v1"), (seg.write_v3, "v3")):
        writer(str(tmp_path / sub))
        back = ImmutableSegment.load(str(tmp_path / sub))
        for c in ("w", "b", "u"):
            assert back.columns[c].dictionary is None and back.columns[c].fwd == seg.columns[c].fwd
            assert back.columns[c].raw_values.tolist() == seg.columns[c].raw_values.tolist()


@pytest.mark.parametrize("sql", QUERIES[:4])
def test_oracle_groups_raw_strings_by_value(sql, rs_table, oracle_engine):
    q = parse(sql)
    got = oracle_engine.execute(rs_table, q)
    cols = {c: np.concatenate([_vals(s, c) for s in rs_table.segments]) for c in ("w", "b", "u", "k", "v")}
    m = np.ones(len(cols["v"]), dtype=bool)
    if "v > 0" in sql:
        m &= cols["v"] > 0
    if "v < 500" in sql:
        m &= cols["v"] < 500
    if "k = 3" in sql:
        m &= cols["k"] == 3
    want = {}
    for i in np.flatnonzero(m):
        key = tuple(cols[c][i].item() if hasattr(cols[c][i], "item") else cols[c][i] for c in q.group_by)
        want.setdefault(key, []).append(i)
    assert set(got.rows) == set(want)
    for key, idx in want.items():
        for ag, g in zip(q.aggregations, got.rows[key]):
            x = cols[ag.arg.cols[0]][idx] if ag.function != "COUNT" else None
            w = len(idx) if ag.function == "COUNT" else float(np.sum(x)) if ag.function == "SUM" else \
                float(np.max(x)) if ag.function == "MAX" else (float(np.sum(x)), len(idx)) if ag.function == "AVG" \
                else set(x.tolist())
            assert g == w, (key, ag, g, w)


def test_first_seen_truncation_of_raw_string_keys(rs_table, oracle_engine):
    """NoDictionarySingleColumnGroupKeyGenerator.getKeyForValue (:416-424): per segment the first `limit` distinct
    values in doc order, then merged by value."""
    limit = 500
    cfg = InstanceConfig.with_groups_limit(limit)
    res = oracle_engine.execute(rs_table, parse("SELECT u, COUNT(*) FROM t GROUP BY u"), config=cfg)
    want = {}
    for s in rs_table.segments:
        seen = {}
        for x in _vals(s, "u").tolist():
            if x in seen:
                seen[x] += 1
            elif len(seen) < limit:
                seen[x] = 1
        for x, c in seen.items():
            want[(x,)] = want.get((x,), 0) + c
    assert {k: v[0] for k, v in res.rows.items()} == want and res.groups_limit_reached


FILTERS = [
    ("w = 'beta'", lambda w, b, u, k, v: w == "beta"),
    ("w <> 'beta'", lambda w, b, u, k, v: w != "beta"),
    ("w = 'absent'", lambda w, b, u, k, v: False),
    ("w <> 'absent'", lambda w, b, u, k, v: True),
    ("w IN ('alpha', '', 'zeta', 'nope')", lambda w, b, u, k, v: w in ("alpha", "", "zeta")),
    ("w NOT IN ('alpha', 'kappa')", lambda w, b, u, k, v: w not in ("alpha", "kappa")),
    ("w BETWEEN 'beta' AND 'iota'", lambda w, b, u, k, v: "beta" <= w <= "iota"),
    ("w > 'eta' AND v < 100", lambda w, b, u, k, v: w > "eta" and v < 100),
    ("w >= 'zzz'", lambda w, b, u, k, v: w >= "zzz"),
    ("u < 'user01000' OR k = 2", lambda w, b, u, k, v: u < "user01000" or k == 2),
    ("b = '0a5a'", lambda w, b, u, k, v: b == "0a5a"),
    ("b IN ('0a5a', '205a', '275a') AND NOT w = 'alpha'",
     lambda w, b, u, k, v: b in ("0a5a", "205a", "275a") and w != "alpha"),
    ("b > '1f5a'", lambda w, b, u, k, v: b > "1f5a"),
]


def _decoded(table):
    return {c: np.concatenate([_vals(s, c) for s in table.segments]) for c in ("w", "b", "u", "k", "v")}


@pytest.mark.parametrize("where,pred", FILTERS, ids=[f[0] for f in FILTERS])
def test_oracle_filters_raw_strings_by_value(where, pred, rs_table, oracle_engine):
    """Scan filters on raw STRING / BYTES columns: the oracle (lowered onto each segment's derived dictionary) equals a
    per-doc evaluation of the raw values, counts and entries scanned included."""
    cols = _decoded(rs_table)
    n = len(cols["v"])
    m = np.array([bool(pred(*(cols[c][i] for c in ("w", "b", "u", "k", "v")))) for i in range(n)])
    got = oracle_engine.execute(rs_table, parse(f"SELECT COUNT(*), SUM(v) FROM t WHERE {where}"))
    assert got.rows[()][0] == int(m.sum()) and got.rows[()][1] == float(cols["v"][m].sum())
    assert got.stats.num_docs_scanned == int(m.sum())
    grouped = oracle_engine.execute(rs_table, parse(f"SELECT w, COUNT(*) FROM t WHERE {where} GROUP BY w"))
    want = {}
    for i in np.flatnonzero(m):
        want[(cols["w"][i],)] = want.get((cols["w"][i],), 0) + 1
    assert {k: r[0] for k, r in grouped.rows.items()} == want


def test_raw_string_filter_is_a_scan_of_every_doc(rs_table, oracle_engine):
    """A raw-value evaluator is never always-false (FilterPlanNode short-cuts only those): a literal no segment holds
    still scans every doc."""
    r = oracle_engine.execute(rs_table, parse("SELECT COUNT(*) FROM t WHERE w = 'absent'"))
    assert r.rows[()][0] == 0
    assert r.stats.num_entries_scanned_in_filter == sum(s.num_docs for s in rs_table.segments)


@pytest.mark.gpu
@pytest.mark.parametrize("sql", QUERIES)
def test_raw_strings_on_device(sql, rs_table, gpu_engine, oracle_engine):
    from helpers import assert_same_result
    q = parse(sql)
    g, o = gpu_engine.execute(rs_table, q), oracle_engine.execute(rs_table, q)
    if q.order_by:
        assert reduce_to_rows(q, g) == reduce_to_rows(q, o)
    else:
        assert_same_result(g, o, table=rs_table)


@pytest.mark.gpu
@pytest.mark.parametrize("where,pred", FILTERS, ids=[f[0] for f in FILTERS])
def test_raw_string_filters_on_device(where, pred, rs_table, gpu_engine, oracle_engine):
    from helpers import assert_same_result
    for sql in (f"SELECT COUNT(*), SUM(v), MAX(v) FROM t WHERE {where}",
                f"SELECT w, k, COUNT(*), MIN(v) FROM t WHERE {where} GROUP BY w, k",
                f"SELECT k, DISTINCTCOUNT(u) FROM t WHERE {where} GROUP BY k"):
        q = parse(sql)
        assert_same_result(gpu_engine.execute(rs_table, q), oracle_engine.execute(rs_table, q), table=rs_table)


@pytest.mark.gpu
def test_raw_string_truncation_on_device(rs_table, gpu_engine, oracle_engine):
    from helpers import assert_same_result
    cfg = InstanceConfig.with_groups_limit(500)
    q = parse("SELECT u, COUNT(*), SUM(v) FROM t GROUP BY u")
    g, o = gpu_engine.execute(rs_table, q, config=cfg), oracle_engine.execute(rs_table, q, config=cfg)
    assert_same_result(g, o, table=rs_table)
    assert g.groups_limit_reached == o.groups_limit_reached
