"""Multi-rank combine on CPU (gloo, world_size 2): the collective logic pinot_amd.combine runs over RCCL on GPUs.

* allreduce_state: SUM / MIN / MAX semantics per dense state array (the device partials' merge), including the exact
  fixed-point double sums as 32-bit limbs (pg_partials_copy's form): one SUM all-reduce, then the carries folded, gives
  the exact 128-bit sum on every rank.
* gather_merge_results: sparse value-keyed merge; segments sharded over ranks merge to the single-process answer
  (checked against the CPU oracle over the whole table and the reference's known answers)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _worker_state(rank, world, port, q):
    _init(rank, world, port)
    from pinot_amd.combine import allreduce_state
    g = torch.Generator().manual_seed(rank)
    rng = np.random.default_rng(100 + rank)
    # 20 signed 128-bit sums per rank (SK_FX pairs), in pg_partials_copy's limb form: limb k = bits [32k, 32k + 32)
    vals = [int(x) for x in rng.integers(-(1 << 62), 1 << 62, 20)]
    vals = [v * (1 << 60) + int(w) for v, w in zip(vals, rng.integers(0, 1 << 60, 20))]
    limbs = [((v % (1 << 128)) >> (32 * k)) & 0xFFFFFFFF for v in vals for k in range(4)]
    st = {"i64": torch.cat([torch.randint(0, 1000, (50,), generator=g), torch.tensor(limbs, dtype=torch.int64)]),
          "mn": torch.randint(-100, 100, (30,), generator=g), "mx": torch.randint(-100, 100, (30,), generator=g),
          "stats": torch.tensor([rank + 1] * 6)}
    orig = {k: v.clone() for k, v in st.items()}
    allreduce_state(st)
    allg = {}
    for k, v in orig.items():
        parts = [torch.empty_like(v) for _ in range(world)]
        dist.all_gather(parts, v)
        allg[k] = torch.stack(parts)
    every = [None] * world
    dist.all_gather_object(every, vals)
    summed = st["i64"][50:].tolist()
    folded = []  # fx_limbs_kernel's fold: carry each limb's excess upward, mod 2^128, as a signed value
    for i in range(20):
        c, w = 0, 0
        for k in range(4):
            t = summed[4 * i + k] + c
            w |= (t & 0xFFFFFFFF) << (32 * k)
            c = t >> 32
        folded.append(w - (1 << 128) if w >> 127 else w)
    exact = [sum(vs[i] for vs in every) for i in range(20)]
    ok = (torch.equal(st["i64"], allg["i64"].sum(0)) and folded == exact
          and torch.equal(st["mn"], allg["mn"].min(0).values) and torch.equal(st["mx"], allg["mx"].max(0).values)
          and torch.equal(st["stats"], torch.tensor([world * (world + 1) // 2] * 6)))
    q.put((rank, ok))
    dist.destroy_process_group()


def _worker_header(rank, world, port, q):
    """The per-step layout header (combine._layout_header): every rank sees the same error flag and the same
    fingerprint maxima / minima, so all of them take the same branch even when only one rank's layout changed."""
    _init(rank, world, port)
    from pinot_amd.combine import _layout_header
    from pinot_amd import abi
    dev = torch.device("cpu")
    same = [0, 365, 3, 0, 0, 0, 0, 3, 0]
    out = [_layout_header(None, list(same), 0, None, dev)]
    changed = list(same) if rank == 0 else [1, 1 << 20, 3, 0, 0, 0, 0, 3, 0]   # rank 1 regrew into a hash table
    out.append(_layout_header(None, changed, 0, None, dev))
    out.append(_layout_header(RuntimeError("x") if rank == 1 else None, list(same), 0, None, dev))
    # one rank's segment reached numGroupsLimit: every rank's combined result reports it
    out.append(_layout_header(None, list(same), abi.PG_RESULT_GROUPS_LIMIT_REACHED if rank == 1 else 0, None, dev))
    q.put((rank, out))
    dist.destroy_process_group()


def test_layout_header_gives_every_rank_the_same_decision():
    res = _run(_worker_header)
    (_, a), (_, b) = res
    from pinot_amd import abi
    assert a == b
    eq, chg, err, lim = a
    assert eq[0] == 0 and eq[1] == 0 and eq[2] == eq[3]        # no error, identical layouts: dense all-reduce
    assert chg[0] == 0 and chg[2][:2] != chg[3][:2] and chg[2][2:] == chg[3][2:]   # mixed modes: row exchange
    assert err[0] == 1                                         # one rank failed: every rank raises
    assert lim[1] == abi.PG_RESULT_GROUPS_LIMIT_REACHED        # the OR of the ranks' result flags


def _worker_sharded(rank, world, port, q):
    _init(rank, world, port)
    from conftest import build_sv_segment
    from oracle.oracle import OracleEngine
    from pinot_amd.combine import gather_merge_results
    from pinot_amd.plan import Table, reduce_to_rows
    from pinot_amd.query import parse
    seg = build_sv_segment()
    segs = [seg] * 4                      # the reference's 4-segment setup
    mine = segs[rank::world]              # round-robin sharding of segments over ranks
    full = Table("testTable", segs)
    out = []
    for sql in ["SELECT SUM(column1) AS v1, SUM(column3) AS v2 FROM testTable GROUP BY column9 "
                "ORDER BY v1 DESC, v2 DESC LIMIT 1",
                "SELECT column11, column12, SUM(column1), MIN(column6), DISTINCTCOUNT(column7), AVG(column3) "
                "FROM testTable GROUP BY column11, column12 ORDER BY column11, column12 LIMIT 100",
                "SELECT COUNT(*), MAX(column1), DISTINCTCOUNT(column3) FROM testTable WHERE column6 < 500000000"]:
        qc = parse(sql)
        part = OracleEngine().execute(Table("testTable", mine), qc)
        merged = gather_merge_results(part)
        whole = OracleEngine().execute(full, qc)
        out.append((reduce_to_rows(qc, merged)[1] == reduce_to_rows(qc, whole)[1],
                    merged.stats.num_docs_scanned == whole.stats.num_docs_scanned))
    q.put((rank, all(a and b for a, b in out), reduce_to_rows(parse(
        "SELECT SUM(column1) AS v1, SUM(column3) AS v2 FROM testTable GROUP BY column9 ORDER BY v1 DESC, v2 DESC "
        "LIMIT 1"), gather_merge_results(OracleEngine().execute(Table("testTable", mine), parse(
            "SELECT SUM(column1) AS v1, SUM(column3) AS v2 FROM testTable GROUP BY column9 ORDER BY v1 DESC, v2 DESC "
            "LIMIT 1"))))[1]))
    dist.destroy_process_group()


def _worker_sharded_shapes(rank, world, port, q):
    """Raw STRING / BYTES filters and keys, several multi-value keys (also under numGroupsLimit): each rank's oracle
    result over its round-robin share of the segments, merged by value, equals the single-process answer."""
    _init(rank, world, port)
    from helpers import assert_same_result
    from oracle.oracle import OracleEngine
    from pinot_amd.combine import gather_merge_results
    from pinot_amd.plan import InstanceConfig, Table
    from pinot_amd.query import parse
    from test_mv_group_by import _segments as mv_segments
    from test_raw_strings import _segments as rs_segments
    ok = True
    for segs, sqls, cfg in (
            (rs_segments(4, seed=23), ["SELECT w, k, COUNT(*), SUM(v) FROM t WHERE w > 'beta' AND b <> '0a5a' GROUP BY w, k",
                                       "SELECT u, DISTINCTCOUNT(b), MAX(v) FROM t WHERE u < 'user01500' GROUP BY u"], None),
            (mv_segments(4, seed=29), ["SELECT k, words, tags, COUNT(*), SUM(v) FROM t GROUP BY k, words, tags"], None),
            (mv_segments(4, seed=31), ["SELECT tags, words, COUNT(*), SUM(v) FROM t GROUP BY tags, words"],
             InstanceConfig.with_groups_limit(40))):
        full = Table("t", segs)
        mine = Table("t", segs[rank::world])
        for sql in sqls:
            qc = parse(sql)
            part = OracleEngine().execute(mine, qc, config=cfg) if cfg else OracleEngine().execute(mine, qc)
            merged = gather_merge_results(part)
            whole = OracleEngine().execute(full, qc, config=cfg) if cfg else OracleEngine().execute(full, qc)
            try:
                assert_same_result(merged, whole, table=full)
            except AssertionError:
                ok = False
    q.put((rank, ok))
    dist.destroy_process_group()


def _run(fn, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=fn, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(res, key=lambda r: r[0])


def test_allreduce_state_semantics():
    res = _run(_worker_state)
    assert all(ok for _, ok in res)


def test_sharded_segments_merge_to_single_process_answer(expected):
    res = _run(_worker_sharded)
    assert all(r[1] for r in res)
    # InterSegmentAggregationSingleValueQueriesTest.java:162-165 known answer, through the 2-rank merge
    assert [list(map(float, row)) for row in res[0][2]] == [[69526727335224.0, 69225631719808.0]]


def test_sharded_raw_string_and_multi_value_shapes_merge():
    res = _run(_worker_sharded_shapes)
    assert all(ok for _, ok in res)
