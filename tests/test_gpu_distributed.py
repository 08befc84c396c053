"""Two ranks on one MI355X (gloo, world_size 2, both on cuda:0): each rank runs pg_execute_partial over half of the
segments and pinot_amd.combine merges the DEVICE partial states -- the dense all-reduce path (small dense key space)
and the row-exchange path (hash states, DISTINCTCOUNT bitmaps: all_to_all of rows by owner, pg_partials_merge) -- and
the merged result must equal the CPU oracle over the whole table.  The same code runs over RCCL at N GPUs.

Double sums (test_two_ranks_double_sums_are_bit_identical): SUM / AVG over DOUBLE / FLOAT columns and expressions
accumulate as exact fixed-point integers (SK_FX), so the device result is the same bits in two runs, on 1 rank and on
2 ranks (dense all-reduce of 32-bit limbs, and the row exchange), and within 1e-9 of the oracle's sequential double
sum; +-inf / NaN inputs give IEEE's sum exactly."""
import os
import socket
import sys
import traceback

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CASES = [
    # (sql, force hash table)  -- dense all-reduce, then row exchange
    ("SELECT daysSinceEpoch, SUM(clicks), SUM(impressions) FROM adAnalytics WHERE daysSinceEpoch BETWEEN 18000 AND "
     "18089 AND accountId < 300000 GROUP BY daysSinceEpoch ORDER BY daysSinceEpoch LIMIT 400", False),
    ("SELECT COUNT(*), SUM(clicks), MIN(impressions), MAX(accountId), AVG(clicks) FROM adAnalytics "
     "WHERE accountId < 5000", False),
    ("SELECT daysSinceEpoch, COUNT(*), SUM(clicks), MIN(impressions), MAX(impressions), AVG(clicks) FROM adAnalytics "
     "WHERE clicks < 100 GROUP BY daysSinceEpoch", True),
    ("SELECT daysSinceEpoch, DISTINCTCOUNT(clicks), SUM(impressions) FROM adAnalytics WHERE accountId < 20000 "
     "GROUP BY daysSinceEpoch", False),
    ("SELECT accountId, COUNT(*), SUM(impressions) FROM adAnalytics WHERE clicks < 5 GROUP BY accountId", False),
    ("SELECT DISTINCTCOUNT(impressions), COUNT(*) FROM adAnalytics WHERE accountId < 1000", False),
    # the config-2 query itself: selective stream + list-mode scan on each rank, dense all-reduce
    ("CONFIG2", False),
    # untrimmed high-cardinality group-by (~10^5 groups with value sets): the owners' finalized rows come back as
    # flat device byte buffers (no pickled objects)
    ("SELECT accountId, COUNT(*), DISTINCTCOUNT(clicks) FROM adAnalytics WHERE clicks < 500 GROUP BY accountId", False),
]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, backend="gloo"):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        sys.path.insert(0, ROOT)
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(0)
        if backend == "nccl":  # RCCL (one rank: the box has one GPU, and RCCL refuses two ranks on one device)
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        from helpers import assert_same_result
        from oracle.oracle import OracleEngine
        from pinot_amd import abi, synth
        from pinot_amd.combine import merge_partials_across_ranks
        from pinot_amd.gpu import GpuEngine
        from pinot_amd.plan import Table
        from pinot_amd.query import parse
        eng = GpuEngine(0)
        segs = [synth.make_segment_np(synth.ADANALYTICS, s, 60_001 + 777 * s) for s in range(4)]
        table = Table("adAnalytics", segs)          # table-global key spaces: the same on every rank
        mine = segs[rank::world]
        paths = []
        for sql, force_hash in CASES:
            qc = parse(synth.adanalytics_query(1000) if sql == "CONFIG2" else sql)
            flags = abi.PG_PLAN_VALUE_SETS | (abi.PG_PLAN_HASH_GROUPS if force_hash else 0)
            plan = eng.make_plan(table, qc, segments=mine, flags=flags)
            p = eng.run_partial(plan)
            pc = p.contents
            paths.append("dense" if pc.mode == abi.PG_STATE_DENSE and pc.bitmap_words == 0 else "rows")
            merged = merge_partials_across_ranks(eng, plan, p)
            whole = OracleEngine().execute(table, qc)
            assert_same_result(merged, whole, table=table)
        # the state layout of ONE rank changes between steps (rank 0 groups in a hash table at step 2): the per-step
        # layout header gives both ranks the same decision (row exchange at step 2, dense all-reduce around it)
        qc = parse(synth.adanalytics_query(1000))
        whole = OracleEngine().execute(table, qc)
        for hash_rank0 in (False, True, False):
            flags = abi.PG_PLAN_VALUE_SETS | (abi.PG_PLAN_HASH_GROUPS if hash_rank0 and rank == 0 else 0)
            plan = eng.make_plan(table, qc, segments=mine, flags=flags)
            assert_same_result(merge_partials_across_ranks(eng, plan, eng.run_partial(plan)), whole, table=table)
        # queries in flight (bench.py --inflight): worker threads run the per-GPU part while this thread merges each
        # query across ranks in submission order
        from concurrent.futures import ThreadPoolExecutor
        plan = eng.make_plan(table, qc, segments=mine, flags=abi.PG_PLAN_VALUE_SETS)
        with ThreadPoolExecutor(3) as ex:
            for f in [ex.submit(eng.run_partial, plan) for _ in range(8)]:
                assert_same_result(merge_partials_across_ranks(eng, plan, f.result()), whole, table=table)
        q.put((rank, True, paths))
        dist.destroy_process_group()
    except Exception:
        q.put((rank, False, traceback.format_exc()))


def test_two_ranks_merge_device_partials():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    for rank, ok, info in res:
        assert ok, info
    assert "dense" in res[0][2] and "rows" in res[0][2]


def test_rccl_one_rank_merge_device_partials():
    """The same merges over RCCL (backend "nccl"): one rank, so the collectives are RCCL's single-rank all-reduce /
    all_to_all / all_gather, run on torch's stream between the library's own streams -- the hand-off of the library's
    partial state to RCCL and back, on the real collective library (N > 1 needs an 8-GPU node)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(0, 1, _free_port(), q, "nccl"))
    p.start()
    rank, ok, info = q.get(timeout=240)
    p.join(timeout=60)
    assert ok, info
    assert "dense" in info and "rows" in info


DOUBLE_CASES = [
    # (sql, force hash table)
    ("SELECT SUM(d), AVG(w), SUM(f), COUNT(*), SUM(d * w) FROM t", False),            # aggregation-only: LDS slot
    ("SELECT g, SUM(d), AVG(f), SUM(d * w), SUM(i), MIN(d) FROM t GROUP BY g", False),  # dense table
    ("SELECT g, SUM(d), AVG(f), SUM(d * w), SUM(i), MIN(d) FROM t GROUP BY g", True),   # hash table: row exchange
    ("SELECT g, SUM(w), AVG(d + w) FROM t WHERE i < 500 GROUP BY g", False),
    ("SELECT g, SUM(s), AVG(s) FROM t GROUP BY g", False),                               # +-inf / NaN inputs
    ("SELECT SUM(s), SUM(d - w) FROM t WHERE g < 20", False),
]


def _double_segments():
    import numpy as np
    from pinot_amd.segment import ImmutableSegment
    rng = np.random.default_rng(2024)
    segs = []
    for si in range(4):
        n = 50_000 + 3_331 * si
        s_col = rng.normal(size=n) * 1e3
        if si == 0:
            s_col[rng.integers(0, n, 5)] = np.inf      # +inf in some groups
        if si == 2:
            s_col[rng.integers(0, n, 5)] = -np.inf     # -inf in others (NaN where both meet)
        if si == 1:
            s_col[7] = np.nan
        data = {"g": rng.integers(0, 40, n), "i": rng.integers(0, 1000, n),
                "d": np.round(rng.normal(size=n) * 1e6, 3), "f": rng.normal(size=n).astype(np.float32),
                "w": rng.lognormal(0, 6, n) * rng.choice([-1.0, 1.0], n), "s": s_col}
        segs.append(ImmutableSegment.create(f"dbl{si}", data, {"g": "INT", "i": "INT", "d": "DOUBLE", "f": "FLOAT",
                                                              "w": "DOUBLE", "s": "DOUBLE"}))
    return segs


def _bits(rows):
    """The rows with every float replaced by its IEEE bits (so NaN compares equal to the same NaN)."""
    import struct

    def conv(v):
        if isinstance(v, float):
            return struct.unpack("<Q", struct.pack("<d", v))[0]
        if isinstance(v, tuple):
            return tuple(conv(x) for x in v)
        return v
    return {k: [conv(v) for v in row] for k, row in rows.items()}


def _worker_double(rank, world, port, q):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        sys.path.insert(0, ROOT)
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        from helpers import assert_same_result
        from oracle.oracle import OracleEngine
        from pinot_amd import abi
        from pinot_amd.combine import merge_partials_across_ranks
        from pinot_amd.gpu import GpuEngine
        from pinot_amd.plan import Table
        from pinot_amd.query import parse
        eng = GpuEngine(0)
        segs = _double_segments()
        table = Table("t", segs)
        mine = segs[rank::world]
        n_fx = []
        for sql, force_hash in DOUBLE_CASES:
            qc = parse(sql)
            flags = abi.PG_PLAN_HASH_GROUPS if force_hash else 0
            one = eng.run_plan(eng.make_plan(table, qc, flags=flags))           # 1 rank: every segment
            again = eng.run_plan(eng.make_plan(table, qc, flags=flags))
            assert _bits(one.rows) == _bits(again.rows), sql                    # run to run: the same bits
            plan = eng.make_plan(table, qc, segments=mine, flags=flags)
            p = eng.run_partial(plan)
            n_fx.append(int(p.contents.n_fx))
            two = merge_partials_across_ranks(eng, plan, p)                      # 2 ranks: half the segments each
            assert _bits(two.rows) == _bits(one.rows), (sql, sorted(two.rows.items())[:2], sorted(one.rows.items())[:2])
            assert_same_result(one, OracleEngine().execute(table, qc), table=table)
        q.put((rank, True, n_fx))
        dist.destroy_process_group()
    except Exception:
        q.put((rank, False, traceback.format_exc()))


def test_two_ranks_double_sums_are_bit_identical():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_double, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    for rank, ok, info in res:
        assert ok, info
    assert all(n > 0 for n in res[0][2])   # every case has exact fixed-point sums (SK_FX)


WIDE_KEYS = "column1, column3, column5, column6, column7, column9, column11, column12, column17"
WIDE_CASES = [
    # 9 keys (more than a packed key takes): tuple states, merged by the row exchange with their tuples re-interned
    f"SELECT COUNT(*), SUM(column18), MIN(column6), MAX(column3), AVG(column7) FROM t GROUP BY {WIDE_KEYS}",
    f"SELECT COUNT(*), SUM(column1) FROM t WHERE column3 > 1000000000 AND column11 <> 'P' GROUP BY {WIDE_KEYS}, "
    "column18, daysSinceEpoch",
    f"SELECT column1, column3, column6, COUNT(*), DISTINCTCOUNT(column11) FROM t GROUP BY {WIDE_KEYS} "
    "ORDER BY COUNT(*) DESC, column1, column3, column6 LIMIT 7",
]
RAW_CASES = [
    # raw (no-dictionary) group keys (NoDictionarySingleColumnGroupKeyGenerator / ...MultiColumn...)
    "SELECT ts, COUNT(*), SUM(m_long) FROM t WHERE m_int > 3000 GROUP BY ts",
    "SELECT u, k, COUNT(*), MAX(m_double) FROM t GROUP BY u, k",
]


def _wide_segments():
    """4 segments of the reference's SV test data (BaseSingleValueQueriesTest), segment i without every fourth row
    starting at i: most tuples sit on both ranks, some on one only."""
    import numpy as np
    from conftest import GOLDEN, SV_SCHEMA
    from pinot_amd.segment import ImmutableSegment
    z = np.load(os.path.join(GOLDEN, "test_data_sv.npz"))
    full = {k: (z[k] if z[k].dtype.kind != "U" else z[k].astype(object)) for k in SV_SCHEMA}
    n = len(full["column1"])
    segs = []
    for si in range(4):
        keep = (np.arange(n) % 4) != si
        segs.append(ImmutableSegment.create(f"sv{si}", {k: v[keep] for k, v in full.items()},
                                            {k: v[0] for k, v in SV_SCHEMA.items()},
                                            inverted=("column6", "column7", "column11", "column17", "column18"),
                                            field_types={k: v[1] for k, v in SV_SCHEMA.items()}))
    return segs


def _worker_wide(rank, world, port, q):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        sys.path.insert(0, ROOT)
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        from helpers import assert_same_result
        from oracle.oracle import OracleEngine
        from pinot_amd import abi
        from pinot_amd.combine import merge_partials_across_ranks
        from pinot_amd.gpu import GpuEngine
        from pinot_amd.plan import InstanceConfig, Table, reduce_to_rows
        from pinot_amd.query import parse
        from test_raw_index import _raw_segments
        eng = GpuEngine(0)
        modes = []
        for segs, cases in ((_wide_segments(), WIDE_CASES), (_raw_segments(4, 30_000, seed=5), RAW_CASES)):
            table = Table("t", segs)
            mine = segs[rank::world]
            for sql in cases:
                qc = parse(sql)
                for flags in (abi.PG_PLAN_VALUE_SETS, abi.PG_PLAN_VALUE_SETS | abi.PG_PLAN_HASH_GROUPS):
                    plan = eng.make_plan(table, qc, segments=mine, flags=flags)
                    p = eng.run_partial(plan)
                    modes.append(int(p.contents.mode))
                    merged = merge_partials_across_ranks(eng, plan, p)
                    whole = OracleEngine().execute(table, qc)
                    if qc.order_by:
                        assert reduce_to_rows(qc, merged)[1] == reduce_to_rows(qc, whole)[1], sql
                    else:
                        assert_same_result(merged, whole, table=table)
        # numGroupsLimit with tuple keys: each segment keeps its first tuples; the flag is the OR over the ranks
        table = Table("t", _wide_segments())
        qc = parse(f"SELECT COUNT(*), SUM(column1) FROM t GROUP BY {WIDE_KEYS}")
        cfg = InstanceConfig.with_groups_limit(500)
        plan = eng.make_plan(table, qc, segments=table.segments[rank::world], config=cfg)
        merged = merge_partials_across_ranks(eng, plan, eng.run_partial(plan))
        whole = OracleEngine().execute(table, qc, config=cfg)
        assert_same_result(merged, whole, table=table)
        assert merged.groups_limit_reached == whole.groups_limit_reached
        q.put((rank, True, modes))
        dist.destroy_process_group()
    except Exception:
        q.put((rank, False, traceback.format_exc()))


def test_two_ranks_merge_wide_and_raw_keys():
    """A 9-key group-by (and raw-key group-bys) over 2 ranks: tuple states exported with their key tuples, re-interned
    on the owner (PG_STATE_TUPLES rows), equal to the oracle over all segments."""
    import torch.multiprocessing as mp
    from pinot_amd import abi
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_wide, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    for rank, ok, info in res:
        assert ok, info
    assert abi.PG_STATE_TUPLES in res[0][2]
