"""Double SUM / AVG over wide-range data: the exact fixed-point sums (SK_FX) cut
every input into exponent windows sized from the table's smallest nonzero and largest |value| (pg_internal.h
fx_split), so one 1e30 or Double.MAX_VALUE in a DOUBLE column no longer rounds the small values of other rows, groups
or filters to 0.  GPU vs the oracle's sequential double sum (SumAggregationFunction.java:71-126,
AvgAggregationFunction.java:65-139) at north_star's 1e-9, and bit-identical across 1 and 2 ranks, including a column
whose bound lies in [0.5, 1) (sum_exp 0, which once meant "let every GPU derive its own unit")."""
import os
import socket
import sys
import traceback

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

QUERIES = [
    "SELECT SUM(d), AVG(d), COUNT(*) FROM t WHERE d < 100",
    "SELECT SUM(d), AVG(d), MAX(d) FROM t",
    "SELECT g, SUM(d), AVG(d) FROM t GROUP BY g",
    "SELECT g, SUM(d), AVG(d) FROM t WHERE d < 100 GROUP BY g ORDER BY g LIMIT 100",
    "SELECT SUM(a * b), AVG(a * b) FROM t WHERE a < 1 AND b < 1",
    "SELECT g, SUM(a * b) FROM t WHERE a < 1 AND b < 1 GROUP BY g",
    "SELECT SUM(a * b), SUM(a + d), SUM(h) FROM t",
    "SELECT g, SUM(h), AVG(h) FROM t GROUP BY g",
]


def wide_segments(n=40_000, big_values=(1e30, float(np.finfo(np.float64).max))):
    """4 segments.  d: DOUBLE in [0.01, 100) plus one huge value per listed big value (its row in group 99 alone);
    a, b: DOUBLE log-uniform in [1e-3, 1e9]; h: DOUBLE in (0.5, 1) whose largest value differs between the
    segments of the two ranks; g: INT group key 0..49."""
    from pinot_amd.segment import ImmutableSegment
    rng = np.random.default_rng(77)
    segs = []
    for si in range(4):
        m = n + 1_111 * si
        d = rng.uniform(0.01, 100.0, m)
        g = rng.integers(0, 50, m)
        if si in (1, 3) and big_values:
            d[13] = big_values[0 if si == 1 else -1]
            g[13] = 99
        a = np.exp(rng.uniform(np.log(1e-3), np.log(1e9), m))
        b = np.exp(rng.uniform(np.log(1e-3), np.log(1e9), m))
        h = rng.uniform(0.5, 0.6 if si % 2 == 0 else 0.95, m)
        segs.append(ImmutableSegment.create(f"w{si}", {"g": g, "d": d, "a": a, "b": b, "h": h},
                                            {"g": "INT", "d": "DOUBLE", "a": "DOUBLE", "b": "DOUBLE", "h": "DOUBLE"}))
    return segs


@pytest.fixture(scope="module")
def engine(gpu_engine):
    return gpu_engine


@pytest.mark.parametrize("sql", QUERIES)
@pytest.mark.parametrize("hash_groups", [False, True])
def test_wide_range_double_sums_match_oracle(engine, sql, hash_groups):
    from helpers import assert_same_result
    from oracle.oracle import OracleEngine
    from pinot_amd import abi
    from pinot_amd.plan import Table
    from pinot_amd.query import parse
    table = Table("t", wide_segments())
    qc = parse(sql)
    flags = abi.PG_PLAN_HASH_GROUPS if hash_groups else 0
    got = engine.run_plan(engine.make_plan(table, qc, flags=flags))
    want = OracleEngine().execute(table, qc)
    assert_same_result(got, want, table=table)
    if "GROUP BY" in sql and "d < 100" not in sql and "a < 1" not in sql and "(h)" not in sql:
        assert (99,) in got.rows   # the huge values' own group


def test_plan_carries_table_global_windows(engine):
    """The plan's SUM over a column bounded in [0.5, 1): PG_SUM_BOUNDS with sum_exp 0, and the same fixed-point
    signature from the segments of either rank (so their partial states merge)."""
    from pinot_amd import abi
    from pinot_amd.plan import Table
    from pinot_amd.query import parse
    segs = wide_segments()
    table = Table("t", segs)
    qc = parse("SELECT g, SUM(h) FROM t GROUP BY g")
    sigs = set()
    for mine in (segs[0::2], segs[1::2]):
        plan = engine.make_plan(table, qc, segments=mine)
        ag = plan.plan.aggs[0]
        assert ag.sum_flags & abi.PG_SUM_BOUNDS and ag.sum_exp == 0 and ag.sum_exp_lo == -1
        p = engine.run_partial(plan)
        sigs.add((int(p.contents.fx_sig), int(p.contents.n_fx)))
        engine.lib.pg_partials_free(p)
    assert len(sigs) == 1, sigs


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
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
        from test_gpu_distributed import _bits
        eng = GpuEngine(0)
        segs = wide_segments()
        table = Table("t", segs)
        mine = segs[rank::world]
        for sql in QUERIES:
            qc = parse(sql)
            for flags in (0, abi.PG_PLAN_HASH_GROUPS):
                one = eng.run_plan(eng.make_plan(table, qc, flags=flags))
                plan = eng.make_plan(table, qc, segments=mine, flags=flags)
                two = merge_partials_across_ranks(eng, plan, eng.run_partial(plan))
                assert _bits(two.rows) == _bits(one.rows), sql
                assert_same_result(two, OracleEngine().execute(table, qc), table=table)
        q.put((rank, True, None))
        dist.destroy_process_group()
    except Exception:
        q.put((rank, False, traceback.format_exc()))


def test_two_ranks_wide_range_sums_are_bit_identical():
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
