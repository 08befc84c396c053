"""Runtime behaviour of the C ABI on an MI355X: in-flight cancellation and deadlines (BaseOperator.nextBlock's
interrupt check, QueryContext.getEndTimeMs), and re-entrancy (several host threads issuing pg_execute at once, as
Pinot's combine worker threads and concurrent queries do)."""
import threading
import time

import numpy as np
import pytest

from helpers import assert_same_result
from pinot_amd.gpu import PinotGpuError
from pinot_amd.plan import Table
from pinot_amd.query import parse

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def long_scan(gpu_engine):
    """~200 M rows of config-4 shape through the per-doc atomic group-by (PG_PART=0: one long scan launch of tens of
    ms; the radix-partitioned pipeline finishes the same query in a few ms, mostly outside the scan kernel)."""
    import os
    old = os.environ.get("PG_PART")
    os.environ["PG_PART"] = "0"
    yield _long_scan(gpu_engine)
    if old is None:
        os.environ.pop("PG_PART", None)
    else:
        os.environ["PG_PART"] = old


def _long_scan(gpu_engine):
    import torch
    from pinot_amd import synth
    from pinot_amd.segment import ImmutableSegment
    segs = []
    table = None
    for s in range(24):
        dcs = synth.make_columns_torch(synth.HIGHCARD, s, 8_000_000, torch.device("cuda"))
        seg = ImmutableSegment(f"ev{s}", 8_000_000, {dc.spec.name: dc.meta_column() for dc in dcs})
        if table is None:
            table = Table("events", [seg])
        gpu_engine.register_device_segment(seg, table, dcs)
        segs.append(seg)
    table = Table("events", segs)
    from pinot_amd import synth as sy
    from pinot_amd.plan import InstanceConfig
    plan = gpu_engine.make_plan(table, parse(sy.highcard_query()), flags=0, trim=True,
                                config=InstanceConfig(num_groups_limit=10_000_000))
    gpu_engine.run_plan(plan)
    t0 = time.perf_counter()
    ref = gpu_engine.run_plan(plan)
    full = time.perf_counter() - t0
    return plan, ref, full


def _now_ms():
    return int(time.clock_gettime(time.CLOCK_MONOTONIC) * 1000)


def test_deadline_stops_running_scan(gpu_engine, long_scan):
    from pinot_amd import abi
    plan, ref, full = long_scan
    assert full > 0.01, full
    plan.plan.deadline_ms = _now_ms() + max(2, int(full * 1000 / 8))
    t0 = time.perf_counter()
    with pytest.raises(PinotGpuError) as e:
        gpu_engine.run_plan(plan)
    el = time.perf_counter() - t0
    plan.plan.deadline_ms = 0
    assert e.value.code == abi.PG_E_TIMEOUT
    assert el < 0.7 * full, (el, full)
    assert gpu_engine.run_plan(plan).rows == ref.rows  # the library is intact afterwards


def test_cancel_from_another_thread(gpu_engine, long_scan):
    from pinot_amd import abi
    plan, ref, full = long_scan
    plan.plan.query_id = 4242
    out = {}

    def run():
        t0 = time.perf_counter()
        try:
            out["res"] = gpu_engine.run_plan(plan)
        except PinotGpuError as ex:
            out["err"] = ex.code
        out["el"] = time.perf_counter() - t0

    th = threading.Thread(target=run)
    th.start()
    time.sleep(full / 6)
    assert gpu_engine.lib.pg_cancel(4242) == 0
    th.join()
    assert out.get("err") == abi.PG_E_CANCELLED, out
    assert out["el"] < 0.8 * full, (out["el"], full)
    plan.plan.query_id = 4243  # a fresh id runs to completion
    assert gpu_engine.run_plan(plan).rows == ref.rows
    plan.plan.query_id = 0


def test_partitioned_group_by_matches_atomic_at_scale(gpu_engine, long_scan):
    """The radix-partitioned group-by (pg_part.hip) over the same 192 M rows gives the per-doc atomic path's result:
    at this size every split block runs many LDS counting-sort rounds (the small parity cases run one partial round)."""
    import os
    plan, ref, full = long_scan
    os.environ["PG_PART"] = "1"
    try:
        res = gpu_engine.run_plan(plan)
    finally:
        os.environ["PG_PART"] = "0"
    assert res.rows == ref.rows


def test_concurrent_executes_from_two_threads(gpu_engine, oracle_engine, sv_table_inter):
    """Two host threads, each with its own stream and parameter arena, run different queries at once; every result
    matches the oracle."""
    queries = ["SELECT column11, COUNT(*), SUM(column1), MAX(column3) FROM t GROUP BY column11",
               "SELECT COUNT(*), SUM(column7), MIN(column6) FROM t WHERE column6 < 500000000",
               "SELECT column9, DISTINCTCOUNT(column7) FROM t WHERE column3 > 1000000000 GROUP BY column9",
               "SELECT column12, AVG(column17) FROM t WHERE column11 NOT IN ('t', 'P') GROUP BY column12"]
    expect = {sql: oracle_engine.execute(sv_table_inter, parse(sql)) for sql in queries}
    plans = {sql: gpu_engine.make_plan(sv_table_inter, parse(sql)) for sql in queries}
    errors = []

    def worker(k):
        try:
            for i in range(12):
                sql = queries[(i + k) % len(queries)]
                assert_same_result(gpu_engine.run_plan(plans[sql]), expect[sql], table=sv_table_inter)
        except Exception as ex:  # surfaced in the main thread
            errors.append(repr(ex))

    ths = [threading.Thread(target=worker, args=(k,)) for k in range(2)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errors, errors


def test_trace_records_each_device_call(gpu_engine, sv_table_inter):
    """pg_last_trace (pinot_trace.h): the per-call recording that stands for the reference's operator trace scopes --
    the kernels that ran, each filter leaf's form per segment, the stream's driving leaf, docs matched."""
    from pinot_amd import synth
    from pinot_amd.plan import Table
    segs = [synth.make_segment_np(synth.ADANALYTICS, s, 100_003) for s in range(3)]
    t = Table("adAnalytics", segs)
    r = gpu_engine.execute(t, synth.adanalytics_query(1000))
    tr = gpu_engine.last_trace()
    assert "stream" in tr["path"] and tr["stream_leaf"] == 1          # accountId IN drives the stream
    assert tr["leaf_forms"][0] == {"SCAN_RANGE": 3}                   # daysSinceEpoch BETWEEN: a dictId range
    assert tr["leaf_forms"][1] in ({"SCAN_SET_LDS": 3}, {"SCAN_SET_LUT": 3})
    assert tr["num_docs_matched"] == r.stats.num_docs_scanned and tr["group_mode"] == "dense"
    assert tr["reruns"] == 0 and tr["num_segments"] == 3 and tr["device_ms"] > 0
    # the reference's test data: sorted daysSinceEpoch, inverted column11, a scan on column1
    gpu_engine.execute(sv_table_inter, "SELECT COUNT(*) FROM t WHERE daysSinceEpoch = 126164076 AND "
                                       "column11 IN ('P', 'o') AND column6 < 500000000")
    tr = gpu_engine.last_trace()
    assert tr["leaf_forms"][0] == {"SORTED_RANGE": 4}
    assert tr["leaf_forms"][1] == {"INVERTED": 4} and "prepass" in tr["path"]
    assert "SCAN_RANGE" in tr["leaf_forms"][2] and "index_count" not in tr["path"]
    # index leaves only (sorted range + inverted set) under COUNT(*): the fused index count, no pre-pass bitmaps
    gpu_engine.execute(sv_table_inter, "SELECT COUNT(*) FROM t WHERE daysSinceEpoch = 126164076 AND "
                                       "column11 IN ('P', 'o')")
    tr = gpu_engine.last_trace()
    assert tr["leaf_forms"][0] == {"SORTED_RANGE": 4} and tr["leaf_forms"][1] == {"INVERTED": 4}
    assert tr["path"] == ["index_count"]
    # metadata answers: MIN / MAX / COUNT over match-all segments
    gpu_engine.execute(sv_table_inter, "SELECT COUNT(*), MAX(column1) FROM t")
    tr = gpu_engine.last_trace()
    assert "nonscan" in tr["path"] and tr["num_segments_nonscan"] == 4
