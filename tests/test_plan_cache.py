"""The engine's compiled-plan cache (GpuEngine.cached_plan): the same SQL text over the same resident segments reuses
the lowered plan, with results identical to a freshly planned run; anything the plan depends on (segments, flags, trim,
instance config, residency) misses."""
import pytest

from pinot_amd.plan import InstanceConfig, Table

from test_gpu_parity import assert_same_result

SQL = ("SELECT column9, SUM(column1), COUNT(*) FROM t WHERE column7 IN (1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12) "
       "AND column3 > 1000000 GROUP BY column9")


@pytest.mark.gpu
def test_repeated_sql_hits_the_plan_cache(gpu_engine, oracle_engine, sv_table_inter):
    from pinot_amd.query import parse
    h0, m0 = gpu_engine.plan_cache_hits, gpu_engine.plan_cache_misses
    first = gpu_engine.execute(sv_table_inter, SQL)
    second = gpu_engine.execute(sv_table_inter, SQL)
    assert gpu_engine.plan_cache_misses == m0 + 1 and gpu_engine.plan_cache_hits == h0 + 1
    assert first.rows == second.rows and first.stats == second.stats
    assert_same_result(second, oracle_engine.execute(sv_table_inter, parse(SQL)), table=sv_table_inter)
    # a QueryContext (not SQL text) is planned afresh
    gpu_engine.execute(sv_table_inter, parse(SQL))
    assert gpu_engine.plan_cache_hits == h0 + 1


@pytest.mark.gpu
def test_plan_cache_key_covers_segments_trim_and_config(gpu_engine, sv_segment):
    t2 = Table("testTable", [sv_segment] * 2)
    t4 = Table("testTable", [sv_segment] * 4)
    m0 = gpu_engine.plan_cache_misses
    r2 = gpu_engine.execute(t2, SQL)
    r4 = gpu_engine.execute(t4, SQL)  # another table object / segment list: a miss
    assert gpu_engine.plan_cache_misses == m0 + 2
    assert r4.stats.num_docs_scanned == 2 * r2.stats.num_docs_scanned
    gpu_engine.execute(t2, SQL, config=InstanceConfig(num_groups_limit=50_000))  # another instance config: a miss
    gpu_engine.execute(t2, SQL, trim=True)                                 # another trim: a miss
    assert gpu_engine.plan_cache_misses == m0 + 4
    h = gpu_engine.plan_cache_hits
    gpu_engine.execute(t2, SQL, config=InstanceConfig(num_groups_limit=50_000))
    assert gpu_engine.plan_cache_hits == h + 1


@pytest.mark.gpu
def test_released_segment_drops_its_plans(gpu_engine):
    from conftest import build_sv_segment
    seg = build_sv_segment()
    t = Table("testTable", [seg])
    before = gpu_engine.execute(t, SQL)
    gpu_engine.release(seg)  # the residency key is gone: the next run re-uploads and re-plans
    m = gpu_engine.plan_cache_misses
    after = gpu_engine.execute(t, SQL)
    assert gpu_engine.plan_cache_misses == m + 1
    assert before.rows == after.rows
    gpu_engine.release(seg)
