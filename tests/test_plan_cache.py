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


SHAPE_A = ("SELECT column9, SUM(column1), COUNT(*) FROM t WHERE column7 IN (1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12) "
           "AND column3 > 1000000 GROUP BY column9")
SHAPE_B = ("SELECT column9, SUM(column1), COUNT(*) FROM t WHERE column7 IN (2, 5, 9, 300, 4000, 70000, 123456) "
           "AND column3 > 900000000 GROUP BY column9")


def test_query_shape_ignores_only_filter_literals():
    from pinot_amd.plan import query_shape
    from pinot_amd.query import parse
    assert query_shape(parse(SHAPE_A)) == query_shape(parse(SHAPE_B))
    assert query_shape(parse(SHAPE_A)) != query_shape(parse(SHAPE_A.replace("column3 >", "column3 >=")))
    assert query_shape(parse(SHAPE_A)) != query_shape(parse(SHAPE_A.replace("SUM(column1)", "MAX(column1)")))
    assert query_shape(parse(SHAPE_A)) != query_shape(parse(SHAPE_A + " LIMIT 7"))


def test_relowered_plan_equals_a_fresh_plan(sv_segment):
    """CPlan.relower (the shape cache's hit): the plan of query A re-lowered for query B's literals is the plan of B --
    the same image, leaf for leaf."""
    import numpy as np
    from pinot_amd.plan import CPlan, dict_id_set
    from pinot_amd.query import parse
    from test_abi import _decode_image_leaves
    t = Table("t", [sv_segment] * 3)

    def id_sets(col_id, dt, lit, keys):
        name = [c for c, i in t.column_ids.items() if i == col_id][0]
        row = dict_id_set(sv_segment.columns[name].dictionary, list(lit))
        out = np.zeros((len(keys), len(lit)), dtype=np.int32)
        out[:, :len(row)] = row
        return out, np.full(len(keys), len(row), dtype=np.uint32)
    a = CPlan(t, parse(SHAPE_A), t.segments, [1, 2, 3], trim="server", id_sets=id_sets)
    b = CPlan(t, parse(SHAPE_B), t.segments, [1, 2, 3], trim="server", id_sets=id_sets)
    r = a.relower(parse(SHAPE_B), id_sets)
    assert _decode_image_leaves(r.image()[0])[1] == _decode_image_leaves(b.image()[0])[1]
    assert _decode_image_leaves(r.image()[0])[1] != _decode_image_leaves(a.image()[0])[1]
    assert r.image()[0].tobytes() == b.image()[0].tobytes()


@pytest.mark.gpu
def test_literal_only_change_hits_the_shape_cache(gpu_engine, oracle_engine, sv_table_inter):
    """A parametrised query with fresh literals misses the SQL-text cache but hits the shape cache (only its leaves
    are lowered again) and answers as the oracle does."""
    from pinot_amd.query import parse
    gpu_engine.execute(sv_table_inter, SHAPE_A)
    s0, m0 = gpu_engine.plan_shape_hits, gpu_engine.plan_cache_misses
    got = gpu_engine.execute(sv_table_inter, SHAPE_B)
    assert gpu_engine.plan_shape_hits == s0 + 1 and gpu_engine.plan_cache_misses == m0
    assert_same_result(got, oracle_engine.execute(sv_table_inter, parse(SHAPE_B)), table=sv_table_inter)
