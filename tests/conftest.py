"""Shared fixtures.  `-m "not gpu"` tests run in the build container (no GPU); `-m gpu` tests run on an MI355X
and call the product path through the C ABI (pinot_amd.gpu -> libpinot_gpu.so)."""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libpinot_gpu.so)")


@pytest.fixture(scope="session")
def expected():
    with open(os.path.join(GOLDEN, "expected.json")) as f:
        return json.load(f)


# BaseSingleValueQueriesTest.java:95-105 schema (column -> data type, field type)
SV_SCHEMA = {
    "column1": ("INT", "METRIC"), "column3": ("INT", "METRIC"), "column5": ("STRING", "DIMENSION"),
    "column6": ("INT", "DIMENSION"), "column7": ("INT", "DIMENSION"), "column9": ("INT", "DIMENSION"),
    "column11": ("STRING", "DIMENSION"), "column12": ("STRING", "DIMENSION"), "column17": ("INT", "METRIC"),
    "column18": ("INT", "METRIC"), "daysSinceEpoch": ("INT", "TIME"),
}


def build_sv_segment(inverted=("column6", "column7", "column11", "column17", "column18")):
    from pinot_amd.segment import ImmutableSegment
    z = np.load(os.path.join(GOLDEN, "test_data_sv.npz"))
    data = {k: (z[k] if z[k].dtype.kind != "U" else z[k].astype(object)) for k in SV_SCHEMA}
    return ImmutableSegment.create("testTable_126164076_167572854", data, {k: v[0] for k, v in SV_SCHEMA.items()},
                                   inverted=inverted, field_types={k: v[1] for k, v in SV_SCHEMA.items()})


@pytest.fixture(scope="session")
def sv_segment():
    return build_sv_segment()


@pytest.fixture(scope="session")
def sv_table_inner(sv_segment):
    from pinot_amd.plan import Table
    return Table("testTable", [sv_segment])


@pytest.fixture(scope="session")
def sv_table_inter(sv_segment):
    """4 identical segments: 2 segments x 2 simulated servers (BaseQueriesTest.getBrokerResponse :151-190)."""
    from pinot_amd.plan import Table
    return Table("testTable", [sv_segment] * 4)


@pytest.fixture(scope="session")
def oracle_engine():
    from oracle.oracle import OracleEngine
    return OracleEngine()


@pytest.fixture(scope="session")
def gpu_engine():
    # torch (device buffers of the synthetic segments, RCCL) carries its own HIP runtime beside the system one
    # libpinot_gpu links; torch must open the device first or it reports no GPU afterwards (bench.py does the same)
    import torch
    torch.zeros(1, device="cuda")
    from pinot_amd.gpu import GpuEngine
    return GpuEngine(0)
