"""Isolate the filtered double-sum discrepancy: which filters / columns / staging settings reproduce it."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle.oracle import OracleEngine  # noqa: E402
from pinot_amd.gpu import GpuEngine  # noqa: E402
from pinot_amd.plan import Table  # noqa: E402
from pinot_amd.query import parse  # noqa: E402
from test_gpu_wide_sums import wide_segments  # noqa: E402

eng = GpuEngine(0)
for big in [(1e30, float(np.finfo(np.float64).max)), ()]:
    segs = wide_segments(big_values=big)
    t = Table("t", segs)
    for sql in ["SELECT COUNT(*), SUM(d) FROM t WHERE d < 100", "SELECT COUNT(*), SUM(d) FROM t WHERE d < 50",
                "SELECT COUNT(*), SUM(h) FROM t WHERE d < 50", "SELECT COUNT(*), SUM(d) FROM t WHERE g < 30",
                "SELECT COUNT(*), MIN(d), MAX(d) FROM t WHERE d < 50", "SELECT COUNT(*), SUM(a) FROM t WHERE a < 1000",
                "SELECT COUNT(*), SUM(d) FROM t WHERE h < 0.7"]:
        q = parse(sql)
        got = eng.run_plan(eng.make_plan(t, q))
        want = OracleEngine().execute(t, q)
        tr = eng.last_trace()
        print(bool(big), os.environ.get("PG_STAGE_KB", "-"), sql, "|", got.rows[()], "| want", want.rows[()],
              "| ok" if np.allclose([float(x) for x in got.rows[()]], [float(x) for x in want.rows[()]], rtol=1e-9) else "| BAD",
              tr["path"], tr.get("leaf_forms"), flush=True)
