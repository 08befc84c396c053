"""Diagnose the exact-sum windows on the GPU: device vs oracle for wide-range data, plus the raw fx state."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle.oracle import OracleEngine  # noqa: E402
from pinot_amd import abi  # noqa: E402
from pinot_amd.gpu import GpuEngine  # noqa: E402
from pinot_amd.plan import Table  # noqa: E402
from pinot_amd.query import parse  # noqa: E402
from test_gpu_wide_sums import wide_segments  # noqa: E402

import torch  # noqa: E402
torch.cuda.init()
eng = GpuEngine(0)
for big in [(1e30, float(np.finfo(np.float64).max)), (1e30,), ()]:
    segs = wide_segments(big_values=big)
    t = Table("t", segs)
    for sql in ["SELECT SUM(d) FROM t WHERE d < 100", "SELECT SUM(d) FROM t", "SELECT SUM(h) FROM t",
                "SELECT g, SUM(d) FROM t WHERE d < 100 GROUP BY g ORDER BY g LIMIT 3"]:
        q = parse(sql)
        plan = eng.make_plan(t, q)
        ag = plan.plan.aggs[0]
        got = eng.run_plan(plan)
        want = OracleEngine().execute(t, q)
        p = eng.run_partial(plan)
        pc = p.contents
        nfx = pc.n_fx
        fx = np.zeros(2 * nfx * min(pc.num_slots, 1), dtype=np.uint64)
        import torch
        if pc.mode == abi.PG_STATE_DENSE and pc.num_slots == 1:
            buf = torch.empty(4 * nfx, dtype=torch.int64, device="cuda")
            eng.lib.pg_partials_copy(p, abi.PG_COPY_OUT, None, C.c_void_p(buf.data_ptr()), None, None, None)
            limbs = buf.cpu().numpy().reshape(nfx, 4)
            nz = [(w, [int(x) for x in limbs[w]]) for w in range(nfx) if limbs[w].any()]
        else:
            nz = "n/a"
        eng.lib.pg_partials_free(p)
        print(big, sql, "exp", ag.sum_exp, ag.sum_exp_lo, hex(ag.sum_flags), "n_fx", nfx, "trace", eng.last_trace()["path"],
              "\n   got", sorted(got.rows.items())[:2], "\n  want", sorted(want.rows.items())[:2], "\n  windows", nz, flush=True)
