import sys, ctypes as C; sys.path.insert(0,'/root/repo'); sys.path.insert(0,'/root/repo/tests')
import numpy as np, torch
from conftest import build_sv_segment
from pinot_amd.gpu import GpuEngine
from pinot_amd import abi
from oracle.oracle import OracleEngine
from pinot_amd.plan import Table
from pinot_amd.query import parse
seg=build_sv_segment(); t=Table("t",[seg])
g=GpuEngine(0); o=OracleEngine()
F=" WHERE column1 > 100000000 AND column3 BETWEEN 20000000 AND 1000000000 AND column5 = 'gFuH' AND (column6 < 500000000 OR column11 NOT IN ('t', 'P')) AND daysSinceEpoch = 126164076"
base="SELECT COUNT(*), SUM(column1), MAX(column3), MIN(column6), AVG(column7) FROM t"
for q in [base, base+F, base+" GROUP BY column9", base+" GROUP BY column9", "SELECT COUNT(*) FROM t GROUP BY column9", base+" GROUP BY column9"]:
    try:
        rg=g.execute(t,q)
    except Exception as e:
        print("ERR", q[-40:], e); continue
    ro=o.execute(t,q)
    cnt_g=sum(v[0] for v in rg.rows.values()); cnt_o=sum(v[0] for v in ro.rows.values())
    print(q[-30:], "groups", len(rg.rows), len(ro.rows), "count", cnt_g, cnt_o, "equal", rg.rows==ro.rows, "stats", rg.stats.num_docs_scanned, flush=True)
    if rg.rows != ro.rows:
        bad=[k for k in ro.rows if rg.rows.get(k)!=ro.rows[k]][:3]
        for k in bad: print("  ", k, rg.rows.get(k), ro.rows[k])
        extra=[k for k in rg.rows if k not in ro.rows][:3]; print("  extra", extra)
# raw partial dump
plan=g.make_plan(t, parse(base+" GROUP BY column9"))
p=g.run_partial(plan); pc=p.contents
print("partials slots", pc.num_slots, pc.n_i64, pc.n_f64, pc.n_min, pc.n_max, "stats", pc.stats.num_docs_scanned)
i64=torch.zeros(pc.num_slots*pc.n_i64, dtype=torch.int64, device='cuda')
print("copy rc", g.lib.pg_partials_copy(p, 0, C.c_void_p(i64.data_ptr()), None, None, None, None, None))
a=i64.cpu().numpy().reshape(pc.num_slots, pc.n_i64)
print("count sum", a[:,0].sum(), "nonzero slots", (a[:,0]>0).sum(), "first", a[:5])
g.lib.pg_partials_free(p)
