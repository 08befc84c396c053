#!/bin/bash
# config 5: the persistent index-count grid size (PG_IDX_GRID; 0 = the resident slots)
set -o pipefail
mkdir -p gpurun_out
for g in ${GRIDS:-0 1024 512 768 1568}; do
  PG_IDX_GRID=$g timeout -k 10 200 python -u bench.py --workload index --steps 30 --warmup 5 --no-cpu > gpurun_out/idxg_$g.json 2> gpurun_out/idxg_$g.err || { echo "grid $g failed"; tail -20 gpurun_out/idxg_$g.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/idxg_$g.json')); print('grid $g', round(d['ms_per_step'],4), d['step_breakdown_ms']['scan_ms'])"
done
