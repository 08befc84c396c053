#!/bin/bash
# smoke + GPU parity suite + scan probe (ring 1 / ring 2); stops at the first failure
set -o pipefail
mkdir -p gpurun_out
SEGS=${SEGS:-128}
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --tb=short > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for V in ${PROBE_VARIANTS:-"PG_STAGE_RING=1" "PG_STAGE_RING=2"}; do
  env $V timeout -k 10 200 python -u tools/scan_probe.py --segments $SEGS --reps 10 > gpurun_out/probe.log 2>&1 || { echo "probe $V failed"; tail -20 gpurun_out/probe.log; exit 1; }
  echo "== $V"; grep -v amdgpu.ids gpurun_out/probe.log
done
