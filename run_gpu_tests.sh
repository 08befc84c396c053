#!/bin/bash
# staged GPU validation: stop at the first failure (no retries)
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --tb=short"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 200 $T -k "golden_inner" > gpurun_out/t1.log 2>&1 || { echo "t1 failed"; exit 1; }
timeout -k 10 200 $T -k "golden_inter" > gpurun_out/t2.log 2>&1 || { echo "t2 failed"; exit 1; }
timeout -k 10 400 $T > gpurun_out/t3.log 2>&1 || { echo "t3 failed"; exit 1; }
echo "tests ok"
