#!/bin/bash
# round 6 (third session): smoke, the multi-value group-by tests (several MV keys: new device code), then the GPU suite.
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 240 --timeout-method thread --tb=short"
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 $T -m gpu tests/test_mv_group_by.py tests/test_raw_strings.py > gpurun_out/d_new.log 2>&1 || { echo "new tests failed"; tail -60 gpurun_out/d_new.log; exit 1; }
tail -1 gpurun_out/d_new.log
timeout -k 10 900 $T -m gpu tests > gpurun_out/d_gpu_tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAIL|ERROR" gpurun_out/d_gpu_tests.log | tail -5; tail -60 gpurun_out/d_gpu_tests.log; exit 1; }
tail -1 gpurun_out/d_gpu_tests.log
echo "r06_d ok"
