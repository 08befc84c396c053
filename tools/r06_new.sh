#!/bin/bash
# round 6: smoke, the new parity tests (wide-range double sums, in-library multi-device combine), then the GPU suite
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 240 --timeout-method thread --tb=short"
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 $T tests/test_gpu_wide_sums.py tests/test_having.py > gpurun_out/new1.log 2>&1 || { echo "new1 failed"; tail -60 gpurun_out/new1.log; exit 1; }
tail -2 gpurun_out/new1.log
timeout -k 10 600 $T tests/test_gpu_multidevice.py > gpurun_out/new2.log 2>&1 || { echo "new2 failed"; tail -80 gpurun_out/new2.log; exit 1; }
tail -2 gpurun_out/new2.log
timeout -k 10 1000 $T -m gpu tests ${PYTEST_ARGS} > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; grep -E "PASS|FAIL|ERROR" gpurun_out/gpu_tests.log | tail -5; tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
