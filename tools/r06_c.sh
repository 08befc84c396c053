#!/bin/bash
# round 6 (third session): smoke, the raw STRING / BYTES filter tests, the GPU suite, then the global-atomic probe
# (tools/l2_atomic_probe.hip).  Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 240 --timeout-method thread --tb=short"
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 $T -m gpu tests/test_raw_strings.py > gpurun_out/c_new.log 2>&1 || { echo "new tests failed"; tail -60 gpurun_out/c_new.log; exit 1; }
tail -1 gpurun_out/c_new.log
timeout -k 10 900 $T -m gpu tests > gpurun_out/c_gpu_tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAIL|ERROR" gpurun_out/c_gpu_tests.log | tail -5; tail -60 gpurun_out/c_gpu_tests.log; exit 1; }
tail -1 gpurun_out/c_gpu_tests.log
if [ -x tools/l2_atomic_probe ]; then
  timeout -k 10 120 tools/l2_atomic_probe > gpurun_out/c_atomic_probe.jsonl 2>&1 || { echo "probe failed"; cat gpurun_out/c_atomic_probe.jsonl; exit 1; }
  cat gpurun_out/c_atomic_probe.jsonl
fi
echo "r06_c ok"
