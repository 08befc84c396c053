#!/bin/bash
# round-5 GPU validation: smoke, the GPU test suite, then config 2's bench line (stop at the first failure, no retries)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/r05_smoke.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/r05_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -60 gpurun_out/r05_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r05_gpu_tests.log
if [ -n "$BENCH" ]; then
  timeout -k 10 300 python -u bench.py $BENCH > gpurun_out/r05_bench.json 2> gpurun_out/r05_bench.err || { echo "bench failed"; tail -30 gpurun_out/r05_bench.err; exit 1; }
  cat gpurun_out/r05_bench.json
fi
echo "r05 ok"
