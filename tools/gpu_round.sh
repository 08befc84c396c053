#!/bin/bash
# GPU tests (all -m gpu), then one bench line per workload; each step under its own time limit, first failure ends it.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread --tb=short ${PYTEST_ARGS} \
  > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAIL|Error|error" gpurun_out/gpu_tests.log | head -20; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for WL in ${WORKLOADS:-highcard index}; do
  timeout -k 10 400 python -u bench.py --workload $WL --steps 10 --warmup 3 ${BENCH_ARGS} > gpurun_out/bench_$WL.json 2> gpurun_out/bench_$WL.err \
    || { echo "bench $WL failed"; tail -20 gpurun_out/bench_$WL.err; exit 1; }
  echo "$WL: $(python3 -c "import json;d=json.loads(open('gpurun_out/bench_$WL.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['parity_sample'])")"
done
