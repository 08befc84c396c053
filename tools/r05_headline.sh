#!/bin/bash
# config-2 checks: stream / parity GPU tests, bench line, kernel timeline (dev tool)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_stream.py \
  tests/test_gpu_parity.py -k "${TESTS_K:-stream or config2 or adanalytics or in_ or exact}" > gpurun_out/hl_tests.log 2>&1 \
  || { echo "tests failed"; tail -30 gpurun_out/hl_tests.log; exit 1; }
tail -2 gpurun_out/hl_tests.log
timeout -k 10 300 python3 bench.py --workload adanalytics --no-cpu --steps 20 --warmup 5 > gpurun_out/hl_bench.json 2> gpurun_out/hl_bench.err || { echo "bench failed"; tail -5 gpurun_out/hl_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/hl_bench.json')); print(round(d['ms_per_step'],4), d['step_breakdown_ms'], d.get('parity_full'), d['roofline']['kernel_ms'])"
WORKLOADS=adanalytics TAG=tlh bash tools/timeline.sh > /dev/null && python3 tools/timeline.py gpurun_out/tlh_adanalytics | tail -14
