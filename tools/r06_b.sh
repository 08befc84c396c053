#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread --tb=short -m gpu tests/test_plan_cache.py tests/test_gpu_runtime.py tests/test_abi.py > gpurun_out/b_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/b_tests.log; exit 1; }
tail -1 gpurun_out/b_tests.log
WORKLOADS="adanalytics index" TAG=r06b STEPS=30 bash tools/bench_all.sh || exit 1
python3 -c "
import json
for w in ('adanalytics','index'):
    d=json.load(open('gpurun_out/r06b_bench_%s.json'%w)); print(w, d['host_plan_lowering_ms'], d['host_plan_lowering_cold_ms'], d['host_plan_relower_ms'])"
bash tools/r06_host.sh
