#!/bin/bash
# GPU suite + serial / in-flight bench lines of configs 2, 3, 5 (regression check after a kernel change)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/${TAG:-chk}_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/${TAG:-chk}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${TAG:-chk}_gpu_tests.log
for w in adanalytics ssb index highcard; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu --steps 30 --warmup 5 --no-full-parity > gpurun_out/${TAG:-chk}_$w.json 2> gpurun_out/${TAG:-chk}_$w.err || { echo "bench $w failed"; tail -20 gpurun_out/${TAG:-chk}_$w.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],4), d['serial_ms_per_step'], d['step_breakdown_ms'])" gpurun_out/${TAG:-chk}_$w.json $w
done
