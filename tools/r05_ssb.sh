#!/bin/bash
# config 3 check: the stream GPU tests, then the ssb bench with the further leaves' slice prefetch off / on / off / on
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "stream or ssb or extra or stage or prefilter" > gpurun_out/ssb_tests.log 2>&1 \
  || { echo "stream tests failed"; tail -40 gpurun_out/ssb_tests.log; exit 1; }
tail -2 gpurun_out/ssb_tests.log
for v in 0 1 0 1; do
  PG_STREAM_STAGE_PRE=$v timeout -k 10 300 python3 bench.py --workload ssb --no-cpu --no-full-parity --steps 10 --warmup 3 > gpurun_out/ssb_$v.json 2> gpurun_out/ssb_$v.err || { echo "bench failed"; tail -5 gpurun_out/ssb_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ssb_$v.json')); print('pre=$v', round(d['ms_per_step'],4), d['step_breakdown_ms'], d['roofline']['kernel_ms'], round(d['roofline']['frac'],3))"
done
