#!/bin/bash
# stream tests + filter-kind probe + config 2 / 3 bench lines (dev loop); first failure ends it
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > gpurun_out/stream_tests.log 2>&1 || { echo "stream tests failed"; tail -30 gpurun_out/stream_tests.log; exit 1; }
tail -1 gpurun_out/stream_tests.log
timeout -k 10 300 python3 tools/scan_probe.py --segments 128 --reps 10 --only ${PROBE:-count,in_only,range_narrow,in_100,config2} > gpurun_out/probe.txt 2>&1 || { echo "probe failed"; tail -20 gpurun_out/probe.txt; exit 1; }
cat gpurun_out/probe.txt
for W in ${WORKLOADS:-adanalytics ssb}; do
  timeout -k 10 200 python3 bench.py --workload $W --no-cpu --steps 20 --warmup 5 > gpurun_out/q_$W.json 2> gpurun_out/q_$W.err || { echo "bench $W failed"; tail -20 gpurun_out/q_$W.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/q_$W.json')); b=d['step_breakdown_ms']; print('$W', round(d['ms_per_step'],3), 'ms', '%.3g'%d['value'], 'stream', b['prefilter_ms'], 'scan', b['scan_ms'], 'compile', b['host_compile_ms'], 'exec_wall', b['execute_wall_ms'], 'fin', b['finalize_wall_ms'])"
done
