#!/bin/bash
# config-2 step with / without the phase-timing events, and the kernel timeline without them (dev tool)
set -o pipefail
mkdir -p gpurun_out
for v in 1 0 1 0; do
  PG_TIMING_EVENTS=$v timeout -k 10 300 python3 bench.py --workload adanalytics --no-cpu --no-full-parity --steps 30 --warmup 5 > gpurun_out/ev_$v.json 2> gpurun_out/ev_$v.err || { echo "bench failed"; tail -5 gpurun_out/ev_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ev_$v.json')); print('events=$v', round(d['ms_per_step'],4))"
done
PG_TIMING_EVENTS=0 WORKLOADS=adanalytics TAG=tle bash tools/timeline.sh > /dev/null && python3 tools/timeline.py gpurun_out/tle_adanalytics | tail -6
