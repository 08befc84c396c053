#!/bin/bash
# stream-path check: its GPU tests, the full GPU suite, then configs 2 and 3 with and without the stream (no CPU leg)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -x -v --timeout 120 --timeout-method thread --tb=short > gpurun_out/stream_tests.log 2>&1 || { echo "stream tests failed"; tail -40 gpurun_out/stream_tests.log; exit 1; }
tail -2 gpurun_out/stream_tests.log
if [ -z "$SKIP_SUITE" ]; then bash tools/gpu_tests.sh || exit 1; fi
for W in ${WORKLOADS:-adanalytics ssb}; do
for V in 1 0; do
  PG_STREAM=$V timeout -k 10 300 python3 bench.py --workload $W --no-cpu --steps 20 --warmup 5 > gpurun_out/${W}_stream$V.json 2> gpurun_out/${W}_stream$V.err || { echo "bench $W stream=$V failed"; tail -20 gpurun_out/${W}_stream$V.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/${W}_stream$V.json')); print('$W stream=$V', round(d['ms_per_step'],3), 'ms/step', '%.3g'%d['value'], 'kernel_ms', round(d['roofline']['kernel_ms'],3), d['roofline']['kernel'], d['step_breakdown_ms'])"
done
done
