#!/bin/bash
# gpu tests, then one short bench line per workload (no CPU leg); each GPU step under its own limit, first failure ends it
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-q}
bash tools/gpu_tests.sh || exit 1
for W in ${WORKLOADS:-adanalytics ssb highcard}; do
  timeout -k 10 300 python3 bench.py --workload $W --no-cpu --steps 10 --warmup 3 > gpurun_out/${TAG}_$W.json 2> gpurun_out/${TAG}_$W.err || { echo "bench $W failed"; tail -20 gpurun_out/${TAG}_$W.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_$W.json')); print('$W', round(d['ms_per_step'],3), 'ms/step', '%.3g'%d['value'], d['unit'], 'frac', round(d['roofline']['frac'],3), d['step_breakdown_ms'])"
done
