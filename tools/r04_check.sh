#!/bin/bash
# full GPU suite, then short bench lines (WORKLOADS) with the host phase profile of the last; first failure ends it
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
bash tools/gpu_tests.sh || exit 1
for W in ${WORKLOADS:-highcard index}; do
  PG_HOST_PROFILE=1 timeout -k 10 300 python3 bench.py --workload $W --no-cpu --steps 10 --warmup 3 > $O/chk_$W.json 2> $O/chk_$W.err || { echo "bench $W failed"; tail -20 $O/chk_$W.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/chk_$W.json'));print('$W', round(d['ms_per_step'],3), d['step_breakdown_ms'], round(d['roofline']['frac'],3), d['parity_sample'])"
  grep "pg host" $O/chk_$W.err | tail -1
done
