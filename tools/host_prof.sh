#!/bin/bash
# host phase profile (PG_HOST_PROFILE=1) of the default bench line of configs 2, 5 and 3; each GPU step under its own
# limit, first failure ends it
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
TAG=${TAG:-hp}
for w in ${WORKLOADS:-adanalytics index ssb}; do
  PG_HOST_PROFILE=1 timeout -k 10 300 python3 bench.py --workload $w --no-cpu --steps 20 --warmup 3 $BENCH_ARGS \
    > $O/${TAG}_$w.json 2> $O/${TAG}_$w.err || { echo "$w failed"; tail -20 $O/${TAG}_$w.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/${TAG}_$w.json'));print('$w', round(d['ms_per_step'],3), d['step_breakdown_ms'])"
  tail -3 $O/${TAG}_$w.err
done
