#!/bin/bash
# A/B of library variants on one workload: "name:lib" pairs in $VARIANTS (lib relative to pinot_amd/), each a short
# bench line (no CPU leg); every step under its own limit, the first failure ends the run
set -o pipefail
mkdir -p gpurun_out
WL=${WL:-ssb}
for V in $VARIANTS; do
  N=${V%%:*}; LIB=${V#*:}
  PINOT_GPU_LIB=$PWD/pinot_amd/$LIB timeout -k 10 300 python3 bench.py --workload $WL --no-cpu --steps 10 --warmup 3 > gpurun_out/ab_${N}_$WL.json 2> gpurun_out/ab_${N}_$WL.err \
    || { echo "bench $N failed"; tail -20 gpurun_out/ab_${N}_$WL.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab_${N}_$WL.json')); print('$N $WL', round(d['ms_per_step'],3), 'ms/step frac', round(d['roofline']['frac'],3), d['step_breakdown_ms'])"
done
