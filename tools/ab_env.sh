#!/bin/bash
# A/B of runtime knobs on one workload: "name:ENV=V,ENV2=V" entries in $VARIANTS ("base:" = defaults), each a short bench
set -o pipefail
mkdir -p gpurun_out
WL=${WL:-adanalytics}
for V in $VARIANTS; do
  N=${V%%:*}; E=${V#*:}
  env $(echo $E | tr ',' ' ') timeout -k 10 300 python3 bench.py --workload $WL --no-cpu --steps 20 --warmup 3 > gpurun_out/abe_${N}_$WL.json 2> gpurun_out/abe_${N}_$WL.err || { echo "variant $N failed"; tail -20 gpurun_out/abe_${N}_$WL.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/abe_${N}_$WL.json'));print('$N $WL', round(d['ms_per_step'],3), 'frac', round(d['roofline']['frac'],3), d['step_breakdown_ms'])"
done
