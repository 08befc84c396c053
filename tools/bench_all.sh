#!/bin/bash
# every workload's bench line (configs 2-5) with the full-parity check; stop at the first failure
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for w in ${WORKLOADS:-adanalytics ssb highcard index}; do
  timeout -k 10 420 python -u bench.py --workload $w --steps ${STEPS:-20} --warmup 5 ${BENCH_ARGS} > gpurun_out/${TAG:-r06}_bench_$w.json 2> gpurun_out/${TAG:-r06}_bench_$w.err || { echo "bench $w failed"; tail -30 gpurun_out/${TAG:-r06}_bench_$w.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/${TAG:-r06}_bench_$w.json')); print('$w', round(d['ms_per_step'],4), 'ms', 'frac', round(d['roofline']['frac'],3), 'parity_full', d.get('parity_full'), d.get('parity_full_scope'), 'sample', d.get('parity_sample'), 'lowering', d.get('host_plan_lowering_ms'), d['step_breakdown_ms'])"
done
echo "bench all ok"
