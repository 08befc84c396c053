#!/bin/bash
# in-flight A/B: the same bench with 1, 2, 3 queries in flight (adanalytics, ssb)
set -o pipefail
mkdir -p gpurun_out
for w in ${WORKLOADS:-adanalytics ssb}; do
  for n in ${INFLIGHT:-1 2 3}; do
    timeout -k 10 300 python -u bench.py --workload $w --no-cpu --steps 40 --warmup 5 --no-full-parity --inflight $n \
      > gpurun_out/if_${w}_$n.json 2> gpurun_out/if_${w}_$n.err || { echo "bench $w $n failed"; tail -20 gpurun_out/if_${w}_$n.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d['serial_ms_per_step'], d['roofline']['kernel_ms'])" gpurun_out/if_${w}_$n.json
  done
done
