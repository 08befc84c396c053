#!/bin/bash
# quick check: selected GPU tests (-k $K), the highcard bench per PG_DIRECT_WAVES, the headline bench, a highcard trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread --tb=short \
  -k "${K:-radix or config4 or speculative or dict_id_sets}" > gpurun_out/part_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/part_tests.log; exit 1; }
tail -2 gpurun_out/part_tests.log
for W in ${WAVES:-4 8}; do
  PG_DIRECT_WAVES=$W timeout -k 10 300 python -u bench.py --workload highcard --steps 10 --warmup 3 --no-cpu > gpurun_out/hc_w$W.json 2> gpurun_out/hc_w$W.err \
    || { echo "bench failed"; tail -20 gpurun_out/hc_w$W.err; exit 1; }
  echo "waves $W: $(python3 -c "import json;d=json.loads(open('gpurun_out/hc_w$W.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['step_breakdown_ms'])")"
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/ad.json 2> gpurun_out/ad.err || { echo "bench failed"; tail -20 gpurun_out/ad.err; exit 1; }
echo "adanalytics: $(python3 -c "import json;d=json.loads(open('gpurun_out/ad.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['host_plan_lowering_ms'],d['step_breakdown_ms'])")"
PG_HOST_PROFILE=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 2 --no-cpu > /dev/null 2> gpurun_out/ad_hostprof.err || true
bash tools/ktrace2.sh r03b_hc highcard
