#!/bin/bash
# every -m gpu test, then bench + kernel trace of the given workloads ($WORKLOADS)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --tb=short > gpurun_out/gpu_tests.log 2>&1 \
  || { echo "gpu tests failed"; grep -E "FAIL|Error" gpurun_out/gpu_tests.log | head -20; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for WL in ${WORKLOADS:-index}; do
  timeout -k 10 400 python -u bench.py --workload $WL --steps 10 --warmup 3 --no-cpu > gpurun_out/b_$WL.json 2> gpurun_out/b_$WL.err \
    || { echo "bench $WL failed"; tail -20 gpurun_out/b_$WL.err; exit 1; }
  echo "$WL: $(python3 -c "import json;d=json.loads(open('gpurun_out/b_$WL.json').read().strip().splitlines()[-1]);print(d['value'],round(d['ms_per_step'],4),round(d['roofline']['frac'],3),d['step_breakdown_ms'])")"
  bash tools/ktrace2.sh ${TAG:-r03x}_$WL $WL > /dev/null || exit 1
  grep -E "mean_ms" gpurun_out/${TAG:-r03x}_${WL}_trace.txt | grep -v "be_to_native\|bswap\|decode_pack\|sorted_to_packed\|popc_words\|select_rows\|set_last" | cut -c1-120
done
