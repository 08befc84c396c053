#!/bin/bash
# knob sweep of the selective stream + list kernel (dev tool): one short bench line per setting, no CPU leg
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > gpurun_out/stream_tests.log 2>&1 || { echo "stream tests failed"; tail -30 gpurun_out/stream_tests.log; exit 1; }
tail -1 gpurun_out/stream_tests.log
run() {  # workload, label, env...
  local W=$1 L=$2; shift 2
  env "$@" timeout -k 10 200 python3 bench.py --workload $W --no-cpu --steps 20 --warmup 5 > gpurun_out/sw_${W}_$L.json 2> gpurun_out/sw_${W}_$L.err || { echo "bench $W $L failed"; tail -20 gpurun_out/sw_${W}_$L.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/sw_${W}_$L.json')); b=d['step_breakdown_ms']; print('$W $L', round(d['ms_per_step'],3), 'ms', '%.3g'%d['value'], 'stream', b['prefilter_ms'], 'scan', b['scan_ms'], 'compile', b['host_compile_ms'], 'exec_wall', b['execute_wall_ms'])"
}
for W in adanalytics ssb; do
  run $W base PG_STREAM=1 || exit 1
  run $W ig256 PG_STREAM_ITEM_GROUPS=256 || exit 1
  run $W ig2048 PG_STREAM_ITEM_GROUPS=2048 || exit 1
  run $W bpc4 PG_STREAM_BLOCKS_PER_CU=4 || exit 1
  run $W bpc12 PG_STREAM_BLOCKS_PER_CU=12 || exit 1
  run $W lb256 PG_LIST_BLOCKS=256 || exit 1
  run $W lb512 PG_LIST_BLOCKS=512 || exit 1
  run $W lb1024 PG_LIST_BLOCKS=1024 || exit 1
done
