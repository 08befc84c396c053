#!/bin/bash
# stream / list grid sweep for configs 2 and 3 (dev tool): one short bench line per setting, no CPU leg
set -o pipefail
mkdir -p gpurun_out
run() {  # workload, label, env...
  local W=$1 L=$2; shift 2
  env "$@" timeout -k 10 200 python3 bench.py --workload $W --no-cpu --steps 20 --warmup 5 > gpurun_out/sw2_${W}_$L.json 2> gpurun_out/sw2_${W}_$L.err || { echo "bench $W $L failed"; tail -20 gpurun_out/sw2_${W}_$L.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/sw2_${W}_$L.json')); b=d['step_breakdown_ms']; print('$W $L', round(d['ms_per_step'],3), 'ms', 'stream', b['prefilter_ms'], 'scan', b['scan_ms'], 'kernel', round(b['prefilter_ms'] + b['scan_ms'], 4))"
}
run ssb base PG_STREAM=1 || exit 1
run ssb bpc8 PG_STREAM_BLOCKS_PER_CU=8 || exit 1
run ssb bpc10 PG_STREAM_BLOCKS_PER_CU=10 || exit 1
run ssb bpc12 PG_STREAM_BLOCKS_PER_CU=12 || exit 1
run ssb bpc12lb1024 PG_STREAM_BLOCKS_PER_CU=12 PG_LIST_BLOCKS=1024 || exit 1
run ssb lb768 PG_LIST_BLOCKS=768 || exit 1
run adanalytics base PG_STREAM=1 || exit 1
run adanalytics bpc8 PG_STREAM_BLOCKS_PER_CU=8 || exit 1
run adanalytics bpc10 PG_STREAM_BLOCKS_PER_CU=10 || exit 1
run adanalytics lb384 PG_LIST_BLOCKS=384 || exit 1
run adanalytics lb768 PG_LIST_BLOCKS=768 || exit 1
