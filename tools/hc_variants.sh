#!/bin/bash
# config-4 (highcard) bench under launch-knob variants; one line per variant (scan pipeline ms, step ms)
set -o pipefail
mkdir -p gpurun_out
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --workload highcard --no-cpu --steps 5 --warmup 2 > gpurun_out/hcv_$tag.json 2> gpurun_out/hcv_$tag.err || { echo "variant $tag failed"; tail -5 gpurun_out/hcv_$tag.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/hcv_$tag.json')); print('$tag', round(d['ms_per_step'],3), d['step_breakdown_ms'])"
}
run default PG_X=0 && run ring1 PG_STAGE_RING=1 && run nostage PG_NO_STAGING=1 && run bpc2 PG_SCAN_BLOCKS_PER_CU=2 && run bpc4 PG_SCAN_BLOCKS_PER_CU=4
