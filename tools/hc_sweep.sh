#!/bin/bash
# config 4 staging / grid sweep (dev tool): one short bench line per setting
set -o pipefail
mkdir -p gpurun_out
run() { local L=$1; shift; env "$@" timeout -k 10 200 python3 bench.py --workload highcard --no-cpu --steps 5 --warmup 2 > gpurun_out/hc_$L.json 2> gpurun_out/hc_$L.err || { echo "bench $L failed"; tail -20 gpurun_out/hc_$L.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/hc_$L.json')); b=d['step_breakdown_ms']; print('$L', round(d['ms_per_step'],3), 'ms', 'scan+part', b['scan_ms'], 'fin', b['finalize_wall_ms'])"; }
run base PG_STREAM=1 || exit 1
run st36 PG_STAGE_KB=36 || exit 1
run st36r1 PG_STAGE_KB=36 PG_STAGE_RING=1 || exit 1
run st36r1b8 PG_STAGE_KB=36 PG_STAGE_RING=1 PG_SCAN_BLOCKS_PER_CU=8 || exit 1
run r1 PG_STAGE_RING=1 || exit 1
