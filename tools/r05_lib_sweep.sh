#!/bin/bash
# config-4 bench per variant library (tools/variant.sh pg_part builds): names ... ("base" = the main library)
set -o pipefail
mkdir -p gpurun_out
for n in "$@"; do
  L=$PWD/pinot_amd/libpinot_gpu_$n.so; [ "$n" = base ] && L=$PWD/pinot_amd/libpinot_gpu.so
  PINOT_GPU_LIB=$L timeout -k 10 300 python3 bench.py --workload ${WL:-highcard} --no-cpu --no-full-parity --steps 5 --warmup 2 > gpurun_out/ls_$n.json 2> gpurun_out/ls_$n.err || { echo "variant $n failed"; tail -5 gpurun_out/ls_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ls_$n.json')); print('$n', round(d['ms_per_step'],3), d['step_breakdown_ms']['scan_ms'])"
done
