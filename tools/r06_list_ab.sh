#!/bin/bash
# config 2 list scan: the block-table flush ablation (PG_LIST_FLUSH_SKIP variant) and the list grid size
set -o pipefail
mkdir -p gpurun_out
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --workload adanalytics --no-cpu --steps 30 --warmup 5 --inflight 1 --no-full-parity \
    > gpurun_out/la_$n.json 2> gpurun_out/la_$n.err || { echo "bench $n failed"; tail -20 gpurun_out/la_$n.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['step_breakdown_ms']['prefilter_ms'], d['step_breakdown_ms']['scan_ms'])" gpurun_out/la_$n.json $n
}
run base X=1
run noflush PINOT_GPU_LIB=pinot_amd/libpinot_gpu_noflush.so
for b in 128 192 256 384; do run lb$b PG_LIST_BLOCKS=$b; run nf_lb$b PG_LIST_BLOCKS=$b PINOT_GPU_LIB=pinot_amd/libpinot_gpu_noflush.so; done
